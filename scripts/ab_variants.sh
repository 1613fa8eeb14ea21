#!/bin/bash
# Same-box A/B of library builds x HDD_DEBUG_FLAGS values on the bench line(s), alternating, after the GPU
# parity suite on the in-tree build.  usage: ab_variants.sh TAG "c2 c4" REPS LIB:FLAGS [LIB:FLAGS ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; WL=$2; REPS=$3; shift 3; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in $(seq 1 $REPS); do
  for w in $WL; do
    for v in "$@"; do
      L=${v%%:*}; F=${v##*:}; n=$(basename $L .so)_f$F
      HDD_AMD_LIB=$PWD/$L HDD_DEBUG_FLAGS=$F timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${w}_${n}_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $w $n rc=$rc"; tail -5 $OUT/${w}_${n}_$rep.log; exit $rc; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], '%.4f ms/step' % d['ms_per_step'], 'kernel %.4f ms' % r['kernel_ms_avg'], round(r['frac'], 4))" $OUT/${w}_${n}_$rep.log $w $n
    done
  done
done
