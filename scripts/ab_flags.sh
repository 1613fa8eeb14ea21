#!/bin/bash
# Same-box A/B of an HDD_DEBUG_FLAGS bit (read once per context): GPU parity suite on the default build,
# then alternating bench lines with the flag off (default path) and on.  usage: ab_flags.sh FLAGS tag "c2 c4" [reps]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
FL=$1; TAG=${2:-ab}; WL=${3:-"c2 c4"}; REPS=${4:-3}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in $(seq 1 $REPS); do
  for w in $WL; do
    for v in default flag$FL; do
      if [ $v = default ]; then F=0; else F=$FL; fi
      HDD_DEBUG_FLAGS=$F timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${w}_${v}_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $w $v rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], '%.4f ms/step' % d['ms_per_step'], 'kernel %.4f ms' % r['kernel_ms_avg'], round(r['frac'], 4))" $OUT/${w}_${v}_$rep.log $w $v
    done
  done
done
