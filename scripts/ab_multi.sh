#!/bin/bash
# Same-box A/B/C... of several HDD_DEBUG_FLAGS values on the bench lines, alternating.
# usage: ab_multi.sh tag "c2 c4" reps flagA flagB ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; WL=$2; REPS=$3; shift 3; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for w in $WL; do
    for F in "$@"; do
      HDD_DEBUG_FLAGS=$F timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${w}_f${F}_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $w $F rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'flags', sys.argv[3], 'kernel %.4f ms' % r['kernel_ms_avg'], round(r['frac'], 4))" $OUT/${w}_f${F}_$rep.log $w $F
    done
  done
done
