#!/bin/bash
# Same-box comparison of several values of one environment switch on a bench line, alternating.
# usage: ab_envs.sh tag workload reps VAR val1 val2 ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; W=$2; REPS=$3; VAR=$4; shift 4; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python bench.py --workload $W --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${W}_${v}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $W $v rc=$rc"; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], 'kernel %.4f ms' % r['kernel_ms_avg'], round(r['frac'], 4))" $OUT/${W}_${v}_$rep.log $W $VAR=$v
  done
done
