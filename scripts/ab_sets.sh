#!/bin/bash
# Same-box comparison of several environment settings on one bench line, alternating.  A setting is a string of
# VAR=value words ("-" = none).  usage: ab_sets.sh tag workload reps "HDD_DEBUG_FLAGS=0" "HDD_DEBUG_FLAGS=1 HDD_P1_WGCU=6" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; W=$2; REPS=$3; shift 3; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  i=0
  for S in "$@"; do
    i=$((i+1))
    [ "$S" = "-" ] && E="" || E="$S"
    env $E timeout -k 10 200 python bench.py --workload $W --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${W}_s${i}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $W [$S] rc=$rc"; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], '[%s]' % sys.argv[3], 'kernel %.4f ms' % r['kernel_ms_avg'], round(r['frac'], 4))" $OUT/${W}_s${i}_$rep.log $W "$S"
  done
done
