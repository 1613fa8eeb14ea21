#!/bin/bash
# Same-box A/B of an HDD_DEBUG_FLAGS bit on scripts/bench_configs.py rows (default path vs flag), after the
# named GPU test files; then a rocprofv3 kernel-stats pass of the rows on the default path.
# usage: ab_cfg_flags.sh FLAGS TAG "cfgs" "test files" [reps]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); FL=$1; TAG=$2; CFG=$3; TESTS=$4; REPS=${5:-3}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in $(seq 1 $REPS); do
  for v in default flag$FL; do
    if [ $v = default ]; then F=0; else F=$FL; fi
    HDD_DEBUG_FLAGS=$F timeout -k 10 300 python -u scripts/bench_configs.py $CFG --steps 50 --warmup 10 > $OUT/${v}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "configs $v rc=$rc"; tail -5 $OUT/${v}_$rep.log; exit $rc; }
    echo "$v $(grep -o '"[a-z_0-9]*_ms": [0-9.]*' $OUT/${v}_$rep.log | tr '\n' ' ')"
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 "$ROOT/scripts/bench_configs.py" $CFG --steps 20 --warmup 5 > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
