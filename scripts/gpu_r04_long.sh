#!/bin/bash
# Sustained runs (power-management transient): bench.py C2 / C4 with 400 timed steps after 50 warmup,
# and a kernel trace of a 300-step C2 run for the per-launch durations over time.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 400 --warmup 50 --no-cpu-baseline > $OUT/bench_c2_400.log 2>&1
rc=$?; echo "c2 rc=$rc"; tail -1 $OUT/bench_c2_400.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload c4 --steps 400 --warmup 50 --no-cpu-baseline > $OUT/bench_c4_400.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -1 $OUT/bench_c4_400.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace_c2" -o run --output-format csv -- \
   python3 "$ROOT/bench.py" --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/trace_c2.log" 2>&1)
rc=$?; echo "trace rc=$rc"; exit $rc
