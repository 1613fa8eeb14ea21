#!/bin/bash
# Full measurement pass: GPU parity suite, the bench line (with CPU baseline), rocprofv3 kernel stats of
# the bench and of the C3/C4/C5 configurations.  Each GPU step time-limited; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/round_${1:-r01}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_configs.py c3 c4 c5 > "$OUT/bench_configs.log" 2>&1
rc=$?; echo "configs rc=$rc"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_configs" -o run --output-format csv -- \
  python3 "$ROOT/scripts/bench_configs.py" c3 c4 c5 --samples 16 > "$OUT/prof_configs.log" 2>&1
rc=$?; echo "rocprof configs rc=$rc"; exit $rc
