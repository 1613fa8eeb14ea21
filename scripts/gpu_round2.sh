#!/bin/bash
# Round-2 measurement pass: GPU parity suite, the bench line (CPU baseline, attainable copy/fill), the
# config table (C3, C4, C5, 8(f) rows, block operators), the literal C5 256^3 streamed run, rocprofv3
# kernel stats of the bench.  Each GPU step time-limited; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${1:-r02c}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_c4.log" 2>&1
rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_configs.py c3 c4 c5 f ops > "$OUT/configs.log" 2>&1
rc=$?; echo "configs rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_configs.py c5s > "$OUT/c5s.log" 2>&1
rc=$?; echo "c5s rc=$rc"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
rc=$?; echo "rocprof bench rc=$rc"; exit $rc
