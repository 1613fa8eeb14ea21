#!/bin/bash
# One GPU session: parity tests, a bench line, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / timeout (anything but pytest's 0/1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$TAG.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -2 "$OUT/bench_$TAG.log"
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench_$TAG.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
exit $rc
