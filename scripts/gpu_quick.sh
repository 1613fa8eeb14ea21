#!/bin/bash
# Quick GPU iteration: parity tests, the bench line, C3/C4 configs (each step time-limited, stop at first failure).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; TAG=${1:-q}; shift || true
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench_$TAG.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_configs.py c3 c4 --samples 16 "$@" > $OUT/cfg_$TAG.log 2>&1
rc=$?; echo "cfg rc=$rc"; grep config $OUT/cfg_$TAG.log; exit $rc
