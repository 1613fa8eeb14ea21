#!/bin/bash
# GPU test pass: the given test files first (verbose, stop at the first failure), then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_focus.log 2>&1
  rc=$?; echo "focus rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_focus.log | tail -25; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; exit $rc
