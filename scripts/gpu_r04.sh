#!/bin/bash
# Round-4 pass: focused GPU tests (given files), the Q1 / sharded GPU tests under HDD_DEBUG_FLAGS (the half-image
# kernel selected by the context), the whole GPU suite, smoke, then a same-box A/B of the C4 bench line.
# Each GPU step time-limited; stops at the first failure.
# usage: [NOSUITE=1] [ABREPS=3] [ABFLAG=1048576] gpu_r04.sh TAG [test files...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
PYT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread"
if [ $# -gt 0 ]; then
  timeout -k 10 600 $PYT -v "$@" > $OUT/pytest_focus.log 2>&1
  rc=$?; echo "focus rc=$rc"; tail -3 $OUT/pytest_focus.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ABFLAG:-}" ]; then
  HDD_DEBUG_FLAGS=$ABFLAG timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_sharded.py tests/test_device_transport.py \
    tests/test_gpu_known_answer.py tests/test_gpu_expectations.py > $OUT/pytest_flag.log 2>&1
  rc=$?; echo "flag suite rc=$rc"; tail -2 $OUT/pytest_flag.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NOSUITE:-}" ]; then
  timeout -k 10 900 $PYT tests > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ABFLAG:-}" ]; then
  bash scripts/ab_envs.sh $TAG c4 ${ABREPS:-3} HDD_DEBUG_FLAGS 0 $ABFLAG
fi
