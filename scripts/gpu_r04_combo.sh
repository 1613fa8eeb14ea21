#!/bin/bash
# One GPU call for a busy pool: the new tests, the pair-lane A/B, the Q1 size / XCD-rotation probe, then the
# round-4 measurement pass (scripts/gpu_r04_pass.sh).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04h}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_q1_half.py tests/test_known_two_element.py tests/test_gpu_surface.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_sets.sh $TAG c4 2 - HDD_DEBUG_FLAGS=134217728 HDD_DEBUG_FLAGS=1048576 || exit 1
bash scripts/ab_sets.sh $TAG c2 2 - HDD_DEBUG_FLAGS=67108864 || exit 1
timeout -k 10 300 python -u scripts/study/q1_size_sweep.py --sizes 3520x1200,3520x1190,3504x1200,3536x1200,1760x1200,3520x2400 0 1048576 67108864 68157440 > $OUT/sizes.log 2>&1
rc=$?; echo "sizes rc=$rc"; grep -v amdgpu.ids $OUT/sizes.log; [ $rc -eq 0 ] || exit $rc
CFG="c3 c4 c5 f ops" bash scripts/gpu_r04_pass.sh r04
