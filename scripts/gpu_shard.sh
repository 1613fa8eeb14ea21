#!/bin/bash
# sharded-step pass: the sharded GPU tests, then the one-card step study (scripts/study/shard_step.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-shard}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sharded.py tests/test_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in ${SHARD:-"c4 8" "c2 2 8"}; do
  timeout -k 10 400 python scripts/study/shard_step.py $w > $OUT/shard_step_${w// /_}.log 2>&1
  rc=$?; echo "shard_step $w rc=$rc"; grep -v amdgpu.ids $OUT/shard_step_${w// /_}.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
