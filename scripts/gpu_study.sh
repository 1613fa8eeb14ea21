#!/bin/bash
# one-off GPU studies (round 3): A/B (ablate.py, production library) and the sharded-step study.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-study}; mkdir -p $OUT
if [ -n "${ABL:-}" ]; then
  timeout -k 10 300 python scripts/ablate.py $ABL > $OUT/ablate.log 2>&1
  rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids $OUT/ablate.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${SHARD:-}" ]; then
  timeout -k 10 400 python scripts/study/shard_step.py $SHARD > $OUT/shard_step.log 2>&1
  rc=$?; echo "shard_step rc=$rc"; grep -v amdgpu.ids $OUT/shard_step.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
