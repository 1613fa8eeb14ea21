#!/bin/bash
# Round-4 final pass after the P1 split-tile default: sharded / device-transport tests first, the one-card step
# studies (C2 / C4 at N = 8), then the full measurement pass (scripts/gpu_r04_final.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_sharded.py tests/test_device_transport.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "shard tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/study/shard_step.py c2 8 > $OUT/shard_step_c2.log 2>&1
rc=$?; echo "shard_step c2 rc=$rc"; grep -E "N=|NO_HALO|b step|b' |e split|c serial" $OUT/shard_step_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/study/shard_step.py c4 8 > $OUT/shard_step_c4.log 2>&1
rc=$?; echo "shard_step c4 rc=$rc"; grep -E "N=|NO_HALO|b step|b''' " $OUT/shard_step_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/study/device_step.py c2 8 > $OUT/device_step_c2.log 2>&1
rc=$?; echo "device_step c2 rc=$rc"; grep -v amdgpu.ids $OUT/device_step_c2.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_final.sh r04
