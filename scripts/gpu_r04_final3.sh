#!/bin/bash
# Round-4 final pass after the launch-first default: sharded / device-transport tests, one-card step studies and
# kernel timelines (N = 8), then the full measurement pass (scripts/gpu_r04_final.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04o; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_device_transport.py tests/test_sharded.py tests/test_gpu_q1_half.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for w in c4 c2; do
  timeout -k 10 400 python -u scripts/study/shard_step.py $w 8 > $OUT/shard_step_$w.log 2>&1
  rc=$?; echo "shard_step $w rc=$rc"; grep -E "N=|NO_HALO|b step|b''' |b'''' |e split" $OUT/shard_step_$w.log; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
for cfg in "c4 8 0" "c4 8 4" "c2 8 4"; do
  tag=$(echo $cfg | tr ' ' '_')
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$tag" -o run --output-format csv -- \
     python3 "$ROOT/scripts/study/step_timeline.py" $cfg 20 > "$OUT/$tag.log" 2>&1)
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/study/step_timeline.py --summary "$OUT/$tag/run_kernel_trace.csv" > "$OUT/${tag}_timeline.txt" 2>&1
  tail -7 "$OUT/${tag}_timeline.txt"
done
for w in c4 c2; do
  timeout -k 10 400 python -u scripts/study/device_step.py $w 8 > $OUT/device_step_$w.log 2>&1
  rc=$?; echo "device_step $w rc=$rc"; grep -v amdgpu.ids $OUT/device_step_$w.log; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_r04_final.sh r04
