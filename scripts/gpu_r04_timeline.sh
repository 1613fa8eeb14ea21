#!/bin/bash
# Kernel timelines of the sharded step (scripts/study/step_timeline.py under rocprofv3 --kernel-trace).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04m; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "c4 8 0" "c4 8 4" "c2 8 0" "c2 8 4"; do
  tag=$(echo $cfg | tr ' ' '_')
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$tag" -o run --output-format csv -- \
     python3 "$ROOT/scripts/study/step_timeline.py" $cfg 20 > "$OUT/$tag.log" 2>&1)
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/study/step_timeline.py --summary "$OUT/$tag/run_kernel_trace.csv" > "$OUT/${tag}_timeline.txt" 2>&1
  tail -12 "$OUT/${tag}_timeline.txt"
done
