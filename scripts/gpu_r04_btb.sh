#!/bin/bash
# Back-to-back sharded steps under rocprofv3 --kernel-trace (scripts/study/step_timeline.py --btb): the period of
# the persistent launches and the gap between them, default schedule vs one launch (NO_HALO), serial, launch last.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04q; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "c4 8 4" "c4 8 0" "c2 8 4" "c2 8 0"; do
  for fl in 0 4 1 256; do
    tag=$(echo $cfg | tr ' ' '_')_f$fl
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$tag" -o run --output-format csv -- \
       python3 "$ROOT/scripts/study/step_timeline.py" $cfg 40 $fl --btb > "$OUT/$tag.log" 2>&1)
    rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 scripts/study/step_timeline.py --summary "$OUT/$tag/run_kernel_trace.csv" > "$OUT/${tag}_btb.txt" 2>&1
    head -1 "$OUT/${tag}_btb.txt"
  done
done
