#!/bin/bash
# A/B of the step's intra-device event scope (device-scope ev_in / ev_out, default) against system-scope events
# (HDD_EVENT_SYSTEM_FENCE=1): sharded tests, back-to-back kernel traces, one-card step study, device transport.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_sharded.py \
  tests/test_device_transport.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for mode in dev sys; do
  if [ $mode = sys ]; then export HDD_EVENT_SYSTEM_FENCE=1; else unset HDD_EVENT_SYSTEM_FENCE; fi
  for cfg in "c4 8 4" "c4 8 0" "c2 8 0" "c2 8 4"; do
    tag=${mode}_$(echo $cfg | tr ' ' '_')
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$tag" -o run --output-format csv -- \
       python3 "$ROOT/scripts/study/step_timeline.py" $cfg 40 0 --btb > "$OUT/$tag.log" 2>&1)
    rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 scripts/study/step_timeline.py --summary "$OUT/$tag/run_kernel_trace.csv" > "$OUT/${tag}_btb.txt" 2>&1
    head -1 "$OUT/${tag}_btb.txt"
  done
done
for rep in 1 2; do
  for mode in dev sys; do
    if [ $mode = sys ]; then export HDD_EVENT_SYSTEM_FENCE=1; else unset HDD_EVENT_SYSTEM_FENCE; fi
    for w in c4 c2; do
      timeout -k 10 300 python3 scripts/study/shard_step.py $w 8 > $OUT/shard_${w}_${mode}_$rep.log 2>&1
      rc=$?; echo "shard $w $mode $rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
      grep -E "rank|a NO_HALO|b step|b''' |b'''' " $OUT/shard_${w}_${mode}_$rep.log
    done
  done
done
for mode in dev sys; do
  if [ $mode = sys ]; then export HDD_EVENT_SYSTEM_FENCE=1; else unset HDD_EVENT_SYSTEM_FENCE; fi
  timeout -k 10 300 python3 scripts/study/device_step.py c4 8 > $OUT/device_c4_$mode.log 2>&1
  rc=$?; echo "device c4 $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -v Warn $OUT/device_c4_$mode.log | head -4
done
