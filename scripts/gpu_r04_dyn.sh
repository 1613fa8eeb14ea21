#!/bin/bash
# Dynamic tail of the sharded SKIP launch (study bits: 134217728 dynamic tail, 16777216 half-image kernel on the
# SKIP launch): parity tests, then the one-card step study per variant (alternating), and all ranks over the
# device transport (bitwise check of the whole N = 8 decomposition).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04t; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_device_transport.py \
  tests/test_sharded.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in 0 150994944 134217728 16777216; do
    HDD_DEBUG_FLAGS=$f timeout -k 10 300 python3 scripts/study/shard_step.py c4 8 > $OUT/shard_c4_f${f}_$rep.log 2>&1
    rc=$?; echo "shard c4 f=$f $rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep -E "rank|a NO_HALO|b''' " $OUT/shard_c4_f${f}_$rep.log | cut -c1-90
  done
done
for f in 0 134217728; do
  HDD_DEBUG_FLAGS=$f timeout -k 10 300 python3 scripts/study/shard_step.py c2 8 > $OUT/shard_c2_f${f}.log 2>&1
  rc=$?; echo "shard c2 f=$f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -E "rank|a NO_HALO|b step|b''' " $OUT/shard_c2_f${f}.log | cut -c1-90
done
for f in 0 150994944; do
  HDD_DEBUG_FLAGS=$f timeout -k 10 300 python3 scripts/study/device_step.py c4 8 > $OUT/device_c4_f$f.log 2>&1
  rc=$?; echo "device c4 f=$f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -v Warn $OUT/device_c4_f$f.log | head -4
done
