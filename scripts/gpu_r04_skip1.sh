#!/bin/bash
# Single-interval fast path of the SKIP launch's contiguous-image store test: parity tests on the in-tree build,
# then the one-card step study, alternating the committed build (lib_old) and this one.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04x; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_device_transport.py \
  tests/test_sharded.py tests/test_gpu_q1_half.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for L in lib_old lib; do
    HDD_AMD_LIB=$PWD/dune-hdd_amd/$L/libhdd_amd.so timeout -k 10 300 python3 scripts/study/shard_step.py c4 8 > $OUT/shard_c4_${L}_$rep.log 2>&1
    rc=$?; echo "$L $rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep -E "rank|a NO_HALO|b step" $OUT/shard_c4_${L}_$rep.log | cut -c1-90
  done
done
