#!/bin/bash
# one-off GPU studies (round 3): write-pattern microbenchmark (WS=1: wstream6), A/B of kernel variants
# (ABL: production library; ABLAB: the HDD_ABLATION build in lib_ab/, `make -C dune-hdd_amd ablation`), the
# sharded-step study (SHARD="c4 2 4 8").  Each GPU step time-limited; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-study}; mkdir -p $OUT
if [ -n "${WS:-}" ]; then
  timeout -k 10 120 ./scripts/microbench/wstream6 > $OUT/wstream6.log 2>&1
  rc=$?; echo "wstream6 rc=$rc"; cat $OUT/wstream6.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ABL:-}" ]; then
  timeout -k 10 300 python scripts/ablate.py $ABL > $OUT/ablate.log 2>&1
  rc=$?; echo "ablate rc=$rc"; grep -v amdgpu.ids $OUT/ablate.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ABLAB:-}" ]; then
  HDD_AMD_LIB=$PWD/dune-hdd_amd/lib_ab/libhdd_abl.so timeout -k 10 300 python scripts/ablate.py $ABLAB > $OUT/ablate_ab.log 2>&1
  rc=$?; echo "ablate_ab rc=$rc"; grep -v amdgpu.ids $OUT/ablate_ab.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${SHARD:-}" ]; then
  timeout -k 10 400 python scripts/study/shard_step.py $SHARD > $OUT/shard_step.log 2>&1
  rc=$?; echo "shard_step rc=$rc"; grep -v amdgpu.ids $OUT/shard_step.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
