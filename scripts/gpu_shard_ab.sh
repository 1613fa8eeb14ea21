#!/bin/bash
# Sharded-step study on one card under several HDD_DEBUG_FLAGS settings (scripts/study/shard_step.py, loopback
# transfer; scripts/study/device_step.py, all ranks as thread ranks over the device transport).
# usage: gpu_shard_ab.sh TAG WORKLOAD "N..." FLAGS...      e.g. gpu_shard_ab.sh r04c c4 "2 8" 0 4194304 1048576
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; W=$2; NS=$3; shift 3; OUT=gpurun_out/$TAG; mkdir -p $OUT
for F in "$@"; do
  HDD_DEBUG_FLAGS=$F timeout -k 10 400 python -u scripts/study/shard_step.py $W $NS > $OUT/shard_step_${W}_f$F.log 2>&1
  rc=$?; echo "shard_step $W flags=$F rc=$rc"; grep -E "N=|NO_HALO|b step|b''' |f fixup|g full" $OUT/shard_step_${W}_f$F.log
  [ $rc -eq 0 ] || exit $rc
done
for F in "$@"; do
  HDD_DEBUG_FLAGS=$F timeout -k 10 400 python -u scripts/study/device_step.py $W $NS > $OUT/device_step_${W}_f$F.log 2>&1
  rc=$?; echo "device_step $W flags=$F rc=$rc"; cat $OUT/device_step_${W}_f$F.log | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
done
