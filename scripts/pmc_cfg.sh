#!/bin/bash
# Kernel-trace stats + PMC passes for one scripts/bench_configs.py configuration (c3 / c4 / c5 ...):
# each counter group in its own rocprofv3 run (kernel-trace only); stops at the first fault / timeout.
# usage: scripts/pmc_cfg.sh TAG CONFIG [bench_configs args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=$1; CFG=$2; shift 2
ARGS="$CFG --steps 5 --warmup 1 $*"
export TMPDIR=/tmp
cd /tmp
mkdir -p "$OUT/pmc_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pmc_$TAG/stats" -o run --output-format csv -- \
  python3 "$ROOT/scripts/bench_configs.py" $ARGS > "$OUT/pmc_$TAG/stats.log" 2>&1
rc=$?
echo "stats rc=$rc"
[ $rc -eq 0 ] || exit $rc
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc -d "$OUT/pmc_$TAG/p$i" -o run --output-format csv -- \
    python3 "$ROOT/scripts/bench_configs.py" $ARGS > "$OUT/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($pmc) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
