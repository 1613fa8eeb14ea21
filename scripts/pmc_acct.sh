#!/bin/bash
# Wave-cycle accounting of one bench workload's kernel: kernel-trace stats, then SQ counter passes (each in its own
# rocprofv3 run, kernel-trace only) whose terms partition SQ_WAVE_CYCLES -- ACTIVE_INST_ANY (+ its VALU / LDS /
# SCA / VMEM / MISC / FLAT parts) + WAIT_ANY (parked at s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) --
# then FETCH_SIZE / WRITE_SIZE.  Environment (HDD_DEBUG_FLAGS ...) passes through to bench.py.
# usage: scripts/pmc_acct.sh TAG [bench.py args...]      (summary: scripts/pmc_summary.py)
#        PMC_SCRIPT=scripts/bench_configs.py scripts/pmc_acct.sh TAG c3 --steps 5   (any script, args as given)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=$1; shift
SCRIPT=${PMC_SCRIPT:-bench.py}
if [ -n "${PMC_SCRIPT:-}" ]; then ARGS="$*"; else ARGS="--steps 5 --warmup 2 --no-cpu-baseline $*"; fi
export TMPDIR=/tmp
cd /tmp
mkdir -p "$OUT/pmc_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pmc_$TAG/stats" -o run --output-format csv -- \
  python3 "$ROOT/$SCRIPT" $ARGS > "$OUT/pmc_$TAG/stats.log" 2>&1
rc=$?
echo "stats rc=$rc"
[ $rc -eq 0 ] || exit $rc
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pmc -d "$OUT/pmc_$TAG/p$i" -o run --output-format csv -- \
    python3 "$ROOT/$SCRIPT" $ARGS > "$OUT/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($pmc) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
