#!/bin/bash
# PMC passes for the hot kernel (each counter group in its own rocprofv3 run, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r01}
shift || true
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline $*"
export TMPDIR=/tmp
cd /tmp
mkdir -p "$OUT/pmc_$TAG"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc -d "$OUT/pmc_$TAG/p$i" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $BENCH_ARGS > "$OUT/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($pmc) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
