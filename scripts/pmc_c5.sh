#!/bin/bash
# C5 (hex Q3, MFMA) profile: kernel-trace stats + PMC passes (each in its own rocprofv3 run, kernel-trace only).
# Stops at the first fault / abort / timeout; an unknown counter (ordinary error) only skips that pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-c5}
N=${2:-32}
export TMPDIR=/tmp
cd /tmp
mkdir -p "$OUT/pmc_$TAG"
rocprofv3 -L > "$OUT/pmc_$TAG/counters.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pmc_$TAG/stats" -o run --output-format csv -- \
  python3 "$ROOT/scripts/bench_configs.py" c5 --n "$N" --steps 5 --warmup 1 > "$OUT/pmc_$TAG/stats.log" 2>&1
rc=$?
echo "stats rc=$rc"
case $rc in 0|1|2) ;; *) exit $rc ;; esac
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc -d "$OUT/pmc_$TAG/p$i" -o run --output-format csv -- \
    python3 "$ROOT/scripts/bench_configs.py" c5 --n "$N" --steps 3 --warmup 1 > "$OUT/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($pmc) rc=$rc"
  case $rc in 0|1|2) ;; *) exit $rc ;; esac
done
