#!/bin/bash
# Extra evidence on the final build: C3 wave-cycle accounting (scripts/pmc_cfg.sh) and a 300-launch kernel trace
# of the C2 bench command (the power-management transient vs the steady state).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r04l; mkdir -p $OUT
bash scripts/pmc_cfg.sh r04_c3 c3 --samples 8 > $OUT/pmc_c3.log 2>&1
rc=$?; echo "pmc c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc_r04_c3 swipdg_persistent > $OUT/pmc_c3_summary.md 2>&1
grep -A12 "wave-cycle" $OUT/pmc_c3_summary.md
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/long" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/long.log" 2>&1
rc=$?; echo "long trace rc=$rc"; exit $rc
