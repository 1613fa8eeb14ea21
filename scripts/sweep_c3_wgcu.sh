#!/bin/bash
# C3 (P1SmoothPolicy) workgroups-per-CU sweep after the trig change (HDD_P1_WGCU overrides the policy's WGCU)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/sweep_c3; mkdir -p $OUT
for rep in 1 2; do
  for w in 8 4 6 7 5; do
    HDD_P1_WGCU=$w timeout -k 10 200 python scripts/bench_configs.py c3 --samples 4 > $OUT/w${w}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "wgcu=$w rc=$rc"; exit $rc; }
    echo "wgcu=$w $(grep -o '"assembly_ms": [0-9.]*' $OUT/w${w}_$rep.log)"
  done
done
