#!/bin/bash
# Round-3 counter pass on the final build: PMC groups for C3 (P1 smooth, fused) and C4 (Q1) through
# scripts/pmc_cfg.sh, then a 2-rank gloo rehearsal of bench.py's N>1 path (sharded step, host transport) and a
# 3-rank one with --workload c4 (a middle rank with two peers).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03pmc}; mkdir -p $OUT
bash scripts/pmc_cfg.sh c3_r03 c3 || exit $?
bash scripts/pmc_cfg.sh c4_r03 c4 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo > $OUT/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 $OUT/bench_gloo2.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 3 --workload c4 --steps 10 --warmup 3 --backend gloo > $OUT/bench_c4_gloo3.log 2>&1
rc=$?; echo "gloo3 c4 rc=$rc"; tail -1 $OUT/bench_c4_gloo3.log | cut -c1-400; exit $rc
