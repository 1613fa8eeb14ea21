#!/bin/bash
# bench.py's N > 1 path rehearsed on one card (gloo host transport, 2 ranks C2 / 3 ranks C4) and the N = 1 line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04u; mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo > $OUT/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 $OUT/bench_gloo2.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 3 --workload c4 --steps 10 --warmup 3 --backend gloo > $OUT/bench_c4_gloo3.log 2>&1
rc=$?; echo "gloo3 c4 rc=$rc"; tail -1 $OUT/bench_c4_gloo3.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench1.log 2>&1
rc=$?; echo "bench1 rc=$rc"; tail -1 $OUT/bench1.log | cut -c1-300; exit $rc
