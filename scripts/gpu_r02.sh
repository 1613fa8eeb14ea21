#!/bin/bash
# Round-2 GPU pass: the sharded-path tests first, then the whole GPU suite, the bench line, a 2-rank
# rehearsal of the N>1 bench path on the one card (gloo host-staged halo through the C++ step).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r02a}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_sharded.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sharded.log 2>&1
rc=$?; echo "sharded rc=$rc"; tail -3 $OUT/pytest_sharded.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo > $OUT/bench_gloo2.log 2>&1
rc=$?; echo "bench gloo2 rc=$rc"; grep metric $OUT/bench_gloo2.log | cut -c1-600; exit $rc
