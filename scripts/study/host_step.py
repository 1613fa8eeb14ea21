"""Is the sharded step host-bound?  Host enqueue time per step (perf_counter around `reps` calls of
hdd_block_assemble_sharded without synchronisation) against the GPU time per step (the same calls bracketed by
synchronisations), for rank r of an N-rank C4 / C2 decomposition with the loopback transfer, per schedule; plus
the ctypes front-end alone (argument marshalling, no call) and the C entry point called with pre-marshalled
arguments.
usage: python scripts/study/host_step.py c4 8 4"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch  # noqa: E402
import hdd_amd as H  # noqa: E402


def main():
    wl, n, rank = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    if wl == "c4":
        grid = H.Grid.structured(H.CUBE, 3520, 1200, (0.0, 0.0), (5.0, 1.0), px=8, py=8)
        up, ncx, ncell = (5.0, 1.0), 100, 2000
    else:
        grid = H.Grid.structured(H.SIMPLEX, 3200 * n, 640, (0.0, 0.0), (5.0 * n, 1.0), px=n, py=1)
        up, ncx, ncell = (5.0 * n, 1.0), 100 * n, 2000 * n
    perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=ncell)
    ctx = H.Context(0)
    sh = H.Shard(ctx, grid, n, rank)
    k = torch.from_numpy(sh.checkerboard((0.0, 0.0), up, ncx, 20, perm)).cuda()
    _, _, _, pat = sh.pattern(ctx, 0)
    vals = [torch.empty(sh.info.nnz, dtype=torch.float64, device="cuda")]
    kap, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    reps = 200
    rows = {"NO_HALO": H.SHARD_NO_HALO, "default": H.SHARD_NO_TRANSFER,
            "in place": H.SHARD_NO_TRANSFER | H.SHARD_FIX_INPLACE,
            "serial": H.SHARD_NO_TRANSFER | H.SHARD_NO_OVERLAP}
    # pre-marshalled arguments: the C entry point alone
    arr = (H.ScalarFn * 1)(*kap)
    ptrs = (C.c_void_p * 1)(vals[0].data_ptr())
    prm = H.params_for(1, 2)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    fn = H.lib().hdd_block_assemble_sharded
    for name, f in rows.items():
        for _ in range(20):
            H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=f)
        torch.cuda.synchronize()
        res = []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(reps):
                H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=f)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            t3 = time.perf_counter()
            for _ in range(reps):
                fn(ctx.h, sh.h, None, arr, 1, C.byref(ten), C.byref(prm), C.byref(pat), ptrs, f, s)
            t4 = time.perf_counter()
            torch.cuda.synchronize()
            t5 = time.perf_counter()
            res.append(((t1 - t0) / reps * 1e6, (t2 - t0) / reps * 1e6, (t4 - t3) / reps * 1e6, (t5 - t3) / reps * 1e6))
        r = np.median(np.array(res), axis=0)
        print("%s N=%d rank %d %-9s python front-end: enqueue %6.1f us/step, wall %6.1f us/step | C entry: enqueue "
              "%6.1f us/step, wall %6.1f us/step" % (wl, n, rank, name, r[0], r[1], r[2], r[3]), flush=True)
    t0 = time.perf_counter()
    for _ in range(2000):
        H.params_for(1, 2)
        (H.ScalarFn * 1)(*kap)
        (C.c_void_p * 1)(vals[0].data_ptr())
        torch.cuda.current_stream().cuda_stream
    print("front-end marshalling alone: %.1f us per call" % ((time.perf_counter() - t0) / 2000 * 1e6))


if __name__ == "__main__":
    main()
