"""GPU-side cost of the sharded C2 step on one card (what the N-GPU bench adds per rank on top
of the assembly): rank r of an N-strip C2 weak-scaling decomposition (bench.py's layout: (3200 N) x 640 Kuhn
squares), timed as
  (a) NO_HALO       -- the whole owned range in one launch (ghost columns valid): the N = 1 step,
  (b) step          -- pack, loopback copy instead of the transfer (HDD_SHARD_NO_TRANSFER), interior tiles,
                       unpack, halo-boundary tiles: every launch of the real step, RCCL excluded,
  (c) serial step   -- the same without the overlap split (one launch of all tiles after the unpack).
usage: python scripts/study/shard_step.py [N ...]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch
import hdd_amd as H


def timeit(fn, reps=50, rounds=4):
    out = []
    for _ in range(rounds):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return float(np.median(out)), float(np.min(out))


def main():
    ctx = H.Context(0)
    for n in [int(a) for a in sys.argv[1:]] or [2, 8]:
        grid = H.Grid.structured(H.SIMPLEX, 3200 * n, 640, (0.0, 0.0), (5.0 * n, 1.0), px=n, py=1)
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=100 * n * 20)
        for rank in sorted({0, n // 2}):
            sh = H.Shard(ctx, grid, n, rank)
            k = torch.from_numpy(sh.checkerboard((0.0, 0.0), (5.0 * n, 1.0), 100 * n, 20, perm)).cuda()
            _, _, _, pat = sh.pattern(ctx, 0)
            vals = [torch.empty(sh.info.nnz, dtype=torch.float64, device="cuda")]
            kap = [H.scalar_fn(H.FN_CONST, 1.0)]
            ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
            runs = {
                "a NO_HALO (one launch)": H.SHARD_NO_HALO,
                "b step, no transfer": H.SHARD_NO_TRANSFER,
                "c serial step, no transfer": H.SHARD_NO_TRANSFER | H.SHARD_NO_OVERLAP,
            }
            res = {name: timeit(lambda f=f: H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=f))
                   for name, f in runs.items()}
            i = sh.info
            print("N=%d rank %d: %d owned, %d ghosts, tiles %d interior + %d boundary, halo %d/%d elements"
                  % (n, rank, sh.n_own, i.n_ghost, i.n_tiles_interior, i.n_tiles_boundary, i.halo_send, i.halo_recv))
            base = res["a NO_HALO (one launch)"][0]
            for name, (med, mn) in res.items():
                print("  %-28s median %.4f ms  min %.4f ms  (%+.1f %%)" % (name, med, mn, 100 * (med / base - 1)),
                      flush=True)
            del sh


if __name__ == "__main__":
    main()
