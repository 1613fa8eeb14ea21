"""GPU-side cost of the sharded step on one card (what the N-GPU bench adds per rank on top of
the assembly), for rank r of an N-rank decomposition of
  c2  bench.py's weak-scaling layout: (3200 N) x 640 Kuhn squares, one strip per rank;
  c4  BASELINE's 8-GPU config: 3520 x 1200 Q1 quads, 8 x 8 subdomains, column strips of subdomains (strong
      scaling: N = 8 gives each rank 440 x 1200 elements),
timed as
  (a) NO_HALO       -- the whole owned range in one launch (ghost columns valid): the kernel alone,
  (b) step          -- pack, loopback copy instead of the transfer (HDD_SHARD_NO_TRANSFER), unpack and the
                       ghost-adjacent elements in place on the side stream, every other row block on the main
                       stream, join: every launch of the real step, RCCL excluded,
  (b') the same with the fixup after the join on the main stream (HDD_SHARD_FIX_INLINE, round 2),
  (b'') the fixup into a side buffer, every tile, join, one copy kernel (HDD_SHARD_FIX_SCATTER),
  (c) serial step   -- the same without the overlap (one launch of all tiles after the unpack),
  (d) step, graph   -- (b) captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed,
  (e) split tiles   -- round 2's overlap (HDD_SHARD_SPLIT_TILES): interior tiles, unpack, boundary tiles.
usage: python scripts/study/shard_step.py [c2|c4] [N ...]"""
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


def layout(workload, n):
    if workload == "c4":
        grid = H.Grid.structured(H.CUBE, 3520, 1200, (0.0, 0.0), (5.0, 1.0), px=8, py=8)
        return grid, (0.0, 0.0), (5.0, 1.0), 100, 20, 2000
    grid = H.Grid.structured(H.SIMPLEX, 3200 * n, 640, (0.0, 0.0), (5.0 * n, 1.0), px=n, py=1)
    return grid, (0.0, 0.0), (5.0 * n, 1.0), 100 * n, 20, 2000 * n


def main():
    args = sys.argv[1:]
    workload = args.pop(0) if args and args[0] in ("c2", "c4") else "c2"
    ctx = H.Context(0)
    for n in [int(a) for a in args] or [2, 8]:
        grid, lo, up, ncx, ncy, ncell = layout(workload, n)
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=ncell)
        for rank in sorted({0, n // 2}):
            sh = H.Shard(ctx, grid, n, rank)
            k = torch.from_numpy(sh.checkerboard(lo, up, ncx, ncy, perm)).cuda()
            _, _, _, pat = sh.pattern(ctx, 0)
            vals = [torch.empty(sh.info.nnz, dtype=torch.float64, device="cuda")]
            kap = [H.scalar_fn(H.FN_CONST, 1.0)]
            ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
            runs = {
                "a NO_HALO (one launch)": H.SHARD_NO_HALO,
                "b step, no transfer": H.SHARD_NO_TRANSFER,
                "b' step, fixup inline (round 2)": H.SHARD_NO_TRANSFER | H.SHARD_FIX_INLINE,
                "b'' step, fixup + copy kernel": H.SHARD_NO_TRANSFER | H.SHARD_FIX_SCATTER,
                "b''' step, fixup in place": H.SHARD_NO_TRANSFER | H.SHARD_FIX_INPLACE,
                "b'''' step, launch after halo work (r3)": H.SHARD_NO_TRANSFER | H.SHARD_LAUNCH_LAST,
                "c serial step, no transfer": H.SHARD_NO_TRANSFER | H.SHARD_NO_OVERLAP,
                "e split tiles, no transfer": H.SHARD_NO_TRANSFER | H.SHARD_SPLIT_TILES,
            }
            res = {name: timeit(lambda f=f: H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=f))
                   for name, f in runs.items()}
            # (d) the step captured into a graph (side stream: capture needs a non-default stream)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(3):
                    H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=H.SHARD_NO_TRANSFER,
                                       stream=s.cuda_stream)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, stream=s):
                    H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=H.SHARD_NO_TRANSFER,
                                       stream=s.cuda_stream)
                res["d step, no transfer, hipGraph"] = timeit(g.replay)
            except Exception as e:   # report, keep the other numbers
                print("  graph capture failed: %s" % e)
            # (f) the element-list fixup alone, (g) one full launch, on the same rank-local layout through the
            # Python front-end's LocalMesh (grid.local(s0, s1) = the shard's element range)
            s0, s1 = sh.info.s_begin, sh.info.s_end
            loc = grid.local(s0, s1)
            dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
            kl = torch.from_numpy(loc.checkerboard(lo, up, ncx, ncy, perm)).cuda()
            tl = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=kl)
            vl = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
            fix = torch.from_numpy(H.halo_elements(loc)).cuda()
            res["f fixup launch alone"] = timeit(lambda: H.assemble_tiles(ctx, dm, dp, kap, tl, fix, vl, elements=True))
            res["g full launch (LocalMesh)"] = timeit(lambda: H.assemble(ctx, dm, dp, kap, tl, vals=vl))
            del dm, dp, loc
            i = sh.info
            print("%s N=%d rank %d: %d owned, %d ghosts, tiles %d interior + %d boundary, %d ghost-adjacent "
                  "elements, halo %d/%d elements"
                  % (workload, n, rank, sh.n_own, i.n_ghost, i.n_tiles_interior, i.n_tiles_boundary, i.halo_elements,
                     i.halo_send, i.halo_recv))
            base = res["a NO_HALO (one launch)"][0]
            for name, (med, mn) in res.items():
                print("  %-32s median %.4f ms  min %.4f ms  (%+.1f %%)" % (name, med, mn, 100 * (med / base - 1)),
                      flush=True)
            del sh


if __name__ == "__main__":
    main()
