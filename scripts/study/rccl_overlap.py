"""Does an RCCL transfer run BESIDE the persistent assembly kernel on one card?  (the sharded
step overlaps its halo exchange with the full-range assembly, which only pays if the RCCL kernel finds CU
resources while the persistent tiles hold the LDS -- C4's Q1 tiles take all 160 KB of a CU.)

A one-rank RCCL communicator sends a halo-sized message (C4 N=8 middle rank: 2400 doubles; C2: 1280) to itself
on its transfer stream, the same group send/recv the N-GPU step posts:
  (a) the assembly alone, (r) the exchange alone (post + stream wait),
  (o) exchange posted first, then the assembly on the main stream, joined -- if the RCCL kernel co-resides, (o)
      ~ (a); if it waits for the tiles to drain, (o) ~ (a) + (r),
  (s) serial: exchange, then the assembly.
usage: python scripts/study/rccl_overlap.py [c2|c4] ..."""
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
    comm = H.Comm.rccl(H.Comm.rccl_unique_id(), 1, 0, 0)
    for wl in sys.argv[1:] or ["c4", "c2"]:
        et, nx, ny, p, nmsg = (H.CUBE, 3520, 1200, 8, 2400) if wl == "c4" else (H.SIMPLEX, 3200, 640, 1, 1280)
        grid = H.Grid.structured(et, nx, ny, (0, 0), (5, 1), px=p, py=p)
        loc = grid.local()
        perm = 10.0 ** np.random.default_rng(10).uniform(-3, 3, 2000)
        k = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
        dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
        ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
        kap = [H.scalar_fn(H.FN_CONST, 1.0)]
        vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
        a = torch.arange(nmsg, dtype=torch.float64, device="cuda")
        b = torch.empty_like(a)

        def asm():
            H.assemble(ctx, dm, dp, kap, ten, vals=vals)

        def xchg():
            comm.post([0], [a], [b])
            comm.wait()

        def overlap():
            comm.post([0], [a], [b])
            asm()
            comm.wait()

        def serial():
            xchg()
            asm()

        res = {"a assembly alone": timeit(asm), "r exchange alone": timeit(xchg),
               "o exchange beside the assembly": timeit(overlap), "s exchange, then assembly": timeit(serial)}
        base = res["a assembly alone"][0]
        print("%s: %d elements, message %d doubles" % (wl, loc.n_own, nmsg))
        for name, (med, mn) in res.items():
            print("  %-34s median %.4f ms  min %.4f ms  (%+.1f %% of a)" % (name, med, mn, 100 * (med / base - 1)),
                  flush=True)
        assert torch.equal(a, b)
        del dm, dp, vals
    del comm


if __name__ == "__main__":
    main()
