"""Same-box comparison of the C2 assembly through (a) DeviceMesh + hdd_swipdg_assemble (Python-built mesh
arrays, host pattern), (b) the shard + hdd_block_assemble_sharded (the bench path), (c) the shard's mesh
and device pattern through hdd_swipdg_assemble -- to separate the data layout from the entry point."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch
import hdd_amd as H


class _DM:   # a DeviceMesh-like view of the shard's mesh for H.assemble
    def __init__(self, t, loc):
        self.t, self.local, self.coords = t, loc, torch.empty(1, device="cuda")


def main():
    ctx = H.Context(0)
    perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=2000)
    grid = H.Grid.structured(H.SIMPLEX, 3200, 640, (0, 0), (5, 1))
    kap = [H.scalar_fn(H.FN_CONST, 1.0)]
    # (a)
    loc = grid.local()
    ka = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    va = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
    tA = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=ka)
    # (b), (c)
    sh = H.Shard(ctx, grid, 1, 0)
    kb = torch.from_numpy(sh.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
    _, _, _, pat_t = pat = sh.pattern(ctx, 0)
    vb = [torch.empty(sh.info.nnz, dtype=torch.float64, device="cuda")]
    tB = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=kb)
    dpc = type("P", (), {"t": pat_t, "nnz": sh.info.nnz})()
    dmc = _DM(sh.mesh, loc)
    runs = {
        "a DeviceMesh + assemble": lambda: H.assemble(ctx, dm, dp, kap, tA, vals=va),
        "b shard + assemble_sharded": lambda: H.assemble_sharded(ctx, sh, None, kap, tB, pat_t, vb),
        "c shard mesh + assemble": lambda: H.assemble(ctx, dmc, dpc, kap, tB, vals=vb),
    }
    res = {k: [] for k in runs}
    for rnd in range(4):
        for k, fn in runs.items():
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 50)
    torch.cuda.synchronize()
    assert torch.equal(va[0], vb[0]), "paths disagree"
    for k, v in res.items():
        print("%-28s median %.4f ms  min %.4f ms" % (k, np.median(v), np.min(v)), flush=True)


if __name__ == "__main__":
    main()
