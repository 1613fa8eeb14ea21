"""element-list fixup vs the tile kernel, bit for bit, per (element type, tensor, kappa)"""
import os, sys, math
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch
import hdd_amd as H
print("lib", H.lib()._name)
ctx = H.Context(0)
rng = np.random.default_rng(1)
for et in (H.SIMPLEX, H.CUBE):
    grid = H.Grid.structured(et, 96, 40, (0, 0), (5, 1), px=4, py=2)
    loc = grid.local(2, 6)
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    n = loc.n_local
    iso = torch.from_numpy(rng.uniform(0.5, 2, n)).cuda()
    sym = torch.from_numpy(np.stack([rng.uniform(1, 2, n), rng.uniform(-.3, .3, n), rng.uniform(1, 2, n)])).cuda().contiguous()
    kpe = torch.from_numpy(rng.uniform(0.5, 2, n)).cuda()
    for tname, ten in [("iso", H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=iso)),
                       ("sym", H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=sym)), ("const", H.tensor_fn())]:
        for kname, kap in [("const", [H.scalar_fn(H.FN_CONST, 1.0)]),
                           ("pe", [H.scalar_fn(H.FN_PER_ELEM, per_elem=kpe)]),
                           ("sin", [H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=3.0, ky=2.0, order=3)]),
                           ("sin2", [H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=3.0, ky=2.0, order=3),
                                     H.scalar_fn(H.FN_SINUSOID, 0.0, b=1.0, kx=3.0, ky=2.0, order=3)])]:
            ref = H.assemble(ctx, dm, dp, kap, ten)
            vals = [torch.full_like(r, float("nan")) for r in ref]
            lst = torch.arange(loc.n_own, dtype=torch.int32, device="cuda")
            H.assemble_tiles(ctx, dm, dp, kap, ten, lst, vals, elements=True)
            torch.cuda.synchronize()
            for c, (v, r) in enumerate(zip(vals, ref)):
                d = (v != r).sum().item()
                rel = ((v - r).abs().max() / r.abs().max()).item()
                print("et %d %-5s %-5s comp %d: %6d differ of %d, max rel %.3e" % (et, tname, kname, c, d, v.numel(), rel), flush=True)
