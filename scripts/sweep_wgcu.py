import os, sys, subprocess
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch, hdd_amd as H
grid = H.Grid.structured(H.SIMPLEX, 3200, 640, (0, 0), (5, 1))
local = grid.local()
rng = np.random.default_rng(10)
k = torch.from_numpy(local.checkerboard((0, 0), (5, 1), 100, 20, 10.0 ** rng.uniform(-3, 3, 2000))).cuda()
ctx = H.Context(0); dm = H.DeviceMesh(local); dp = H.DevicePattern(local)
kap = [H.scalar_fn(H.FN_CONST, 1.0)]; ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
cfgs = [("0", None)] + [("16", str(w)) for w in (1, 2, 3, 4, 5, 6, 8)]
res = {c: [] for c in cfgs}
for rnd in range(5):
    for c in cfgs:
        os.environ["HDD_DEBUG_FLAGS"] = c[0]
        if c[1]: os.environ["HDD_P1_WGCU"] = c[1]
        for _ in range(3): H.assemble(ctx, dm, dp, kap, ten, vals=vals)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): H.assemble(ctx, dm, dp, kap, ten, vals=vals)
        e1.record(); torch.cuda.synchronize()
        res[c].append(e0.elapsed_time(e1) / 10)
for c in cfgs:
    print("flags=%s wgcu=%s median %.4f ms" % (c[0], c[1], np.median(res[c])))
