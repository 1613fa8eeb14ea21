"""A/B timing of kernel ablations (HDD_DEBUG_FLAGS) in ONE process, interleaved rounds (guide 5.4 rule 24)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch
import hdd_amd as H

flags = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,4,3,5,6,7").split(",")]
nx, ny = 3200, 640
grid = H.Grid.structured(H.SIMPLEX, nx, ny, (0, 0), (5, 1))
local = grid.local()
rng = np.random.default_rng(10)
perm = 10.0 ** rng.uniform(-3, 3, 2000)
k = torch.from_numpy(local.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
ctx = H.Context(0)
dm = H.DeviceMesh(local)
dp = H.DevicePattern(local)
kap = [H.scalar_fn(H.FN_CONST, 1.0)]
ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
res = {f: [] for f in flags}
for rnd in range(6):
    for f in flags:
        os.environ["HDD_DEBUG_FLAGS"] = str(f)
        for _ in range(3):
            H.assemble(ctx, dm, dp, kap, ten, vals=vals)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(10):
            H.assemble(ctx, dm, dp, kap, ten, vals=vals)
        ev[1].record()
        torch.cuda.synchronize()
        res[f].append(ev[0].elapsed_time(ev[1]) / 10)
os.environ["HDD_DEBUG_FLAGS"] = "0"
for f in flags:
    print("flags=%d  median %.4f ms  min %.4f ms" % (f, np.median(res[f]), np.min(res[f])))
