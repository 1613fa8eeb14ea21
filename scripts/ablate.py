"""A/B timing of kernel ablations (HDD_DEBUG_FLAGS) in ONE process, interleaved rounds, several workloads
side by side (one of them unchanged serves as the control for box-to-box clock differences).
Flags (swipdg_persistent_kernel, HDD_ABLATION builds: HDD_AMD_LIB=dune-hdd_amd/lib_ab/libhdd_abl.so): 1 = skip
compute, 2 = drop the value stores (range 0), 4 = skip the neighbour gathers, 32 = each wave a contiguous block
of its XCD's tiles, 64 = global round-robin tiles, 128 / 256 = half / all of a tile's stores before the next
tile's gathers.
usage: python scripts/ablate.py c2:0,1 c4:0,8,16 c3:0"""
import os, sys, math
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch
import hdd_amd as H


def workload(cfg, ctx):
    rng = np.random.default_rng(10)
    perm = 10.0 ** rng.uniform(-3, 3, 2000)
    if cfg in ("rhs", "pattern"):   # the f rows on the C2 mesh (scripts/bench_configs.py f)
        grid = H.Grid.structured(H.SIMPLEX, 3200, 640, (0, 0), (5, 1))
        local = grid.local()
        dm = H.DeviceMesh(local)
        if cfg == "pattern":
            return lambda: H.DevicePattern(local, ctx=ctx, dmesh=dm, on_device=True)
        k = torch.from_numpy(local.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
        ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
        out = torch.empty(3 * local.n_own, dtype=torch.float64, device="cuda")
        return lambda: H.rhs(ctx, dm, force=H.esv2007_force(), kappa=H.scalar_fn(H.FN_CONST, 1.0), tensor=ten,
                             dirichlet=H.scalar_fn(H.FN_CONST, 1.0), out=out)
    if cfg == "c3":
        grid = H.Grid.structured(H.SIMPLEX, 1024, 1024, (-1, -1), (1, 1))
        local = grid.local()
        kap = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, 4 * math.pi, 2 * math.pi, order=3),   # OS2014 affine part
               H.scalar_fn(H.FN_SINUSOID, 0.0, -0.75, 4 * math.pi, 2 * math.pi, order=3)]  # and mu-component
        ten = H.tensor_fn()
    else:
        et, nx, ny, p = (H.SIMPLEX, 3200, 640, 1) if cfg == "c2" else (H.CUBE, 3520, 1200, 8)
        grid = H.Grid.structured(et, nx, ny, (0, 0), (5, 1), px=p, py=p)
        local = grid.local()
        k = torch.from_numpy(local.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
        kap = [H.scalar_fn(H.FN_CONST, 1.0)]
        ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    dm = H.DeviceMesh(local)
    dp = H.DevicePattern(local)
    vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda") for _ in kap]
    return lambda: H.assemble(ctx, dm, dp, kap, ten, vals=vals)


def main():
    groups = sys.argv[1:] or ["c2:0", "c4:0"]
    # the debug flags are read once per context (hdd_ctx_create): one context per flag value
    ctxs = {}
    runs = []
    for g in groups:
        cfg, fl = g.split(":")
        for f in fl.split(","):
            f = int(f)
            if f not in ctxs:
                os.environ["HDD_DEBUG_FLAGS"] = str(f)
                ctxs[f] = H.Context(0)
            runs.append((cfg, f, workload(cfg, ctxs[f])))
    os.environ["HDD_DEBUG_FLAGS"] = "0"
    res = {(c, f): [] for c, f, _ in runs}
    for rnd in range(int(os.environ.get("ABLATE_ROUNDS", "6"))):
        for cfg, f, fn in runs:
            for _ in range(3):
                fn()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            res[(cfg, f)].append(ev[0].elapsed_time(ev[1]) / 10)
    for cfg, f, _ in runs:
        r = res[(cfg, f)]
        print("%s flags=%-3d median %.4f ms  min %.4f ms" % (cfg, f, np.median(r), np.min(r)), flush=True)


if __name__ == "__main__":
    main()
