"""Tiles (single-wave workgroups) per CU of the persistent tile kernels, swept in ONE process, interleaved rounds: one
context per value (HDD_P1_WGCU is read at context creation; it overrides every persistent policy's measured WGCU,
still capped by the LDS).  Only the ablation build reads it (make -C dune-hdd_amd ablation; run with
HDD_AMD_LIB=dune-hdd_amd/lib_ab/libhdd_abl.so): release libraries take no kernel choice from the environment.
A value W + 16 C (C > 0) runs W tiles per CU with at most C resident per CU (the dynamic LDS padded to 160 KB / C).
NOTE: this in-process sweep can mislead (profiles/r06/e_wgcu: bimodal at 3 per CU); confirm a choice with bench.py
in fresh processes, the way the driver measures.
usage: python scripts/sweep_wgcu.py c4|c2|c3 [wgcu ...]   (default: 4 5 6 7 8)"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch  # noqa: E402
import hdd_amd as H  # noqa: E402


def main():
    args = sys.argv[1:]
    wl = args.pop(0) if args and args[0] in ("c2", "c3", "c4") else "c4"
    values = [int(v) for v in args] or [4, 5, 6, 7, 8]
    if wl == "c3":   # OS2014 1024^2 Kuhn, affine part + mu-component (scripts/bench_configs.py c3)
        local = H.Grid.structured(H.SIMPLEX, 1024, 1024, (-1, -1), (1, 1)).local()
        kap = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, 4 * math.pi, 2 * math.pi, order=3),
               H.scalar_fn(H.FN_SINUSOID, 0.0, -0.75, 4 * math.pi, 2 * math.pi, order=3)]
        ten = H.tensor_fn()
    else:
        et, nx, ny, p = (H.SIMPLEX, 3200, 640, 1) if wl == "c2" else (H.CUBE, 3520, 1200, 8)
        grid = H.Grid.structured(et, nx, ny, (0, 0), (5, 1), px=p, py=p)
        local = grid.local()
        rng = np.random.default_rng(10)
        k = torch.from_numpy(local.checkerboard((0, 0), (5, 1), 100, 20, 10.0 ** rng.uniform(-3, 3, 2000))).cuda()
        kap, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    dm, dp = H.DeviceMesh(local), H.DevicePattern(local)
    vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda") for _ in kap]
    ctxs = {}
    for v in values:
        os.environ["HDD_P1_WGCU"] = str(v)
        ctxs[v] = H.Context(0)
    os.environ.pop("HDD_P1_WGCU", None)
    res = {v: [] for v in values}
    for _ in range(6):
        for v in values:
            for _ in range(3):
                H.assemble(ctxs[v], dm, dp, kap, ten, vals=vals)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                H.assemble(ctxs[v], dm, dp, kap, ten, vals=vals)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 10)
    for v in values:
        print("%s wgcu=%d median %.4f ms  min %.4f ms" % (wl, v, np.median(res[v]), np.min(res[v])), flush=True)


if __name__ == "__main__":
    main()
