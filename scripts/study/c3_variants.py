#!/usr/bin/env python3
"""C3 (OS2014 1024^2 Kuhn, affine part + mu-component, sinusoid kappa) under its verification variants, interleaved
rounds in ONE process on one box: the default two-component pass (P1SmoothFusedPolicy TWO), one launch per component
(HDD_VARIANT_C3_PER_COMPONENT: P1SmoothPolicy, one value stream per wave, two waves per SIMD).  Prints the median / min per variant and checks that the variants agree
(to rounding: the fused volume moment is a_c sum w + b_c sum w sin).
usage: python scripts/study/c3_variants.py [rounds]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch  # noqa: E402
import hdd_amd as H  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n = 1024
    grid = H.Grid.structured(H.SIMPLEX, n, n, (-1, -1), (1, 1))
    loc = grid.local()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    kx, ky = 4 * math.pi, 2 * math.pi
    fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, kx, ky, order=3), H.scalar_fn(H.FN_SINUSOID, 0.0, -0.75, kx, ky, order=3)]
    variants = {"two_pass": 0, "per_component": H.VARIANT_C3_PER_COMPONENT}
    ctxs, vals = {}, {}
    for name, v in variants.items():
        ctxs[name] = H.Context(0)
        ctxs[name].set_variant(v)
        vals[name] = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda") for _ in range(2)]
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name in variants:
            fn = lambda: H.assemble(ctxs[name], dm, dp, fns, H.tensor_fn(), vals=vals[name])
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 20)
    for name in variants:
        print("c3 %-14s median %.4f ms  min %.4f ms" % (name, np.median(res[name]), np.min(res[name])), flush=True)
    a, b = vals["two_pass"], vals["per_component"]
    for c in range(2):
        d = (a[c] - b[c]).abs().max().item()
        m = b[c].abs().max().item()
        print("component %d: max |two_pass - per_component| = %.3g (max |value| %.3g)" % (c, d, m))


if __name__ == "__main__":
    main()
