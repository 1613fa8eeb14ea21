#!/usr/bin/env python3
"""C3 (OS2014 1024^2 Kuhn, two components, sinusoid kappa): does the placement of the two value arrays relative to
each other change the two-component pass's store rate?  Each wave writes its tile's row blocks at the same offset X
of both arrays, so the two write fronts sit at a fixed distance; if that distance maps both onto the same HBM
channels / banks they contend.  Variants: two separate allocations (the default), and slices of one buffer with the
second array starting nnz * 8 + skew bytes after the first (skews in bytes, multiples of 256).  Interleaved rounds
in one process; prints median / min per placement and checks that every placement writes identical values.
usage: python scripts/study/c3_skew.py [rounds]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch  # noqa: E402
import hdd_amd as H  # noqa: E402

SKEWS = [0, 256, 4096, 65536, 1 << 20, (1 << 20) + 4096, 3 << 20, 9 * 4096 + 256]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n = 1024
    grid = H.Grid.structured(H.SIMPLEX, n, n, (-1, -1), (1, 1))
    loc = grid.local()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    kx, ky = 4 * math.pi, 2 * math.pi
    fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, kx, ky, order=3), H.scalar_fn(H.FN_SINUSOID, 0.0, -0.75, kx, ky, order=3)]
    ctx = H.Context(0)
    nnz = dp.nnz
    place = {"separate": [torch.empty(nnz, dtype=torch.float64, device="cuda") for _ in range(2)]}
    big = torch.empty(2 * nnz + max(SKEWS) // 8, dtype=torch.float64, device="cuda")
    for s in SKEWS:
        o = nnz + s // 8
        place["skew_%d" % s] = [big[:nnz], big[o:o + nnz]]
    print("nnz %d, separate arrays at +%d bytes" % (nnz, place["separate"][1].data_ptr() - place["separate"][0].data_ptr()),
          flush=True)
    res = {k: [] for k in place}
    for _ in range(rounds):
        for name, vals in place.items():
            fn = lambda: H.assemble(ctx, dm, dp, fns, H.tensor_fn(), vals=vals)
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 20)
    for name in place:
        print("c3 %-22s median %.4f ms  min %.4f ms" % (name, np.median(res[name]), np.min(res[name])), flush=True)
    ref = [v.clone() for v in place["separate"]]
    H.assemble(ctx, dm, dp, fns, H.tensor_fn(), vals=place["separate"])
    for name, vals in place.items():
        if name == "separate":
            continue
        H.assemble(ctx, dm, dp, fns, H.tensor_fn(), vals=vals)
        same = all(torch.equal(vals[c], ref[c]) for c in range(2))
        print("%s: values identical to separate: %s" % (name, same), flush=True)


if __name__ == "__main__":
    main()
