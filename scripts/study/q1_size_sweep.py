"""C4-type Q1 assemblies (SPE10 checkerboard, 8 x 8 subdomains, one launch) of growing size under several verification
variants (hdd_ctx_set_variant), interleaved rounds in one process -- where the half-image kernel on vertex-indexed
geometry (default, 0) and the whole-tile kernel (1 = HDD_VARIANT_Q1_WHOLE_TILE; 3 = on element-major coords) cross over.
usage: python scripts/study/q1_size_sweep.py [--sizes NXxNY,...] [variants ...]     (default: 0 1 3)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch  # noqa: E402
import hdd_amd as H  # noqa: E402


def main():
    args = sys.argv[1:]
    sizes = [(440, 1200), (880, 1200), (1760, 1200), (3520, 1200), (3520, 2400)]
    if args and args[0] == "--sizes":
        sizes = [tuple(int(v) for v in z.split("x")) for z in args[1].split(",")]
        args = args[2:]
    flags = [int(f) for f in args] or [0, 1, 3]
    ctxs = {}
    for f in flags:
        ctxs[f] = H.Context(0)
        ctxs[f].set_variant(f)
    perm = 10.0 ** np.random.default_rng(10).uniform(-3, 3, 2000)
    for nx, ny in sizes:
        grid = H.Grid.structured(H.CUBE, nx, ny, (0, 0), (5.0 * nx / 3520, 1.0 * ny / 1200), px=8, py=8)
        loc = grid.local()
        dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
        k = torch.from_numpy(loc.checkerboard((0, 0), (5.0 * nx / 3520, 1.0 * ny / 1200), 100, 20, perm)).cuda()
        kap, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
        vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
        res = {f: [] for f in flags}
        for _ in range(5):
            for f in flags:
                for _ in range(3):
                    H.assemble(ctxs[f], dm, dp, kap, ten, vals=vals)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    H.assemble(ctxs[f], dm, dp, kap, ten, vals=vals)
                e1.record()
                torch.cuda.synchronize()
                res[f].append(e0.elapsed_time(e1) / 10)
        line = "  ".join("variant %d %.4f ms" % (f, np.median(res[f])) for f in flags)
        print("%d x %d (%d elements, %d tiles): %s" % (nx, ny, loc.n_own, (loc.n_own + 63) // 64, line), flush=True)
        del dm, dp, vals, loc


if __name__ == "__main__":
    main()
