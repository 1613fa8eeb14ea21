"""Timeline of the sharded step's kernels on one card (run under `rocprofv3 --kernel-trace`), for rank r of an
N-rank C4 / C2 decomposition with the loopback transfer (HDD_SHARD_NO_TRANSFER): `reps` steps after a warmup,
each step bracketed by a tiny marker fill so the trace can be cut into steps.  Summarise with --summary <csv>.
With --btb the steps run back to back (no host synchronisation between them, one marker before and one after),
and the summary lists every kernel of the run with its start relative to the previous persistent launch's start
and end: the step-to-step period and the gap the join leaves between the launches.
usage: python scripts/study/step_timeline.py c4 8 0 [reps [flags]] [--btb]
       python scripts/study/step_timeline.py --summary <run_kernel_trace.csv>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))


def summary(path):
    import csv
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "FillFunctor" in name:          # the marker between steps
            if cur:
                steps.append(cur)
            cur = []
            continue
        if cur is not None:
            cur.append((name.split("(")[0].replace("void ", "")[:90], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if cur:
        steps.append(cur)
    steps = [s for s in steps if s]
    if len(steps) == 1 and sum("persistent" in n for n, _, _ in steps[0]) > 2:   # --btb: one segment
        return summary_btb(steps[0])
    steps = steps[-5:]
    for k, s in enumerate(steps):
        t0 = min(b for _, b, _ in s)
        t1 = max(e for _, _, e in s)
        print("step %d: %.1f us" % (k, (t1 - t0) / 1e3))
        for name, b, e in s:
            print("   %7.1f .. %7.1f us  %s" % ((b - t0) / 1e3, (e - t0) / 1e3, name))


def summary_btb(seg):
    pers = [(b, e) for n, b, e in seg if "persistent" in n]
    per = [(pers[i + 1][0] - pers[i][0]) / 1e3 for i in range(len(pers) - 1)]
    gap = [(pers[i + 1][0] - pers[i][1]) / 1e3 for i in range(len(pers) - 1)]
    dur = [(e - b) / 1e3 for b, e in pers]
    print("%d persistent launches back to back: period median %.1f us (min %.1f, max %.1f), launch median %.1f us, "
          "gap end -> next start median %.1f us (min %.1f, max %.1f)"
          % (len(pers), np.median(per), min(per), max(per), np.median(dur), np.median(gap), min(gap), max(gap)))
    t0 = pers[len(pers) // 2][0]
    for name, b, e in seg:   # the middle of the run in detail
        if -150e3 <= b - t0 <= 250e3:
            print("   %7.1f .. %7.1f us  %s" % ((b - t0) / 1e3, (e - t0) / 1e3, name))


def main():
    btb = "--btb" in sys.argv
    if btb:
        sys.argv.remove("--btb")
    if sys.argv[1] == "--summary":
        return summary(sys.argv[2])
    import torch
    import hdd_amd as H
    wl, n, rank = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    flags = H.SHARD_NO_TRANSFER | (int(sys.argv[5]) if len(sys.argv) > 5 else 0)
    if wl == "c4":
        grid = H.Grid.structured(H.CUBE, 3520, 1200, (0.0, 0.0), (5.0, 1.0), px=8, py=8)
        up, ncx, ncell = (5.0, 1.0), 100, 2000
    else:
        grid = H.Grid.structured(H.SIMPLEX, 3200 * n, 640, (0.0, 0.0), (5.0 * n, 1.0), px=n, py=1)
        up, ncx, ncell = (5.0 * n, 1.0), 100 * n, 2000 * n
    perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=ncell)
    ctx = H.Context(0)
    sh = H.Shard(ctx, grid, n, rank)
    k = torch.from_numpy(sh.checkerboard((0.0, 0.0), up, ncx, 20, perm)).cuda()
    _, _, _, pat = sh.pattern(ctx, 0)
    vals = [torch.empty(sh.info.nnz, dtype=torch.float64, device="cuda")]
    kap, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    marker = torch.empty(64, dtype=torch.float64, device="cuda")
    for _ in range(10):
        H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=flags)
    torch.cuda.synchronize()
    if btb:
        marker.fill_(0.0)
        torch.cuda.synchronize()
        for _ in range(reps):
            H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=flags)
        torch.cuda.synchronize()
    for _ in range(0 if btb else reps):
        marker.fill_(0.0)
        torch.cuda.synchronize()
        H.assemble_sharded(ctx, sh, None, kap, ten, pat, vals, flags=flags)
        torch.cuda.synchronize()
    marker.fill_(1.0)
    torch.cuda.synchronize()
    print("done", wl, n, rank)


if __name__ == "__main__":
    main()
