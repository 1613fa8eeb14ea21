"""The sharded step over the in-process device transport (hdd_device_hub): all N ranks of a decomposition as
thread ranks on ONE card, each with its own context, shard, stream and device communicator -- the stream /
event schedule of the RCCL branch (pack on the transfer stream, the exchange there, the ghost-adjacent element
pass right behind it, the SKIP launch on the rank's stream, event join).

Timed (host wall clock over `reps` steps of every rank, each rank's stream synchronised at the end):
  all ranks, sharded step (default / in place / inline / serial schedules)
against
  all ranks, one launch each of the owned range with valid ghosts (HDD_SHARD_NO_HALO, the same threads)
  the whole grid in one launch (the single-GPU bench kernel).
On one card the N ranks share the CUs, so this is the whole-grid cost of the decomposition (the N-GPU step
time is not measurable here); the difference between the step and the NO_HALO rows is what the exchange
schedule adds when every rank runs it at once.
usage: python scripts/study/device_step.py [c2|c4] [N ...]"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import torch  # noqa: E402
import hdd_amd as H  # noqa: E402


def layout(workload, n):
    if workload == "c4":
        return H.Grid.structured(H.CUBE, 3520, 1200, (0.0, 0.0), (5.0, 1.0), px=8, py=8), (5.0, 1.0), 100, 2000
    return (H.Grid.structured(H.SIMPLEX, 3200 * n, 640, (0.0, 0.0), (5.0 * n, 1.0), px=n, py=1), (5.0 * n, 1.0),
            100 * n, 2000 * n)


class Rank:
    def __init__(self, hub, grid, n, r, up, ncx, perm):
        self.ctx = H.Context(0)
        self.sh = H.Shard(self.ctx, grid, n, r)
        k = self.sh.checkerboard((0.0, 0.0), up, ncx, 20, perm)
        owned = np.zeros(self.sh.n_local, bool)
        owned[self.sh.own_begin:self.sh.own_end] = True
        k[~owned] = np.nan          # ghosts come from the exchange
        self.k = torch.from_numpy(k).cuda()
        self.k_valid = torch.from_numpy(self.sh.checkerboard((0.0, 0.0), up, ncx, 20, perm)).cuda()
        _, _, _, self.pat = self.sh.pattern(self.ctx, 0)
        self.vals = [torch.empty(self.sh.info.nnz, dtype=torch.float64, device="cuda")]
        self.comm = H.Comm.device(hub, r, 0)
        self.stream = torch.cuda.Stream()
        self.kap = [H.scalar_fn(H.FN_CONST, 1.0)]


def run_all(ranks, flags, reps, valid=False):
    errs = [None] * len(ranks)

    def work(i):
        R = ranks[i]
        ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=R.k_valid if valid else R.k)
        try:
            for _ in range(reps):
                H.assemble_sharded(R.ctx, R.sh, R.comm, R.kap, ten, R.pat, R.vals, flags=flags,
                                   stream=R.stream.cuda_stream)
            R.stream.synchronize()
        except Exception as e:  # noqa: BLE001
            errs[i] = e

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(ranks))]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    assert all(e is None for e in errs), errs
    return dt / reps * 1e3


def main():
    args = sys.argv[1:]
    workload = args.pop(0) if args and args[0] in ("c2", "c4") else "c4"
    reps, rounds = 40, 4
    for n in [int(a) for a in args] or [2, 8]:
        grid, up, ncx, ncell = layout(workload, n)
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=ncell)
        hub = H.DeviceHub(n)
        ranks = [Rank(hub, grid, n, r, up, ncx, perm) for r in range(n)]
        rows = {
            "NO_HALO, all ranks (one launch each)": (H.SHARD_NO_HALO, True),
            "step, default": (0, False),
            "step, fixup in place": (H.SHARD_FIX_INPLACE, False),
            "step, default, launch after the halo work (r3)": (H.SHARD_LAUNCH_LAST, False),
            "step, fixup inline (round 2)": (H.SHARD_FIX_INLINE, False),
            "step, serial": (H.SHARD_NO_OVERLAP, False),
        }
        res = {}
        for name, (f, valid) in rows.items():
            run_all(ranks, f, 5, valid)   # warm
            res[name] = [run_all(ranks, f, reps, valid) for _ in range(rounds)]
        # the whole grid in one launch (single-GPU reference)
        ctx = H.Context(0)
        loc = grid.local()
        dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
        kl = torch.from_numpy(loc.checkerboard((0.0, 0.0), up, ncx, 20, perm)).cuda()
        tl = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=kl)
        vl = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
        kap = [H.scalar_fn(H.FN_CONST, 1.0)]
        for _ in range(5):
            H.assemble(ctx, dm, dp, kap, tl, vals=vl)
        full = []
        for _ in range(rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                H.assemble(ctx, dm, dp, kap, tl, vals=vl)
            torch.cuda.synchronize()
            full.append((time.perf_counter() - t0) / reps * 1e3)
        res["whole grid, one launch"] = full
        del dm, dp, loc
        # results: every rank's values == the whole-grid assembly's rows (bitwise) after the default step
        run_all(ranks, 0, 2)
        ref = vl[0].cpu().numpy()
        got = np.concatenate([R.vals[0].cpu().numpy() for R in ranks])
        same = ref.shape == got.shape and np.array_equal(ref.view(np.int64), got.view(np.int64))
        info = ranks[n // 2].sh.info
        print("%s N=%d device transport, %d thread ranks on one card (middle rank: %d owned, %d ghost-adjacent, "
              "%d peers); sharded rows == whole grid bitwise: %s"
              % (workload, n, n, ranks[n // 2].sh.n_own, info.halo_elements, info.n_peers, same))
        base = float(np.median(res["NO_HALO, all ranks (one launch each)"]))
        for name, v in res.items():
            print("  %-40s median %.4f ms  min %.4f ms  (%+.1f %% vs NO_HALO)"
                  % (name, np.median(v), np.min(v), 100 * (np.median(v) / base - 1)), flush=True)
        del ranks, hub


if __name__ == "__main__":
    main()
