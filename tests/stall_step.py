"""Subprocess body of tests/test_watchdog.py: a 2-rank sharded step over the in-process device transport whose rank 1
never delivers its halo (hdd_device_hub_stall), synchronised the way bench.py's N > 1 path does (hdd_amd.watchdog).
Expected: the watchdog fires after the deadline, names rank 0 and the halo-exchange stage on stderr, opens the
injected gate (so the device drains) and exits with status 3.  Exit 0 = the stall went unnoticed (a failure)."""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import hdd_amd as H  # noqa: E402
from hdd_amd.watchdog import guarded_sync  # noqa: E402
from test_device_transport import _Rank, _layout  # noqa: E402


def main():
    deadline = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    n = 2
    grid, tk, two = _layout("c4_q1", n)
    hub = H.DeviceHub(n)
    ranks = [_Rank(hub, grid, n, r, tk, two, 0) for r in range(n)]
    for R in ranks:
        R.reset()
    torch.cuda.synchronize()
    hub.stall(1, 30.0)   # rank 1's sends complete only when the gate opens (the kernel ends by itself after 30 s)
    errs = [None] * n

    def work(r):
        R = ranks[r]
        try:
            H.assemble_sharded(R.ctx, R.sh, R.comm, R.kappas, R.tensor, R.pat, R.vals, stream=R.stream.cuda_stream)
        except Exception as e:   # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if any(errs):
        print("enqueue failed: %s" % errs, file=sys.stderr)
        hub.release()
        return 2
    st = ranks[0].sh.step_query()
    print("stage right after enqueue: %s" % (st,), flush=True)
    guarded_sync(torch, ranks[0].sh, 0, "the stalled step", deadline, on_timeout=hub.release,
                 stream=ranks[0].stream.cuda_stream)
    print("watchdog did not fire", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
