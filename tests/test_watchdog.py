"""The sharded step's watchdog (the first multi-GPU run must fail loudly, not hang).

A peer whose halo never arrives is injected on the in-process device transport (hdd_device_hub_stall: the peer's
sends complete only when a device-side gate opens).  Checks:
  * hdd_block_step_query names the stage that has not completed (the halo exchange), hdd_block_step_sync returns
    HDD_ERR_TIMEOUT within its deadline with the rank, stage and peers in the message, and after the gate opens
    the step completes with the correct values;
  * bench.py's synchronisation path (hdd_amd.watchdog.guarded_sync) in a subprocess: non-zero exit status 3 within
    the deadline (+ start-up), the rank and the stage on stderr -- no hang, no retry, no re-exec.
Reference: SURVEY.md 8(e) (halo exchange of the sharded BlockSWIPDG step).
"""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu


def test_step_sync_names_the_stalled_stage():
    import threading

    import torch
    from test_device_transport import _Rank, _layout, _single_gpu
    n = 2
    grid, tk, two = _layout("c4_q1", n)
    hub = H.DeviceHub(n)
    ranks = [_Rank(hub, grid, n, r, tk, two, 0) for r in range(n)]
    for R in ranks:
        R.reset()
    torch.cuda.synchronize()
    hub.stall(1, 30.0)

    def work(r):
        R = ranks[r]
        H.assemble_sharded(R.ctx, R.sh, R.comm, R.kappas, R.tensor, R.pat, R.vals, stream=R.stream.cuda_stream)

    th = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    try:
        time.sleep(0.5)   # (the pack itself takes microseconds)
        st, name = ranks[0].sh.step_query()
        assert st == 2 and "exchange" in name, (st, name)
        t0 = time.perf_counter()
        with pytest.raises(H.HddError) as ei:
            ranks[0].sh.step_sync(1.0, stream=ranks[0].stream.cuda_stream)
        dt = time.perf_counter() - t0
        msg = str(ei.value)
        assert "status 6" in msg and "rank 0 of 2" in msg and "halo exchange" in msg and "peers: 1" in msg, msg
        assert 1.0 <= dt < 5.0, dt
    finally:
        hub.release()
    for R in ranks:
        R.sh.step_sync(60.0, stream=R.stream.cuda_stream)
        assert R.sh.step_query()[0] == 0
    torch.cuda.synchronize()
    got = np.concatenate([np.stack([v.cpu().numpy() for v in R.vals]) for R in ranks], axis=1)
    ref = _single_gpu(grid, tk, two)
    assert np.array_equal(got.view(np.int64), ref.view(np.int64))


def test_guarded_sync_exits_with_the_stage_named():
    deadline = 3.0
    t0 = time.perf_counter()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "stall_step.py"), str(deadline)],
                       capture_output=True, text=True, timeout=100, cwd=ROOT)
    dt = time.perf_counter() - t0
    err = p.stderr
    assert p.returncode == 3, (p.returncode, p.stdout[-2000:], err[-2000:])
    assert "[hdd watchdog] rank 0" in err and "halo exchange" in err and "halo peers [1]" in err, err[-2000:]
    assert "watchdog did not fire" not in p.stdout
    assert dt < 90.0, dt
