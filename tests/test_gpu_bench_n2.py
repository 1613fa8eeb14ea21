"""bench.py's N > 1 path on one card (the driver's 8-GPU command, rehearsed): two ranks under torch.distributed.run
with the gloo host-staged halo transport on cuda:0, small meshes -- the sharded step, the watchdog-guarded
synchronisations, the max-over-ranks timing and the per-rank kernel labels (`kernels_by_rank`), for the C2 strips
(P1, overlapped schedules) and the C4 subdomain columns (Q1, serial step).  RCCL itself refuses two ranks on one
device, so the transport is gloo here; everything above it is the N-GPU code path."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _check_roofline(r, n):
    """N > 1: frac = every rank's algorithmic bytes / the SLOWEST rank's event-timed step / (N x the per-GPU peak)"""
    assert r["peak"] == n * r["peak_per_gpu"]
    assert r["algorithmic_bytes_all_ranks"] >= r["algorithmic_bytes_per_launch"]
    expect = r["algorithmic_bytes_all_ranks"] / (r["step_ms_event_max_rank"] * 1e-3) / 1e9
    assert abs(r["achieved"] - expect) <= 1e-9 * expect
    assert abs(r["frac"] - expect / r["peak"]) <= 1e-9
    s = r["slowest_rank"]
    assert 0 <= s["rank"] < n and abs(s["step_ms_event"] - r["step_ms_event_max_rank"]) <= 1e-12
    assert abs(s["frac"] - s["algorithmic_bytes"] / (s["step_ms_event"] * 1e-3) / 1e9 / r["peak_per_gpu"]) <= 1e-9


def _run(port, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline"] + extra
    env = dict(os.environ, HDD_BENCH_DEADLINE="60")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


@pytest.mark.timeout(300)
def test_bench_two_ranks_c2_strips():
    d, err = _run(29541, ["--nx", "320", "--ny", "64"])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    r = d["roofline"]
    assert sorted(sum(r["kernels_by_rank"].values(), [])) == [0, 1]
    assert all("P1PwcPolicy" in k for k in r["kernels_by_rank"])
    assert r["step_ms_event_max_rank"] >= r["step_ms_event"] > 0
    _check_roofline(r, 2)
    assert "halo peers [1]" in err and "halo peers [0]" in err


@pytest.mark.timeout(300)
def test_bench_two_ranks_c4_columns():
    d, _ = _run(29542, ["--workload", "c4", "--nx", "352", "--ny", "120"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    r = d["roofline"]
    assert sorted(sum(r["kernels_by_rank"].values(), [])) == [0, 1]
    assert all("Q1PwcPolicy" in k for k in r["kernels_by_rank"])
    assert "then every tile" in d["config"]["parallelism"]
    _check_roofline(r, 2)
    # the C4 rank piece at N = 2 is not the profiled N = 1 launch: no stamped figures
    assert r["traffic"] is None and r["kernel_ms_rocprof"] is None
