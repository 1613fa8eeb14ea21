"""The sharded step's RCCL branch on one GPU: N thread ranks of one process over the in-process device transport
(hdd_device_hub / hdd_comm_create_device).

Over RCCL the step packs on the communicator's transfer stream, posts the group send/recv there, computes the
ghost-adjacent elements on that stream right behind the receives and joins it by an event
(shard.hip: ps = comm->xfer, the fixup on ps, hdd_comm_wait's event join).  The device transport takes exactly
that branch -- only the ncclSend/ncclRecv pair is replaced by (wait for the source's packed event, hipMemcpyAsync,
record "copied"; the completion waits for every destination's "copied") -- so these tests execute the stream /
event schedule the driver's 8-GPU run uses, which no host-transport test reaches.

Reference semantics: block-swipdg.hh:355-382 (the owner of ss writes A_ss and A_ss,nn), SURVEY.md 8(e).
Checks, for C2-like strips (P1 Kuhn, one subdomain column per rank) and C4-like subdomain columns (Q1, 2 x 4
subdomains per rank), at N = 2 and N = 3 (a middle rank with two peers):
  * every rank's rows are bit-identical to the single-GPU assembly of the same block grid;
  * Q1 with a smooth diffusion factor (quadrature policy) through every schedule, the side-buffer one included
    (its value-major pass exists for the closed-form policy only: ADVICE r5);
  * the default, in-place, side-buffer (scatter), inline, split-tile and serial schedules agree bit for bit;
  * three consecutive steps per schedule (the second and third re-pack while the previous step's receivers may
    still read the send buffers: the "copied" ordering), with the ghost columns reset to NaN before each
    schedule, so a missing, stale or misrouted halo record shows up as a NaN or a wrong entry.
"""
import os
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "dune-hdd_amd", "python"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
import hdd_amd as H  # noqa: E402

LOWER, UPPER = (0.0, 0.0), (5.0, 1.0)
SCHEDULES = {
    "default": 0,
    "inplace": H.SHARD_FIX_INPLACE,
    "scatter": H.SHARD_FIX_SCATTER,
    "inline": H.SHARD_FIX_INLINE,
    "split": H.SHARD_SPLIT_TILES,
    "serial": H.SHARD_NO_OVERLAP,
}


def _layout(kind, n):
    """(grid, tensor kind, two components, halo geometry)"""
    if kind == "c2_p1":     # bench.py's weak-scaling strips, scaled down: one subdomain column per rank
        return H.Grid.structured(H.SIMPLEX, 96 * n, 24, LOWER, UPPER, px=n, py=1), H.TENSOR_ISO_PER_ELEM, False
    if kind == "c4_q1":     # BASELINE C4's column strips of subdomains, scaled down: 2 x 4 subdomains per rank
        return H.Grid.structured(H.CUBE, 56 * n, 36, LOWER, UPPER, px=2 * n, py=4), H.TENSOR_ISO_PER_ELEM, True
    if kind == "p1_sym":    # symmetric tensor, per-element diffusion factor
        return H.Grid.structured(H.SIMPLEX, 40 * n, 18, LOWER, UPPER, px=2 * n, py=2), H.TENSOR_SYM_PER_ELEM, True
    if kind == "q1_smooth":   # Q1 with a smooth (sinusoid) diffusion factor: the quadrature policy, no closed form
        return H.Grid.structured(H.CUBE, 48 * n, 30, LOWER, UPPER, px=2 * n, py=3), H.TENSOR_ISO_PER_ELEM, "smooth"
    raise ValueError(kind)


def _kappas(two, kap_dev):
    if two == "smooth":
        return [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.5, 3.0, 2.0, order=3)]
    return [H.scalar_fn(H.FN_CONST, 1.0)] + ([H.scalar_fn(H.FN_PER_ELEM, per_elem=kap_dev)] if two else [])


def _coefficients(centers):
    x, y = centers
    iso = 10.0 ** (3.0 * np.sin(3.1 * x) * np.cos(2.3 * y))
    sym = np.ascontiguousarray(np.stack([1.5 + np.sin(x) ** 2, 0.3 * np.cos(2 * x + y), 1.2 + np.cos(y) ** 2]))
    kap = 1.0 + 0.5 * np.sin(5 * x + 3 * y) ** 2
    return iso, sym, kap


def _single_gpu(grid, tk, two):
    import torch
    loc = grid.local()
    iso, sym, kap = _coefficients(loc.centers())
    ctx = H.Context(0)
    dm, dp = H.DeviceMesh(loc, 0), H.DevicePattern(loc, 0)
    tensor = H.tensor_fn(tk, per_elem=torch.from_numpy(iso if tk == H.TENSOR_ISO_PER_ELEM else sym).cuda())
    kappas = _kappas(two, torch.from_numpy(kap).cuda())
    out = np.stack([v.cpu().numpy() for v in H.assemble(ctx, dm, dp, kappas, tensor)])
    torch.cuda.synchronize()
    return out


class _Rank:
    """one thread rank: context, shard, owned coefficients (ghost columns NaN), pattern, device communicator"""

    def __init__(self, hub, grid, n, r, tk, two, flags_extra):
        import torch
        self.ctx = H.Context(0)
        self.sh = H.Shard(self.ctx, grid, n, r)
        owned = np.zeros(self.sh.n_local, bool)
        owned[self.sh.own_begin:self.sh.own_end] = True
        iso, sym, kap = _coefficients(self.sh.centers())
        self.host = []
        for a in (iso if tk == H.TENSOR_ISO_PER_ELEM else sym, kap):
            a = a.copy()
            a[..., ~owned] = np.nan
            self.host.append(a)
        self.dev = [torch.from_numpy(a).cuda() for a in self.host]
        self.tensor = H.tensor_fn(tk, per_elem=self.dev[0])
        self.kappas = _kappas(two, self.dev[1])
        _, _, _, self.pat = self.sh.pattern(self.ctx)
        self.comm = H.Comm.device(hub, r, 0)
        self.stream = torch.cuda.Stream()
        self.flags_extra = flags_extra

    def reset(self):
        import torch
        for d, h in zip(self.dev, self.host):
            d.copy_(torch.from_numpy(h))
        self.vals = [torch.full((self.sh.info.nnz,), float("nan"), dtype=torch.float64, device="cuda")
                     for _ in self.kappas]


def run_device_ranks(grid, n, tk, two, schedules, steps=3, flags_extra=0):
    """-> {schedule: values [n_comp][nnz] concatenated over the ranks}, per-rank shard infos"""
    import torch
    hub = H.DeviceHub(n)
    ranks = [_Rank(hub, grid, n, r, tk, two, flags_extra) for r in range(n)]
    out = {}
    for name, fl in schedules.items():
        for R in ranks:
            R.reset()
        torch.cuda.synchronize()
        errs = [None] * n

        def work(r):
            R = ranks[r]
            try:
                for _ in range(steps):
                    H.assemble_sharded(R.ctx, R.sh, R.comm, R.kappas, R.tensor, R.pat, R.vals,
                                       flags=fl | R.flags_extra, stream=R.stream.cuda_stream)
                R.stream.synchronize()
            except Exception as e:   # noqa: BLE001 -- reported below
                errs[r] = e

        th = [threading.Thread(target=work, args=(r,)) for r in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert all(e is None for e in errs), (name, errs)
        torch.cuda.synchronize()
        out[name] = np.concatenate([np.stack([v.cpu().numpy() for v in R.vals]) for R in ranks], axis=1)
    infos = [R.sh.info for R in ranks]
    return out, infos


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [("c2_p1", 2), ("c2_p1", 3), ("c4_q1", 2), ("c4_q1", 3), ("p1_sym", 3),
                                    ("q1_smooth", 3)])
def test_device_transport_equals_single_gpu(kind, n):
    grid, tk, two = _layout(kind, n)
    got, infos = run_device_ranks(grid, n, tk, two, SCHEDULES)
    peers = [i.n_peers for i in infos]
    assert peers == ([1, 1] if n == 2 else [1, 2, 1]), peers          # n = 3: the middle rank has two peers
    assert all(i.halo_recv > 0 and i.halo_elements > 0 for i in infos)
    ref = _single_gpu(grid, tk, two)
    for name, v in got.items():
        assert v.shape == ref.shape, name
        assert np.isfinite(v).all(), "%s: a ghost column was not filled by the halo" % name
        assert np.array_equal(v.view(np.int64), ref.view(np.int64)), "%s: sharded != single-GPU (bitwise)" % name


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_device_transport_c4_full_size_n8():
    """BASELINE C4 at full size (3520 x 1200 Q1 quads, 8 x 8 subdomains) as 8 thread ranks of one column each on
    one card, at production shard sizes: the default (serial) step, the in-place schedule (half-image SKIP launch
    whose full tiles drop the 1,200 / 2,400 ghost-adjacent elements' chunks at the store, grid reserve, element
    pass beside it) and the value-major side buffer (full launch, copy after the join) -- every rank's rows
    bit-identical to the whole-grid assembly, two steps each.  (The SKIP store path's store-data hazard of round 5
    showed only at this size: 15,448 wrong low words next to skipped elements.)"""
    grid = H.Grid.structured(H.CUBE, 3520, 1200, LOWER, UPPER, px=8, py=8)
    sched = {"default": 0, "inplace": H.SHARD_FIX_INPLACE, "scatter": H.SHARD_FIX_SCATTER}
    got, infos = run_device_ranks(grid, 8, H.TENSOR_ISO_PER_ELEM, False, sched, steps=2)
    assert [i.n_peers for i in infos] == [1] + [2] * 6 + [1]
    ref = _single_gpu(grid, H.TENSOR_ISO_PER_ELEM, False)
    for name in sched:
        v = got[name]
        assert v.shape == ref.shape and np.isfinite(v).all(), name
        assert np.array_equal(v.view(np.int64), ref.view(np.int64)), name


@pytest.mark.gpu
def test_device_transport_c2_full_strips_n4():
    """bench.py's C2 weak-scaling layout at full per-rank size (3200 x 640 Kuhn strips, 4.1 M triangles per rank),
    N = 4 thread ranks on one card: the end ranks take the in-place element pass, the middle ranks (two peers) the
    split-tile default -- every rank's rows bit-identical to the whole-grid assembly, two steps."""
    n = 4
    grid = H.Grid.structured(H.SIMPLEX, 3200 * n, 640, LOWER, (5.0 * n, 1.0), px=n, py=1)
    got, infos = run_device_ranks(grid, n, H.TENSOR_ISO_PER_ELEM, False, {"default": 0}, steps=2)
    assert [i.n_peers for i in infos] == [1, 2, 2, 1]
    ref = _single_gpu(grid, H.TENSOR_ISO_PER_ELEM, False)
    v = got["default"]
    assert v.shape == ref.shape and np.isfinite(v).all()
    assert np.array_equal(v.view(np.int64), ref.view(np.int64))


@pytest.mark.gpu
def test_device_transport_halo_geometry():
    """HDD_SHARD_HALO_GEOMETRY: the ghost coordinates travel too (element-major coords, no vertex arrays)."""
    grid, tk, two = _layout("c4_q1", 3)
    got, _ = run_device_ranks(grid, 3, tk, two, {"default": 0, "serial": H.SHARD_NO_OVERLAP}, steps=2,
                              flags_extra=H.SHARD_HALO_GEOMETRY)
    ref = _single_gpu(grid, tk, two)
    for name, v in got.items():
        assert np.array_equal(v.view(np.int64), ref.view(np.int64)), name


@pytest.mark.gpu
def test_device_transport_post_wait_and_mismatch():
    """hdd_comm_post / hdd_comm_wait on device buffers between two thread ranks (several rounds, the send buffer
    rewritten between them), then a size mismatch: both ranks return an error instead of hanging."""
    import torch
    hub = H.DeviceHub(2)
    comms = [H.Comm.device(hub, r, 0) for r in range(2)]
    src = [torch.arange(5000, dtype=torch.float64, device="cuda") + 1e4 * r for r in range(2)]
    dst = [torch.full((5000,), -1.0, dtype=torch.float64, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    errs, seen = [None, None], [[], []]

    def work(r, rounds, count):
        try:
            s = streams[r]
            for k in range(rounds):
                with torch.cuda.stream(s):
                    src[r].add_(1.0)          # rewrite the send buffer: must wait for the peer's copy
                comms[r].post([1 - r], [src[r][:count[r]]], [dst[r][:count[1 - r]]], stream=s.cuda_stream)
                comms[r].wait(stream=s.cuda_stream)
                with torch.cuda.stream(s):
                    seen[r].append(dst[r][:count[1 - r]].clone())
            s.synchronize()
        except Exception as e:   # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=work, args=(r, 4, [5000, 5000])) for r in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert errs == [None, None], errs
    for r in range(2):
        for k, got in enumerate(seen[r]):
            want = torch.arange(5000, dtype=torch.float64, device="cuda") + 1e4 * (1 - r) + (k + 1)
            assert torch.equal(got, want), (r, k)
    # rank 0 sends 100 doubles, rank 1 expects 200: a protocol error on both ranks
    th = [threading.Thread(target=work, args=(r, 1, [100, 100] if r == 0 else [100, 200])) for r in range(2)]
    errs[:] = [None, None]
    [t.start() for t in th]
    [t.join() for t in th]
    assert all(isinstance(e, H.HddError) for e in errs), errs
    torch.cuda.synchronize()
