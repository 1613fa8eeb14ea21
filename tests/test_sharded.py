"""The sharded BlockSWIPDG step behind the C ABI (hdd_shard_* / hdd_comm_* / hdd_block_assemble_sharded).

Reference semantics: block-swipdg.hh:355-382 (the owner of ss writes A_ss and A_ss,nn), 1136-1179 (boundary),
1270-1326 (coupling).  Each rank evaluates only its OWNED per-element coefficients; the ghost columns start as
NaN and are filled by the face halo inside the C++ step, so a missing or misrouted halo record shows up as a
NaN / wrong entry.  Checks:
  * 2 ranks on one GPU (processes, gloo host transport driven from C++ through the hdd_comm callback): the
    concatenated rows equal the single-GPU assembly of the same block grid bit for bit, and the oracle's
    block-SWIPDG matrix at 1e-12 -- overlapped (interior tiles during the exchange) and serial, with and
    without the geometry in the halo, P1 and Q1, isotropic and symmetric per-element tensors, two
    diffusion-factor components;
  * RCCL: a one-rank communicator exchanging with itself (ncclGroupStart / ncclSend / ncclRecv /
    ncclGroupEnd on the transfer stream, the stream-ordered wait), and the C++ example in RCCL mode;
  * the C++ example driving 3 thread ranks through ShardedBlockSWIPDG with an in-process mailbox transport.
"""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HDD_EXAMPLES_BIN: another build of the examples, e.g. examples/bin_asan (make -C dune-hdd_amd asan)
EXAMPLE = os.path.join(os.environ.get("HDD_EXAMPLES_BIN") or os.path.join(ROOT, "examples", "bin"), "sharded_main")


def _paths():
    for p in (os.path.join(ROOT, "dune-hdd_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


_paths()
import hdd_amd as H  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_unique_id_resolves_librccl():
    """The library finds RCCL at run time (PyTorch's copy through its rpath) and returns a 128-byte id.  In a
    child process: ncclGetUniqueId starts the bootstrap root thread, which waits for ranks that this test
    never creates."""
    code = ("import sys; sys.path.insert(0, %r); import hdd_amd as H; u = H.Comm.rccl_unique_id(); "
            "print(len(u), int(any(u)))" % os.path.join(ROOT, "dune-hdd_amd", "python"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == [str(H.RCCL_ID_BYTES), "1"], r.stdout


LOWER, UPPER = (0.0, 0.0), (5.0, 1.0)
CASES = {
    # name: (elem type, nx, ny, px, py, tensor kind, flags, two components)
    "p1_iso_overlap": (H.SIMPLEX, 40, 10, 4, 1, H.TENSOR_ISO_PER_ELEM, 0, False),
    "p1_iso_serial_geometry": (H.SIMPLEX, 40, 10, 4, 1, H.TENSOR_ISO_PER_ELEM,
                               H.SHARD_NO_OVERLAP | H.SHARD_HALO_GEOMETRY, False),
    "p1_sym_two_comp": (H.SIMPLEX, 36, 12, 4, 2, H.TENSOR_SYM_PER_ELEM, 0, True),
    "q1_iso_overlap_2x2": (H.CUBE, 44, 15, 4, 2, H.TENSOR_ISO_PER_ELEM, 0, True),
    "q1_iso_split_tiles": (H.CUBE, 44, 15, 4, 2, H.TENSOR_ISO_PER_ELEM, H.SHARD_SPLIT_TILES, True),
    # default overlap = the fixup on the side stream into a side buffer + the copy kernel; FIX_INLINE = round 2's
    "q1_iso_fix_inline": (H.CUBE, 44, 15, 4, 2, H.TENSOR_ISO_PER_ELEM, H.SHARD_FIX_INLINE, True),
    "p1_sym_fix_inline": (H.SIMPLEX, 36, 12, 4, 2, H.TENSOR_SYM_PER_ELEM, H.SHARD_FIX_INLINE, False),
    "q1_sym_fix_scatter": (H.CUBE, 44, 15, 4, 2, H.TENSOR_SYM_PER_ELEM, H.SHARD_FIX_SCATTER, True),
    "p1_iso_fix_inplace": (H.SIMPLEX, 40, 10, 4, 1, H.TENSOR_ISO_PER_ELEM, H.SHARD_FIX_INPLACE, False),
}


def _coefficients(centers, owned):
    """per-element data of the test (a function of the barycentre, so every rank computes its own owned part):
    isotropic checkerboard-like tensor, symmetric SPD tensor rows, and a per-element diffusion factor."""
    x, y = centers
    iso = 10.0 ** (3.0 * np.sin(3.1 * x) * np.cos(2.3 * y))
    sym = np.stack([1.5 + np.sin(x) ** 2, 0.3 * np.cos(2 * x + y), 1.2 + np.cos(y) ** 2])
    kap = 1.0 + 0.5 * np.sin(5 * x + 3 * y) ** 2
    for a in (iso, sym, kap):
        a[..., ~owned] = np.nan
    return iso, sym, kap


def _worker(rank, world, port, outdir, case):
    _paths()
    import torch
    import torch.distributed as dist

    import hdd_amd as H
    from hdd_amd.halo import gloo_host_comm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    et, nx, ny, px, py, tk, flags, two = CASES[case]
    grid = H.Grid.structured(et, nx, ny, LOWER, UPPER, px=px, py=py)
    ctx = H.Context(0)
    sh = H.Shard(ctx, grid, world, rank)
    owned = np.zeros(sh.n_local, bool)
    owned[sh.own_begin:sh.own_end] = True
    iso, sym, kap = _coefficients(sh.centers(), owned)
    t_iso = torch.from_numpy(iso).cuda()
    t_sym = torch.from_numpy(np.ascontiguousarray(sym)).cuda()
    t_kap = torch.from_numpy(kap).cuda()
    tensor = H.tensor_fn(tk, per_elem=t_iso if tk == H.TENSOR_ISO_PER_ELEM else t_sym)
    kappas = [H.scalar_fn(H.FN_CONST, 1.0)] + ([H.scalar_fn(H.FN_PER_ELEM, per_elem=t_kap)] if two else [])
    _, _, _, pat = p = sh.pattern(ctx)
    vals = [torch.full((sh.info.nnz,), float("nan"), dtype=torch.float64, device="cuda") for _ in kappas]
    comm = gloo_host_comm(0)
    for _ in range(2):   # two steps: the second re-sends the (now complete) records
        H.assemble_sharded(ctx, sh, comm, kappas, tensor, pat, vals, flags=flags)
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, "val_%d.npy" % rank), np.stack([v.cpu().numpy() for v in vals]))
    np.save(os.path.join(outdir, "info_%d.npy" % rank),
            np.array([sh.info.global_first, sh.n_own, sh.info.n_peers, sh.info.halo_recv]))
    del comm
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_two_ranks_sharded_equals_single_gpu(case):
    import torch
    import torch.multiprocessing as mp
    import oracle as O
    from cases import compare_rows

    et, nx, ny, px, py, tk, flags, two = CASES[case]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, case), nprocs=2, join=True)
        vals = [np.load(os.path.join(d, "val_%d.npy" % r)) for r in range(2)]
        info = [np.load(os.path.join(d, "info_%d.npy" % r)) for r in range(2)]
    assert all(i[2] == 1 and i[3] > 0 for i in info), info          # one peer each, ghosts received
    got = np.concatenate(vals, axis=1)
    assert np.isfinite(got).all(), "a ghost column was not filled by the halo"
    # single-GPU assembly of the same block grid (every subdomain local, no halo)
    grid = H.Grid.structured(et, nx, ny, LOWER, UPPER, px=px, py=py)
    loc = grid.local()
    iso, sym, kap = _coefficients(loc.centers(), np.ones(loc.n_local, bool))
    ctx = H.Context(0)
    dm, dp = H.DeviceMesh(loc, 0), H.DevicePattern(loc, 0)
    tensor = H.tensor_fn(tk, per_elem=torch.from_numpy(iso if tk == H.TENSOR_ISO_PER_ELEM else
                                                        np.ascontiguousarray(sym)).cuda())
    kappas = [H.scalar_fn(H.FN_CONST, 1.0)] + ([H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(kap).cuda())]
                                               if two else [])
    ref = np.stack([v.cpu().numpy() for v in H.assemble(ctx, dm, dp, kappas, tensor)])
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), "sharded != single-GPU (bitwise)"
    if et == H.SIMPLEX and tk == H.TENSOR_ISO_PER_ELEM:   # and the oracle's block restatement
        pc, pev, psd = grid.connectivity()
        og = O.Grid(O.SIMPLEX, pc, pev)
        k_or = iso[np.argsort(loc.global_id)]
        rp, col, oval = O.assemble(og, O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k_or),
                                   O.params())
        assert np.array_equal(col, dp.host[1])
        worst, ok = compare_rows(rp, got[0], oval, 1e-12)
        assert ok, worst


@pytest.mark.gpu
def test_single_rank_shard_equals_assemble():
    """nranks = 1: no peers, no communicator -- the sharded entry is one full assembly (C2 mesh class)."""
    import torch
    grid = H.Grid.structured(H.SIMPLEX, 64, 16, LOWER, UPPER)
    ctx = H.Context(0)
    sh = H.Shard(ctx, grid, 1, 0)
    assert sh.info.n_peers == 0 and sh.info.n_ghost == 0 and sh.info.n_tiles_boundary == 0
    k = sh.checkerboard(LOWER, UPPER, 100, 20, np.linspace(0.5, 3.0, 2000))
    tensor = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(k).cuda())
    _, col, _, pat = sh.pattern(ctx)
    v = [torch.empty(sh.info.nnz, dtype=torch.float64, device="cuda")]
    H.assemble_sharded(ctx, sh, None, [H.scalar_fn(H.FN_CONST, 1.0)], tensor, pat, v)
    loc = grid.local()
    ref = H.assemble(ctx, H.DeviceMesh(loc, 0), H.DevicePattern(loc, 0), [H.scalar_fn(H.FN_CONST, 1.0)], tensor)
    torch.cuda.synchronize()
    assert np.array_equal(col.cpu().numpy(), loc.pattern()[1])
    assert np.array_equal(v[0].cpu().numpy(), ref[0].cpu().numpy())


@pytest.mark.gpu
def test_rccl_self_exchange():
    """A 1-rank RCCL communicator sending to itself: the group send/recv on the transfer stream and the
    stream-ordered wait deliver the message (the 8-GPU path uses exactly these calls)."""
    import torch
    comm = H.Comm.rccl(H.Comm.rccl_unique_id(), 1, 0, 0)
    a = torch.arange(1000, dtype=torch.float64, device="cuda") * 0.5
    b = torch.full((1000,), -1.0, dtype=torch.float64, device="cuda")
    for _ in range(3):
        comm.post([0], [a], [b])
        comm.wait()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    # hdd_comm_post_direct (the serial sharded step's form): the group on the caller's stream, wait a no-op there;
    # a kernel enqueued right after it on that stream sees the received values
    s = torch.cuda.Stream()
    c = torch.full((1000,), -1.0, dtype=torch.float64, device="cuda")
    with torch.cuda.stream(s):
        for k in range(3):
            a.add_(1.0)
            comm.post([0], [a], [c], stream=s.cuda_stream, direct=True)
            comm.wait(stream=s.cuda_stream)
            d = c * 2.0
    torch.cuda.synchronize()
    assert torch.equal(c, a) and torch.equal(d, a * 2.0)
    del comm


@pytest.mark.gpu
def test_cpp_example_thread_ranks():
    """examples/sharded_main threads 3: ShardedBlockSWIPDG on 3 thread ranks (in-process mailbox transport)
    == single-GPU BlockSWIPDG bit for bit, P1 and Q1, parametric SPE10 structure (2 components), and diffusion-
    factor parts of different integration orders (per-element affine part + sinusoid component: one sharded
    call per order, the second without a halo exchange)."""
    r = subprocess.run([EXAMPLE, "threads", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sharded threads ok" in r.stdout, r.stdout
    assert r.stdout.count("mismatches vs single-GPU BlockSWIPDG: 0") == 4, r.stdout


@pytest.mark.gpu
def test_cpp_example_device_transport_threads():
    """examples/sharded_main device 3: the same thread ranks through Parallel::Communicator::device (the
    in-process device transport), i.e. the step's RCCL branch -- transfer stream, fixup on it, event join --
    with a middle rank, three steps each, bit for bit == single-GPU BlockSWIPDG."""
    r = subprocess.run([EXAMPLE, "device", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sharded device-transport threads ok" in r.stdout, r.stdout
    assert r.stdout.count("mismatches vs single-GPU BlockSWIPDG: 0") == 4, r.stdout


@pytest.mark.gpu
def test_cpp_example_rccl_one_rank():
    """examples/sharded_main rccl: the RCCL communicator created from C++ (unique id through a file)."""
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([EXAMPLE, "rccl", os.path.join(d, "id"), "0", "1", "0"], capture_output=True, text=True,
                           timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rccl rank 0/1" in r.stdout and "NON-FINITE" not in r.stdout


@pytest.mark.gpu
def test_no_transfer_flag_keeps_interior_rows():
    """HDD_SHARD_NO_TRANSFER (timing studies): rank 0 of 2 runs every launch of the overlapped step without a
    communicator; the ghost columns then hold the rank's own send buffer (wrong values by design), so exactly
    the rows of elements without a ghost neighbour must equal the single-GPU assembly, bit for bit.  Without
    the flag a NULL communicator is an error."""
    import torch
    grid = H.Grid.structured(H.SIMPLEX, 96, 20, LOWER, UPPER, px=2, py=1)
    ctx = H.Context(0)
    sh = H.Shard(ctx, grid, 2, 0)
    assert sh.info.n_peers == 1 and sh.info.n_tiles_boundary > 0
    k = sh.checkerboard(LOWER, UPPER, 100, 20, np.linspace(0.5, 3.0, 2000))
    tensor = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(k).cuda())
    kap = [H.scalar_fn(H.FN_CONST, 1.0)]
    rp, col, ep, pat = sh.pattern(ctx)
    v = [torch.full((sh.info.nnz,), float("nan"), dtype=torch.float64, device="cuda")]
    with pytest.raises(H.HddError):
        H.assemble_sharded(ctx, sh, None, kap, tensor, pat, v)
    H.assemble_sharded(ctx, sh, None, kap, tensor, pat, v, flags=H.SHARD_NO_TRANSFER)
    loc = grid.local()
    ref = H.assemble(ctx, H.DeviceMesh(loc, 0), H.DevicePattern(loc, 0), kap,
                     H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(
                         loc.checkerboard(LOWER, UPPER, 100, 20, np.linspace(0.5, 3.0, 2000))).cuda()))[0]
    torch.cuda.synchronize()
    got, want = v[0].cpu().numpy(), ref.cpu().numpy()[:sh.info.nnz]
    colv, epv = col.cpu().numpy(), ep.cpu().numpy()
    g0, g1 = sh.info.global_first, sh.info.global_first + sh.n_own   # owned global element ids
    touches = np.zeros(sh.n_own, bool)
    for e in range(sh.n_own):   # an owned element's row block references a ghost (non-owned) column block
        g = colv[epv[e]:epv[e + 1]] // sh.nb
        touches[e] = bool(((g < g0) | (g >= g1)).any())
    assert touches.any() and not touches.all()
    for e in np.flatnonzero(~touches)[:: 7]:
        assert np.array_equal(got[epv[e]:epv[e + 1]], want[epv[e]:epv[e + 1]]), e
    # the same (loopback) ghost values through the three step schedules: off-stream fixup + copy kernel
    # (default), fixup on the stream after the join (FIX_INLINE), exchange first (NO_OVERLAP) -- bit for bit
    for fl in (H.SHARD_FIX_INLINE, H.SHARD_FIX_SCATTER, H.SHARD_FIX_INPLACE, H.SHARD_NO_OVERLAP):
        w = [torch.full((sh.info.nnz,), float("nan"), dtype=torch.float64, device="cuda")]
        H.assemble_sharded(ctx, sh, None, kap, tensor, pat, w, flags=H.SHARD_NO_TRANSFER | fl)
        torch.cuda.synchronize()
        assert np.array_equal(w[0].cpu().numpy().view(np.int64), got.view(np.int64)), fl
