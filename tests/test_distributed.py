"""Sharded (block-SWIPDG strip) assembly: world_size-2/3 process groups.

CPU (gloo): host-only C++ shards (hdd_shard_create without a context): exchanging a per-element field
through their halo plan fills every ghost column with the owner's value; the plans agree pairwise; the gloo
host transport of hdd_amd.halo (several messages per peer, one per halo row) delivers them in order.

GPU: two ranks share cuda:0 (the gloo host transport, since RCCL needs one GPU per rank); each runs the C++
sharded step (hdd_block_assemble_sharded: pack -> exchange straight into the ghost columns -> interior /
boundary tiles); ghost coefficients start as NaN and arrive only through the exchange; the concatenated rows
equal the oracle's global block-SWIPDG matrix.
"""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup_paths():
    for p in (os.path.join(ROOT, "dune-hdd_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


GRID = dict(nx=24, ny=8, lower=(0.0, 0.0), upper=(4.0, 1.0))


def _transport_worker(rank, world, port, outdir):
    """the gloo host transport with repeated peers: messages to one peer arrive in posting order"""
    _setup_paths()
    import torch.distributed as dist
    from hdd_amd.halo import gloo_host_comm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = gloo_host_comm(0)
    cb = comm._keep   # the ctypes callback the C++ step calls; drive the Python side directly
    peer = 1 - rank
    sends = [np.arange(n, dtype=np.float64) + 100 * rank + 10 * k for k, n in enumerate((3, 0, 5))]
    recvs = [np.empty(n) for n in (3, 0, 5)]
    import ctypes as C
    sp = (C.c_void_p * 3)(*[s_.ctypes.data if s_.size else None for s_ in sends])
    rp = (C.c_void_p * 3)(*[r_.ctypes.data if r_.size else None for r_ in recvs])
    cnt = (C.c_int64 * 3)(3, 0, 5)
    rc = cb(None, 3, (C.c_int32 * 3)(peer, peer, peer), sp, cnt, rp, cnt)
    ok = rc == 0 and all(np.array_equal(r_, np.arange(len(r_)) + 100 * peer + 10 * k) for k, r_ in enumerate(recvs))
    np.save(os.path.join(outdir, "ok_%d.npy" % rank), np.array([ok]))
    dist.destroy_process_group()


def test_gloo_host_transport_repeated_peers_cpu():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_transport_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        for r in range(2):
            assert np.load(os.path.join(d, "ok_%d.npy" % r))[0]


def _shard_worker(rank, world, port, outdir, case):
    """rank `rank` of a host-only C++ shard (hdd_shard_create with ctx NULL: the plan the sharded step of
    hdd_block_assemble_sharded moves its halo by) exchanges a per-element field over gloo exactly as the step
    does -- pack send_idx per peer, one message per peer in peer order, unpack into the ghost columns at
    recv_col0 -- and checks every ghost column against the owner's value."""
    _setup_paths()
    import torch
    import torch.distributed as dist

    import hdd_amd as H

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    et, nx, ny, px, py = SHARD_CASES[case]
    g = H.Grid.structured(et, nx, ny, (0.0, 0.0), (5.0, 1.0), px=px, py=py)
    sh = H.Shard(None, g, world, rank)
    gid = sh.global_ids()
    truth = np.sin(0.37 * gid) + 1e-3 * gid          # one distinct value per global element
    vals = truth.copy()
    vals[:sh.own_begin] = np.nan
    vals[sh.own_end:] = np.nan
    peers, sp, idx, rp, col0 = sh.halo_lists()
    ops, recvs = [], []
    for k, p in enumerate(peers):
        send = torch.from_numpy(np.ascontiguousarray(vals[idx[sp[k]:sp[k + 1]]]))
        recv = torch.empty(int(rp[k + 1] - rp[k]), dtype=torch.float64)
        recvs.append(recv)
        assert not torch.isnan(send).any(), "a send list names a ghost column"
        ops += [dist.P2POp(dist.isend, send, int(p)), dist.P2POp(dist.irecv, recv, int(p))]
    for r in (dist.batch_isend_irecv(ops) if ops else []):
        r.wait()
    for k in range(len(peers)):
        vals[col0[k]:col0[k] + len(recvs[k])] = recvs[k].numpy()
    tin, tbd = sh.tile_lists()
    plan = [rank, [int(p) for p in peers], [int(sp[k + 1] - sp[k]) for k in range(len(peers))],
            [int(rp[k + 1] - rp[k]) for k in range(len(peers))]]
    plans = [None] * world
    dist.all_gather_object(plans, plan)
    ok = bool(np.array_equal(vals, truth))
    tiles_ok = bool(np.array_equal(np.sort(np.concatenate([tin, tbd])), np.arange(sh.info.n_tiles)))
    np.save(os.path.join(outdir, "shard_%d.npy" % rank),
            np.array([ok, tiles_ok, sh.info.n_ghost > 0, len(tbd) > 0, len(peers)]))
    if rank == 0:   # the plans agree pairwise: r sends p what p expects from r
        cnt = {(r, p): (sn, rn) for r, ps, sns, rns in plans for p, sn, rn in zip(ps, sns, rns)}
        sym = all((p, r) in cnt and cnt[(r, p)][0] == cnt[(p, r)][1] for (r, p) in cnt)
        np.save(os.path.join(outdir, "sym.npy"), np.array([sym, len(cnt)]))
    dist.destroy_process_group()


SHARD_CASES = {
    # name: (element type, nx, ny, px, py) -- subdomain ids sx * py + sy, so contiguous ranges are columns
    "p1_strips": (0, 90, 12, 6, 1),
    "q1_blocks_2x2": (1, 48, 20, 4, 4),
}


@pytest.mark.parametrize("case,world", [("p1_strips", 2), ("p1_strips", 3), ("q1_blocks_2x2", 3)])
def test_gloo_shard_halo_plan_cpu(case, world):
    """The C++ shard's halo plan on CPU ranks (world_size 2 and 3: a middle rank has two peers; Q1 block
    subdomains): exchanging a field through it fills every ghost column with the owner's value, the plans
    agree pairwise (what r sends p is what p receives from r), and the tile lists partition the owned tiles."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_shard_worker, args=(world, _free_port(), d, case), nprocs=world, join=True)
        res = [np.load(os.path.join(d, "shard_%d.npy" % r)) for r in range(world)]
        sym, n_links = np.load(os.path.join(d, "sym.npy"))
    for r, (ok, tiles_ok, has_ghosts, has_bd, n_peers) in enumerate(res):
        assert ok and tiles_ok and has_ghosts and has_bd, (r, res[r])
    assert sym and n_links == 2 * (world - 1)
    if world == 3:
        assert res[1][4] == 2   # the middle rank talks to both neighbours


def test_host_only_shard_has_no_device_side():
    """A shard created without a context answers the plan queries but refuses the device entry points
    (hdd_shard_mesh / hdd_shard_pattern_fill / hdd_block_assemble_sharded) instead of handing out NULL arrays."""
    _setup_paths()
    import ctypes as C
    import hdd_amd as H
    g = H.Grid.structured(H.SIMPLEX, 40, 6, (0.0, 0.0), (5.0, 1.0), px=2, py=1)
    sh = H.Shard(None, g, 2, 1)
    peers, sp, idx, rp, col0 = sh.halo_lists()
    assert list(peers) == [0] and sp[-1] == len(idx) > 0 and rp[-1] == sh.info.n_ghost
    assert H.lib().hdd_shard_mesh(sh.h, C.byref(H.MeshT())) == 1    # HDD_ERR_INVALID


def test_halo_tile_split():
    """hdd_amd.halo_tiles: interior and boundary tiles partition the owned tiles; every element with a
    ghost face neighbour sits in a boundary tile, and no interior-tile element has one."""
    _setup_paths()
    import hdd_amd as H
    g = H.Grid.structured(H.SIMPLEX, 400, 4, (0, 0), (4, 1), px=4, py=1)
    for s0, s1 in [(0, 1), (1, 3), (3, 4), (0, 4)]:
        loc = g.local(s0, s1)
        t_in, t_bd = H.halo_tiles(loc)
        n_tiles = (loc.n_own + 63) // 64
        assert np.array_equal(np.sort(np.concatenate([t_in, t_bd])), np.arange(n_tiles))
        nb = loc.neighbors[:, loc.own_begin:loc.own_end]
        ghost_adj = ((nb >= 0) & ((nb < loc.own_begin) | (nb >= loc.own_end))).any(axis=0)
        tile_of = np.arange(loc.n_own) // 64
        assert np.isin(tile_of[ghost_adj], t_bd).all()
        assert not ghost_adj[np.isin(tile_of, t_in)].any()
        if (s0, s1) == (0, 4):
            assert len(t_bd) == 0
        else:
            assert 0 < len(t_bd) < n_tiles


def _gpu_worker(rank, world, port, outdir):
    _setup_paths()
    import torch
    import torch.distributed as dist

    import hdd_amd as H
    import oracle as O
    from hdd_amd.halo import gloo_host_comm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    perm = O.spe10_synthetic_permeability()
    g = H.Grid.structured(H.SIMPLEX, GRID["nx"], GRID["ny"], GRID["lower"], GRID["upper"], px=world * 2, py=1)
    ctx = H.Context(0)
    sh = H.Shard(ctx, g, world, rank)
    kcell = sh.checkerboard(GRID["lower"], GRID["upper"], 100, 20, perm)
    kcell[:sh.own_begin] = np.nan          # ghost coefficients arrive only through the exchange
    kcell[sh.own_end:] = np.nan
    kdev = torch.from_numpy(kcell).cuda()
    _, _, _, pat = sh.pattern(ctx, 0)
    comm = gloo_host_comm(0)
    kap, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=kdev)
    val = torch.full((sh.info.nnz,), float("nan"), dtype=torch.float64, device="cuda")
    H.assemble_sharded(ctx, sh, comm, kap, ten, pat, [val])   # overlapped: interior tiles, halo, boundary tiles
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, "val_%d.npy" % rank), val.cpu().numpy())
    np.save(os.path.join(outdir, "rng_%d.npy" % rank), np.array(g.subdomain_range(sh.info.s_begin, sh.info.s_end)))
    np.save(os.path.join(outdir, "ghost_%d.npy" % rank), kdev.cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_one_gpu_match_global_oracle():
    import torch.multiprocessing as mp
    _setup_paths()
    import hdd_amd as H
    import oracle as O
    from cases import compare_rows

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gpu_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        vals = [np.load(os.path.join(d, "val_%d.npy" % r)) for r in range(2)]
        rngs = [np.load(os.path.join(d, "rng_%d.npy" % r)) for r in range(2)]
        ghosts = [np.load(os.path.join(d, "ghost_%d.npy" % r)) for r in range(2)]
    assert all(np.isfinite(gh).all() for gh in ghosts)   # every ghost column was received
    g = H.Grid.structured(H.SIMPLEX, GRID["nx"], GRID["ny"], GRID["lower"], GRID["upper"], px=4, py=1)
    pc, pev, psd = g.connectivity()
    ot, oc, oev = O.kuhn_grid(GRID["nx"], GRID["ny"], GRID["lower"], GRID["upper"])
    key = {tuple(r): i for i, r in enumerate(oev)}
    permu = np.array([key[tuple(r)] for r in pev])
    sub = np.empty(g.ne, np.int32)
    sub[permu] = psd
    perm = O.spe10_synthetic_permeability()
    k = O.checkerboard(O.element_centers(oc, oev), GRID["lower"], GRID["upper"], 100, 20, perm)
    og = O.Grid(ot, oc, oev)
    ei, rp, col, oval = O.assemble_block(og, sub, 4, O.scalar(O.FN_CONST, 1.0),
                                         O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k), O.params())
    assert rngs[0][0] == 0 and rngs[0][1] == rngs[1][0] and rngs[1][1] == g.ne
    got = np.concatenate(vals)
    worst, ok = compare_rows(rp, got, oval, 1e-12)
    assert ok, worst
