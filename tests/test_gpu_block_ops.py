"""Device block operators (BlockSWIPDG::get_local_operator / get_coupling_operator, block-swipdg.hh:625-676):
hdd_block_operator_map_device + hdd_block_operator_values_device against the host map of round 2
(hdd_block_operator_map + hdd_gather_values), entry for entry, for every (ss, nn) operator of P1 / Q1 block
grids with ragged subdomains and of a Q_p hexahedral grid; the nnz predicted from the mesh alone
(block_operator_nnz, used to stay asynchronous) equals the counted one."""
import numpy as np
import pytest

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu


def _host_map(grid, rp, col, ss, nn):
    c = H.C.c_int64()
    H._check(H.lib().hdd_block_operator_map(grid.h, ss, nn, H._p(rp), H._p(col), None, None, None, H.C.byref(c)))
    a, b = grid.subdomain_range(ss, ss + 1)
    orp = np.empty((b - a) * grid.nb + 1, np.int64)
    ocol = np.empty(c.value, np.int32)
    src = np.empty(c.value, np.int64)
    H._check(H.lib().hdd_block_operator_map(grid.h, ss, nn, H._p(rp), H._p(col), H._p(orp), H._p(ocol), H._p(src),
                                            H.C.byref(c)))
    return orp, ocol, src


def _check_batched(ctx, grid, dp, vals, expect):
    """hdd_block_operators_*: every operator of `expect` ({(ss, nn): (orp, ocol, src)}) in one batched call, in
    a shuffled order, with and without the mesh-predicted counts"""
    import torch
    pairs = list(expect)
    np.random.default_rng(7).shuffle(pairs)
    nnz_of = H.block_operator_nnz(grid.local())
    for known in (True, False):
        got = H.block_operators(ctx, grid, dp, vals, pairs, nnz=nnz_of if known else None)
        torch.cuda.synchronize()
        assert list(got) == pairs
        for p, (drp, dcol, dvals) in got.items():
            orp, ocol, src = expect[p]
            assert np.array_equal(drp.cpu().numpy(), orp), p
            assert np.array_equal(dcol.cpu().numpy(), ocol), p
            for v, dv in zip(vals, dvals):
                assert np.array_equal(dv.cpu().numpy(), v.cpu().numpy()[src]), p


def _check_all(ctx, grid, n_comp=2):
    import torch
    loc = grid.local()
    dp = H.DevicePattern(loc)
    rp, col, _ = dp.host
    rng = np.random.default_rng(4)
    vals = [torch.from_numpy(rng.standard_normal(dp.nnz)).cuda() for _ in range(n_comp)]
    nnz_of = H.block_operator_nnz(loc)
    n_ops = 0
    expect = {}
    for ss in range(grid.n_sub):
        for nn in range(grid.n_sub):
            orp, ocol, src = _host_map(grid, rp, col, ss, nn)
            if nn != ss and ocol.size == 0:
                assert (ss, nn) not in nnz_of
                continue
            assert nnz_of[(ss, nn)] == ocol.size
            expect[(ss, nn)] = (orp, ocol, src)
            for known in (True, False):
                drp, dcol, dvals = H.block_operator(ctx, grid, dp, vals, ss, nn,
                                                    nnz=nnz_of[(ss, nn)] if known else None)
                torch.cuda.synchronize()
                assert np.array_equal(drp.cpu().numpy(), orp)
                assert np.array_equal(dcol.cpu().numpy(), ocol)
                for v, dv in zip(vals, dvals):
                    assert np.array_equal(dv.cpu().numpy(), v.cpu().numpy()[src])
            n_ops += 1
    _check_batched(ctx, grid, dp, vals, expect)
    return n_ops


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_device_block_operators_2d(ctx, et):
    grid = H.Grid.structured(et, 53, 29, (0, 0), (5, 1), px=4, py=3)
    n_ops = _check_all(ctx, grid)
    assert n_ops == 12 + 2 * (3 * 3 + 4 * 2)   # local + both directions of every subdomain face


def test_device_block_operators_hex(ctx):
    grid = H.Grid.structured3d((5, 4, 3), (0, 0, 0), (1, 1, 1), p=(2, 2, 1), degree=2)
    assert _check_all(ctx, grid, n_comp=1) == 4 + 2 * 4


def test_device_block_operators_batched_c4_layout(ctx):
    """all operators of an 8 x 8 Q1 block grid (C4's decomposition, 288 operators) in one batched call; the
    concatenated arrays against the per-operator calls"""
    import torch
    grid = H.Grid.structured(H.CUBE, 88, 40, (0, 0), (5, 1), px=8, py=8)
    loc = grid.local()
    dp = H.DevicePattern(loc)
    nnz_of = H.block_operator_nnz(loc)
    assert len(nnz_of) == 288
    vals = [torch.from_numpy(np.random.default_rng(5).standard_normal(dp.nnz)).cuda()]
    got = H.block_operators(ctx, grid, dp, vals, sorted(nnz_of), nnz=nnz_of)
    for (ss, nn), (drp, dcol, dv) in got.items():
        rp, col, v = H.block_operator(ctx, grid, dp, vals, ss, nn, nnz=nnz_of[(ss, nn)])
        assert torch.equal(drp, rp) and torch.equal(dcol, col) and torch.equal(dv[0], v[0])


def test_device_block_operators_batched_errors(ctx):
    grid = H.Grid.structured(H.CUBE, 8, 6, (0, 0), (1, 1), px=2, py=1)
    dp = H.DevicePattern(grid.local())
    rng = (H.C.c_int64 * 4)(0, 4, 0, 8)
    out = __import__("torch").empty(10, dtype=__import__("torch").int64, device="cuda")
    assert H.lib().hdd_block_operators_map_device(ctx.h, H.C.byref(dp.t), 0, rng, out.data_ptr(), None, None, None,
                                                  None) == 1   # HDD_ERR_INVALID: no operators
    bad = (H.C.c_int64 * 4)(0, dp.t.n_rows + 1, 0, 8)
    assert H.lib().hdd_block_operators_map_device(ctx.h, H.C.byref(dp.t), 1, bad, out.data_ptr(), None, None, None,
                                                  None) == 5   # HDD_ERR_RANGE


def test_device_block_operator_map_ranges(ctx):
    import torch
    grid = H.Grid.structured(H.CUBE, 8, 6, (0, 0), (1, 1), px=2, py=1)
    loc = grid.local()
    dp = H.DevicePattern(loc)
    out = torch.empty(10, dtype=torch.int64, device="cuda")
    n = H.C.c_int64()
    for r0, r1, c0, c1 in [(-1, 4, 0, 8), (0, dp.t.n_rows + 1, 0, 8), (5, 4, 0, 8), (0, 4, 9, 8)]:
        rc = H.lib().hdd_block_operator_map_device(ctx.h, H.C.byref(dp.t), r0, r1, c0, c1, out.data_ptr(), None, None,
                                                   H.C.byref(n), None)
        assert rc == 5   # HDD_ERR_RANGE
