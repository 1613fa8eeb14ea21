"""GPU parity of the Q_p hexahedral path (C5: ESV2007 3d structured, SWIPDG p=3; hex_qp.hip, MFMA f64)
against the Q_p oracle (oracle/swipdg_oracle_qp.c), entry-wise, through the C ABI.

Tolerance (fp64): per row, max_j |a_gpu - a_oracle| <= 1e-12 * max_j |a_oracle| (MFMA accumulation order
differs from the oracle's quadrature loop).  Also: the device pattern build equals the host pattern."""
import numpy as np
import pytest

import oracle as O
from cases import compare_rows
from hex_tools import lex_to_product

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu

RTOL = 1e-12
LO, UP = (-1.0, 0.0, 0.5), (1.0, 1.5, 2.0)


def _torch():
    import torch
    return torch


def _setup(n, parts, deg, boundary=H.BOUNDARY_ALL_DIRICHLET):
    g = H.Grid.structured3d(n, LO, UP, p=parts, degree=deg, boundary=boundary)
    ei = lex_to_product(g, n, LO, UP)
    q = O.QpGrid(3, deg, n, LO, UP)
    return g, ei, q


def _spd_tensors(ne, seed):
    rng = np.random.default_rng(seed)
    d = rng.uniform(0.5, 3.0, (ne, 3))
    o = rng.uniform(-0.2, 0.2, (ne, 3))
    return np.stack([d[:, 0], o[:, 0], o[:, 1], d[:, 1], o[:, 2], d[:, 2]], 1)   # xx xy xz yy yz zz


@pytest.mark.parametrize("deg", [1, 2, 3])
@pytest.mark.parametrize("n,parts", [((3, 4, 5), (1, 1, 1)), ((4, 3, 3), (2, 1, 1))])
def test_hex_const_coefficients(ctx, deg, n, parts):
    g, ei, q = _setup(n, parts, deg)
    loc = g.local()
    dm = H.DeviceMesh(loc)
    dp = H.DevicePattern(loc)
    (val,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(dim=3), H.params_for(deg, 3))
    _torch().cuda.synchronize()
    rp, col, _ = dp.host
    orp, ocol, oval = O.qp_assemble(q, O.scalar(), O.qp_tensor(), O.qp_params(q), elem_index=ei)
    assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val.cpu().numpy(), oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("deg", [1, 2, 3])
def test_hex_smooth_kappa_sym_tensor(ctx, deg):
    """sinusoid kappa (integration order 3 -> one more Gauss point per direction) and a symmetric
    per-element tensor; per-element kappa component on the same mesh."""
    torch = _torch()
    n = (3, 3, 4)
    g, ei, q = _setup(n, (1, 1, 1), deg)
    loc = g.local()
    dm = H.DeviceMesh(loc)
    dp = H.DevicePattern(loc)
    T = _spd_tensors(g.ne, 7)                  # product element order
    Tdev = torch.from_numpy(np.ascontiguousarray(T.T)).cuda()
    kel = np.random.default_rng(8).uniform(0.2, 4.0, g.ne)
    kdev = torch.from_numpy(kel).cuda()
    inv = np.empty(g.ne, np.int64)
    inv[ei] = np.arange(g.ne)
    To = np.ascontiguousarray(T[ei])           # oracle (lexicographic) element order
    ten = H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=Tdev, dim=3)
    oten = O.qp_tensor(O.TENSOR_SYM_PER_ELEM, per_elem=To)
    for kap, okap in [
        (H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=3.0, ky=2.0, order=3),
         O.scalar(O.FN_SINUSOID, 1.0, 0.5, 3.0, 2.0, order=3)),
        (H.scalar_fn(H.FN_PER_ELEM, per_elem=kdev), O.scalar(O.FN_PER_ELEM, per_elem=np.ascontiguousarray(kel[ei]))),
    ]:
        (val,) = H.assemble(ctx, dm, dp, [kap], ten, H.params_for(deg, 3))
        torch.cuda.synchronize()
        rp = dp.host[0]
        _, _, oval = O.qp_assemble(q, okap, oten, O.qp_params(q), elem_index=ei)
        worst, ok = compare_rows(rp, val.cpu().numpy(), oval, RTOL)
        assert ok, worst


@pytest.mark.parametrize("deg", [2, 3])
def test_hex_neumann_boundary(ctx, deg):
    g, ei, q = _setup((3, 3, 3), (1, 1, 1), deg, boundary=H.BOUNDARY_ALL_NEUMANN)
    loc = g.local()
    dm = H.DeviceMesh(loc)
    dp = H.DevicePattern(loc)
    (val,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 2.0)], H.tensor_fn(dim=3), H.params_for(deg, 3))
    _torch().cuda.synchronize()
    prm = O.qp_params(q, boundary=O.BOUNDARY_NEUMANN)
    _, _, oval = O.qp_assemble(q, O.scalar(O.FN_CONST, 2.0), O.qp_tensor(), prm, elem_index=ei)
    worst, ok = compare_rows(dp.host[0], val.cpu().numpy(), oval, RTOL)
    assert ok, worst


def test_hex_q3_gemm_equals_register_kernel():
    """p = 3 with per-element data: the reference-matrix GEMM kernel (hex_q3g_kernel, default) against the
    register-fragment MFMA kernel (HDD_VARIANT_HEX_Q3_REGISTER) on 10 x 9 x 7 elements in 2 slabs (ragged last
    16-element group, every workgroup walking several groups, Dirichlet faces), both through the C ABI; and the
    oracle on the same input at the parity tolerance."""
    import os
    torch = _torch()
    deg, n = 3, (10, 9, 7)
    g, ei, q = _setup(n, (2, 1, 1), deg)
    loc = g.local()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    T = _spd_tensors(g.ne, 11)
    kel = np.random.default_rng(12).uniform(0.2, 4.0, g.ne)
    ten = H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=torch.from_numpy(np.ascontiguousarray(T.T)).cuda(), dim=3)
    kap = H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(kel).cuda())
    vals = []
    for variant in (0, H.VARIANT_HEX_Q3_REGISTER):
        c = H.Context(0)
        c.set_variant(variant)
        (v,) = H.assemble(c, dm, dp, [kap], ten, H.params_for(deg, 3))
        torch.cuda.synchronize()
        vals.append(v.cpu().numpy())
        del c
    rp = dp.host[0]
    worst, ok = compare_rows(rp, vals[0], vals[1], RTOL)
    assert ok, worst
    _, _, oval = O.qp_assemble(q, O.scalar(O.FN_PER_ELEM, per_elem=np.ascontiguousarray(kel[ei])),
                               O.qp_tensor(O.TENSOR_SYM_PER_ELEM, per_elem=np.ascontiguousarray(T[ei])),
                               O.qp_params(q), elem_index=ei)
    worst, ok = compare_rows(rp, vals[0], oval, RTOL)
    assert ok, worst


def test_hex_rank_local_slab_equals_global_slice(ctx):
    deg = 3
    g = H.Grid.structured3d((6, 3, 2), LO, UP, p=(3, 1, 1), degree=deg)
    full = g.local()
    dpg = H.DevicePattern(full)
    (gval,) = H.assemble(ctx, H.DeviceMesh(full), dpg, [H.scalar_fn()], H.tensor_fn(dim=3), H.params_for(deg, 3))
    loc = g.local(1, 2)
    dp = H.DevicePattern(loc)
    (val,) = H.assemble(ctx, H.DeviceMesh(loc), dp, [H.scalar_fn()], H.tensor_fn(dim=3), H.params_for(deg, 3))
    _torch().cuda.synchronize()
    a, b = g.subdomain_range(1, 2)
    grp = dpg.host[0]
    lo, hi = grp[a * g.nb], grp[b * g.nb]
    assert np.array_equal(dp.host[1], dpg.host[1][lo:hi])
    gv = gval.cpu().numpy()
    assert np.array_equal(val.cpu().numpy(), gv[lo:hi])


@pytest.mark.parametrize("kind", ["hex3", "simplex", "cube"])
def test_device_pattern_equals_host(ctx, kind):
    torch = _torch()
    if kind == "hex3":
        g = H.Grid.structured3d((5, 4, 3), p=(2, 1, 1), degree=3)
        s0, s1 = 1, 2
    else:
        g = H.Grid.structured(H.SIMPLEX if kind == "simplex" else H.CUBE, 12, 5, px=3, py=2)
        s0, s1 = 1, 4
    loc = g.local(s0, s1)
    host = loc.pattern()
    dpat = H.DevicePattern(loc, ctx=ctx, on_device=True)
    torch.cuda.synchronize()
    assert dpat.nnz == host[1].shape[0]
    assert np.array_equal(dpat.row_ptr.cpu().numpy(), host[0])
    assert np.array_equal(dpat.col.cpu().numpy(), host[1])
    assert np.array_equal(dpat.elem_ptr.cpu().numpy(), host[2])


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_device_pattern_tiles_equal_host(ctx, et):
    """The tiled P1/Q1 device pattern builder over many 64-element tiles (ragged last tile, ghosts,
    block numbering through global ids) equals the host pattern."""
    torch = _torch()
    g = H.Grid.structured(et, 203, 41, px=4, py=3)
    loc = g.local(2, 9)
    host = loc.pattern()
    dpat = H.DevicePattern(loc, ctx=ctx, on_device=True)
    torch.cuda.synchronize()
    assert loc.n_own % 64 != 0
    assert dpat.nnz == host[1].shape[0]
    assert np.array_equal(dpat.row_ptr.cpu().numpy(), host[0])
    assert np.array_equal(dpat.col.cpu().numpy(), host[1])
    assert np.array_equal(dpat.elem_ptr.cpu().numpy(), host[2])


@pytest.mark.parametrize("et,px", [(H.SIMPLEX, 1), (H.CUBE, 1), (H.SIMPLEX, 3)])
def test_device_pattern_uniform_tiles_equal_host(ctx, et, px):
    """Large single- and multi-subdomain meshes, where most tiles are uniform (every element with all faces
    interior: the 16-byte staged path of pattern_fill_tile_kernel) next to boundary tiles, with and without
    global ids (a rank-local slice maps local to global ids through the gid gathers)."""
    torch = _torch()
    g = H.Grid.structured(et, 400, 83, px=px, py=1)
    for s0, s1 in ((0, px), (px - 1, px)):
        loc = g.local(s0, s1)
        host = loc.pattern()
        dpat = H.DevicePattern(loc, ctx=ctx, on_device=True)
        torch.cuda.synchronize()
        assert dpat.nnz == host[1].shape[0]
        assert np.array_equal(dpat.row_ptr.cpu().numpy(), host[0])
        assert np.array_equal(dpat.col.cpu().numpy(), host[1])
        assert np.array_equal(dpat.elem_ptr.cpu().numpy(), host[2])


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_device_elem_ptr_block_sums_equal_scan(et):
    """elem_ptr with per-block offset sums (no scan launch, > 768 blocks: the unrolled loads) and nnz through the
    mapped host word equal the scan-launch + copy scheme (HDD_VARIANT_PATTERN_SCAN_COPY), pattern included."""
    import os
    torch = _torch()
    ctxs = []
    for variant in (0, H.VARIANT_PATTERN_SCAN_COPY):
        ctxs.append(H.Context(0))
        ctxs[-1].set_variant(variant)
    g = H.Grid.structured(et, 1600 if et == H.SIMPLEX else 3200, 500, px=2, py=1)
    loc = g.local()
    assert loc.n_own > 768 * 2048
    pats = [H.DevicePattern(loc, ctx=c, on_device=True) for c in ctxs]
    torch.cuda.synchronize()
    assert pats[0].nnz == pats[1].nnz == int(pats[1].elem_ptr[-1].item())
    for name in ("elem_ptr", "row_ptr", "col"):
        assert torch.equal(getattr(pats[0], name), getattr(pats[1], name)), name
