"""GPU right-hand side (hdd_swipdg_rhs, rhs.hip) against the oracle's restatement of the SWIPDG::init()
functionals (swipdg.hh:251-347), entry-wise (|db| <= 1e-12 max|b|), for P1 triangles, Q1 quadrilaterals and
Q_p hexahedra; and the complete GPU-assembled system (matrix + right-hand side, solved on the host)
reproducing the reference's ESV2007 expectation table."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import oracle as O
from hex_tools import lex_to_product
from mesh_tools import nvb_mesh
from test_oracle_pinning import ALU_H1, ALU_L2, sig3

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _close(got, ref):
    return np.max(np.abs(got - ref)) <= 1e-12 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_rhs_2d(ctx, et):
    torch = _torch()
    n = (7, 5)
    grid = H.Grid.structured(et, *n, (-1, -1), (1, 1))
    loc = grid.local()
    dm = H.DeviceMesh(loc)
    og = O.Grid(*(O.kuhn_grid if et == H.SIMPLEX else O.cube_grid)(*n, (-1, -1), (1, 1)))
    kel = np.random.default_rng(2).uniform(0.5, 2.0, grid.ne)
    kdev = torch.from_numpy(kel).cuda()
    T = np.random.default_rng(3).uniform(0.5, 2.0, grid.ne)
    Tdev = torch.from_numpy(T).cuda()
    cases = [
        (dict(force=H.esv2007_force()), dict(force=O.esv2007_force()), O.BOUNDARY_DIRICHLET),
        (dict(force=H.scalar_fn(H.FN_SINUSOID, 0.3, b=1.5, kx=2.0, ky=-1.0, order=3)),
         dict(force=O.scalar(O.FN_SINUSOID, 0.3, 1.5, 2.0, -1.0, order=3)), O.BOUNDARY_DIRICHLET),
        (dict(force=H.scalar_fn(H.FN_PER_ELEM, per_elem=kdev)), dict(force=O.scalar(O.FN_PER_ELEM, per_elem=kel)),
         O.BOUNDARY_DIRICHLET),
        (dict(dirichlet=H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=1.3, ky=0.7, order=3),
              kappa=H.scalar_fn(H.FN_PER_ELEM, per_elem=kdev), tensor=H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=Tdev)),
         dict(dirichlet=O.scalar(O.FN_SINUSOID, 1.0, 0.5, 1.3, 0.7, order=3), kappa=O.scalar(O.FN_PER_ELEM, per_elem=kel),
              A=O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=T)), O.BOUNDARY_DIRICHLET),
        (dict(neumann=H.scalar_fn(H.FN_COS_PRODUCT, 2.0, kx=0.4, ky=0.9, order=2)),
         dict(neumann=O.scalar(O.FN_COS_PRODUCT, 2.0, 0.0, 0.4, 0.9, order=2)), O.BOUNDARY_NEUMANN),
    ]
    for hk, ok, bkind in cases:
        g2 = grid if bkind == O.BOUNDARY_DIRICHLET else H.Grid.structured(et, *n, (-1, -1), (1, 1),
                                                                          boundary=H.BOUNDARY_ALL_NEUMANN)
        dmm = dm if g2 is grid else H.DeviceMesh(g2.local())
        b = H.rhs(ctx, dmm, prm=H.params(), **hk)
        torch.cuda.synchronize()
        ref = O.rhs_swipdg(og, prm=O.params(boundary=bkind), **ok)
        assert _close(b.cpu().numpy(), ref), hk


@pytest.mark.parametrize("deg", [1, 2, 3])
def test_rhs_hex(ctx, deg):
    torch = _torch()
    n, lo, up = (3, 2, 4), (-1.0, 0.0, 0.5), (1.0, 1.5, 2.0)
    for boundary, bk in [(H.BOUNDARY_ALL_DIRICHLET, O.BOUNDARY_DIRICHLET), (H.BOUNDARY_ALL_NEUMANN, O.BOUNDARY_NEUMANN)]:
        g = H.Grid.structured3d(n, lo, up, p=(2, 1, 1), degree=deg, boundary=boundary)
        ei = lex_to_product(g, n, lo, up)
        q = O.QpGrid(3, deg, n, lo, up)
        dm = H.DeviceMesh(g.local())
        prm = H.params_for(deg, 3)
        oprm = O.qp_params(q, boundary=bk)
        hk = dict(force=H.esv2007_force(3))
        ok = dict(force=O.esv2007_force(3))
        if bk == O.BOUNDARY_DIRICHLET:
            hk.update(dirichlet=H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=1.3, ky=0.7, order=3),
                      kappa=H.scalar_fn(H.FN_CONST, 2.0), tensor=H.tensor_fn(dim=3))
            ok.update(dirichlet=O.scalar(O.FN_SINUSOID, 1.0, 0.5, 1.3, 0.7, order=3), kappa=O.scalar(O.FN_CONST, 2.0))
        else:
            hk.update(neumann=H.scalar_fn(H.FN_CONST, 0.75))
            ok.update(neumann=O.scalar(O.FN_CONST, 0.75))
        b = H.rhs(ctx, dm, prm=prm, **hk)
        torch.cuda.synchronize()
        ref = O.qp_rhs_swipdg(q, prm=oprm, elem_index=ei, **ok)
        assert _close(b.cpu().numpy(), ref), (deg, boundary)


def test_alu_p1_table_from_gpu_system(ctx):
    """GPU matrix + GPU right-hand side -> host solve -> ESV2007 ALU table (3 s.f.)."""
    torch = _torch()
    l2s, h1s = [], []
    for lvl in range(4):
        et, c, ev = nvb_mesh(4, 2 + 2 * lvl)
        grid = H.Grid.from_connectivity(H.SIMPLEX, c, ev)
        loc = grid.local()
        dm = H.DeviceMesh(loc)
        dp = H.DevicePattern(loc)
        (val,) = H.assemble(ctx, dm, dp, [H.scalar_fn()], H.tensor_fn())
        b = H.rhs(ctx, dm, force=H.esv2007_force(), prm=H.params())
        torch.cuda.synchronize()
        rp, col, _ = dp.host
        u = spla.spsolve(O.to_scipy(rp, col, val.cpu().numpy()).tocsc(), b.cpu().numpy())
        og = O.Grid(et, c, ev)
        assert np.array_equal(loc.global_id, np.arange(grid.ne))   # no subdomains: element order kept
        l2, h1 = O.error_norms_esv2007(og, u)
        l2s.append(sig3(l2)); h1s.append(sig3(h1))
    assert l2s == ALU_L2 and h1s == ALU_H1


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["kuhn", "quad", "nvb"])
def test_rhs_vertex_indexed_equals_element_major(case):
    """The right-hand side on the vertex-indexed geometry (the default of DeviceMesh) equals the element-major
    path bit for bit: force + Dirichlet (kappa, tensor) + Neumann data on a mixed-boundary mesh, ragged last
    256-element chunk."""
    import torch
    ctx = H.Context(0)
    if case == "nvb":
        from mesh_tools import nvb_mesh
        et, coords, ev = nvb_mesh(4, 3)
        grid = H.Grid.from_connectivity(et, coords, ev)
    else:
        grid = H.Grid.structured(H.SIMPLEX if case == "kuhn" else H.CUBE, 61, 23, (0, 0), (2, 1))
    loc = grid.local()
    bnd = loc.neighbors[0] == H.NBR_DIRICHLET
    loc.neighbors[0][bnd] = H.NBR_NEUMANN          # some Neumann faces
    rng = np.random.default_rng(8)
    ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(rng.uniform(0.5, 2.0, loc.n_local)).cuda())
    out = []
    for vx in (True, False):
        dm = H.DeviceMesh(loc, vertex_indexed=vx)
        out.append(H.rhs(ctx, dm, force=H.esv2007_force(), kappa=H.scalar_fn(H.FN_CONST, 1.3), tensor=ten,
                         dirichlet=H.scalar_fn(H.FN_SINUSOID, 0.5, 1.0, 2.0, 1.0, order=3),
                         neumann=H.scalar_fn(H.FN_CONST, 0.7)))
    torch.cuda.synchronize()
    assert torch.equal(out[0], out[1])


@pytest.mark.gpu
@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_rhs_split_equals_fused(et):
    """The split 2d path (volume kernel + boundary-element list + face kernel) equals the fused one-kernel path
    (HDD_VARIANT_RHS_FUSED) bit for bit, on meshes from all-boundary (3 x 2) to ragged multi-chunk ones, with
    Dirichlet + Neumann faces, repeated calls (the list's counters reset by the face kernel) and a growing list."""
    import os
    import torch
    ctxs = []
    for variant in (0, H.VARIANT_RHS_FUSED):
        ctxs.append(H.Context(0))
        ctxs[-1].set_variant(variant)
    rng = np.random.default_rng(11)
    for n in [(3, 2), (61, 23), (200, 37)]:
        grid = H.Grid.structured(et, *n, (0, 0), (2, 1))
        loc = grid.local()
        bnd = loc.neighbors[0] == H.NBR_DIRICHLET
        loc.neighbors[0][bnd] = H.NBR_NEUMANN
        ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(rng.uniform(0.5, 2.0, loc.n_local)).cuda())
        dm = H.DeviceMesh(loc)
        kw = dict(force=H.esv2007_force(), kappa=H.scalar_fn(H.FN_CONST, 1.3), tensor=ten,
                  dirichlet=H.scalar_fn(H.FN_SINUSOID, 0.5, 1.0, 2.0, 1.0, order=3), neumann=H.scalar_fn(H.FN_CONST, 0.7))
        fused = H.rhs(ctxs[1], dm, **kw)
        for _ in range(3):
            split = H.rhs(ctxs[0], dm, **kw)
            torch.cuda.synchronize()
            assert torch.equal(split, fused), n
        # generic (run-time rule) variant of the split path: per-element force
        kw.update(force=H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(rng.uniform(-1, 1, loc.n_local)).cuda()))
        assert torch.equal(H.rhs(ctxs[0], dm, **kw), H.rhs(ctxs[1], dm, **kw)), n


def _rhs_split_case():
    """a 2d problem whose RHS takes the split path (volume kernel + boundary-element list + face kernel)"""
    torch = _torch()
    grid = H.Grid.structured(H.SIMPLEX, 64, 16, (0.0, 0.0), (5.0, 1.0))
    dm = H.DeviceMesh(grid.local())
    T = torch.from_numpy(np.random.default_rng(4).uniform(0.5, 2.0, grid.ne)).cuda()
    kw = dict(force=H.esv2007_force(), kappa=H.scalar_fn(H.FN_CONST, 1.0),
              tensor=H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=T),
              dirichlet=H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=1.3, ky=0.7, order=3), prm=H.params())
    return dm, kw, T


def test_rhs_list_survives_failed_face_launch():
    """The boundary-element list of the split RHS is context state.  If the face launch fails after the volume
    kernel has filled the list (error injection: hdd_ctx_set_debug_flags bit 524288), the call returns an error
    and re-arms the list's counters, so the next call on the same context is exact again (bit for bit equal to a
    fresh context), instead of adding the stale entries' faces a second time."""
    torch = _torch()
    dm, kw, _ = _rhs_split_case()
    ref = H.rhs(H.Context(0), dm, **kw).cpu().numpy()
    c = H.Context(0)
    first = H.rhs(c, dm, **kw).cpu().numpy()
    c.set_debug_flags(524288)
    with pytest.raises(H.HddError):
        H.rhs(c, dm, **kw)
    c.set_debug_flags(0)
    for _ in range(2):
        got = H.rhs(c, dm, **kw)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), ref)
    assert np.array_equal(first, ref)


def test_rhs_one_context_two_streams():
    """Split RHS calls with one context on two streams, back to back without host synchronisation: the context
    orders a call on a new stream behind the previous call (the list is shared), so every result is exact."""
    torch = _torch()
    dm, kw, _ = _rhs_split_case()
    ref = H.rhs(H.Context(0), dm, **kw).cpu().numpy()
    c = H.Context(0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.full((ref.size,), float("nan"), dtype=torch.float64, device="cuda") for _ in range(8)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        H.rhs(c, dm, out=o, stream=streams[i % 2].cuda_stream, **kw)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy(), ref), i
