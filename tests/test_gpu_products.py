"""GPU products (hdd_product_assemble: l2, h1_semi, elliptic, boundary_l2, SWIPDG penalty; swipdg.hh:358-508,
over_integrate = 2) against the oracle's restatement, entry-wise (row tolerance 1e-12), on P1 triangles,
Q1 quadrilaterals and Q_p hexahedra.  No reference fixture pins products (parity unpinned beyond the
oracle's own invariants, tests/test_oracle_products.py)."""
import numpy as np
import pytest

import oracle as O
from cases import compare_rows
from hex_tools import lex_to_product

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu

KINDS = [H.PRODUCT_L2, H.PRODUCT_H1_SEMI, H.PRODUCT_ELLIPTIC, H.PRODUCT_BOUNDARY_L2, H.PRODUCT_PENALTY]


def _torch():
    import torch
    return torch


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_products_2d(ctx, et):
    torch = _torch()
    n = (6, 5)
    grid = H.Grid.structured(et, *n, (-1, -1), (1, 1))
    loc = grid.local()
    dm = H.DeviceMesh(loc)
    og = O.Grid(*(O.kuhn_grid if et == H.SIMPLEX else O.cube_grid)(*n, (-1, -1), (1, 1)))
    T = np.random.default_rng(5).uniform(0.5, 2.0, grid.ne)
    Tdev = torch.from_numpy(T).cuda()
    kap = H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=2.0, ky=1.0, order=3)
    okap = O.scalar(O.FN_SINUSOID, 1.0, 0.5, 2.0, 1.0, order=3)
    ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=Tdev)
    oten = O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=T)
    for kind in KINDS:
        dp = H.DevicePattern(loc, volume=kind != H.PRODUCT_PENALTY)
        val = H.product(ctx, dm, kind, dp, kappa=kap, tensor=ten, prm=H.params())
        torch.cuda.synchronize()
        rp, col, oval = O.product(og, kind, kappa=okap, A=oten, prm=O.params())
        assert np.array_equal(dp.host[0], rp) and np.array_equal(dp.host[1], col), kind
        worst, ok = compare_rows(rp, val.cpu().numpy(), oval, 1e-12)
        assert ok, (kind, worst)


@pytest.mark.parametrize("deg", [1, 2, 3])
def test_products_hex(ctx, deg):
    torch = _torch()
    n, lo, up = (3, 2, 3), (-1.0, 0.0, 0.5), (1.0, 1.5, 2.0)
    g = H.Grid.structured3d(n, lo, up, p=(2, 1, 1), degree=deg)
    ei = lex_to_product(g, n, lo, up)
    q = O.QpGrid(3, deg, n, lo, up)
    loc = g.local()
    dm = H.DeviceMesh(loc)
    for kind in KINDS:
        dp = H.DevicePattern(loc, volume=kind != H.PRODUCT_PENALTY)
        val = H.product(ctx, dm, kind, dp, kappa=H.scalar_fn(H.FN_CONST, 1.5), tensor=H.tensor_fn(dim=3))
        torch.cuda.synchronize()
        rp, col, oval = O.qp_product(q, kind, kappa=O.scalar(O.FN_CONST, 1.5), elem_index=ei)
        assert np.array_equal(dp.host[0], rp) and np.array_equal(dp.host[1], col), kind
        worst, ok = compare_rows(rp, val.cpu().numpy(), oval, 1e-12)
        assert ok, (kind, worst)


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_products_pwc_fast_path(ctx, et):
    """The closed-form products on the persistent tile driver (piecewise-constant kappa and tensor): Kuhn
    triangles / sheared parallelograms large enough for full 64-element tiles, a per-element diffusion
    factor and an anisotropic SPD tensor per element, against the oracle's quadrature."""
    torch = _torch()
    nx, ny = 70, 30
    et_, coords, ev = (O.kuhn_grid if et == H.SIMPLEX else O.cube_grid)(nx, ny, (0, 0), (1, 1))
    coords = coords @ np.array([[1.3, 0.45], [-0.2, 0.9]]).T + np.array([0.3, -0.1])
    grid = H.Grid.from_connectivity(et, coords, ev)
    loc = grid.local()
    dm = H.DeviceMesh(loc)
    og = O.Grid(et_, coords, ev)
    rng = np.random.default_rng(11)
    ne = ev.shape[0]
    a = rng.uniform(0.5, 2.0, ne); c = rng.uniform(0.5, 2.0, ne); b = rng.uniform(-0.3, 0.3, ne)
    sym = np.stack([a, b, c], 0)
    kap = rng.uniform(0.1, 10.0, ne)
    hk = H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(kap).cuda())
    ht = H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=torch.from_numpy(np.ascontiguousarray(sym)).cuda())
    ok_ = O.scalar(O.FN_PER_ELEM, per_elem=kap)
    ot = O.tensor(O.TENSOR_SYM_PER_ELEM, per_elem=np.ascontiguousarray(sym.T))
    for kind in KINDS:
        dp = H.DevicePattern(loc, volume=kind != H.PRODUCT_PENALTY)
        val = H.product(ctx, dm, kind, dp, kappa=hk, tensor=ht, prm=H.params())
        torch.cuda.synchronize()
        rp, col, oval = O.product(og, kind, kappa=ok_, A=ot, prm=O.params())
        assert np.array_equal(dp.host[0], rp) and np.array_equal(dp.host[1], col), kind
        worst, ok = compare_rows(rp, val.cpu().numpy(), oval, 1e-12)
        assert ok, (kind, worst)
