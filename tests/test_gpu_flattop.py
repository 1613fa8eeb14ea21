"""The Spe10::Model1 channel with channel_boundary_layer != 0: a sum of dune-stuff FlatTop functions
(problems/spe10.hh:139-148, 213-222), HDD_FN_FLATTOP, evaluated on the device at the quadrature points of the
smooth-coefficient kernels (P1SmoothPolicy / the Q1 quadrature policy / the generic rhs and product kernels).
GPU vs the oracle's restatement, entry-wise (row tolerance 1e-12).  FlatTop is third-party (dune-stuff,
absent here): parity unpinned beyond the restatement (oracle/swipdg_oracle.c: flattop1)."""
import numpy as np
import pytest

import oracle as O
from cases import SPE10_LOWER, SPE10_UPPER, compare_rows

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu

RTOL = 1e-12
FLOOR = 1e-10   # rows of a vanishing coefficient near a support edge: see cases.compare_rows


def _boxes(layer=(0.1, 0.1)):
    """channel-like boxes on the SPE10 domain: two overlapping, one thin, one touching the boundary.
    A box narrower than two layers has overlapping transitions, and FlatTop is then discontinuous at l + d
    (the left transition ends at 1, the right one is already running); a quadrature point exactly there takes
    either side by rounding -- in the reference as here -- so those lines are kept off the meshes' lines."""
    b = [(0.5, 0.21, 1.6, 0.36, 0.7), (1.2, 0.25, 2.0, 0.6, 0.4), (2.5, 0.51, 4.0, 0.57, 1.0),
         (4.3, 0.0, 5.0, 0.3, 0.25)]
    return np.array([(lx, ly, ux, uy, layer[0], layer[1], v) for (lx, ly, ux, uy, v) in b])


def _mesh(et, nx, ny):
    return (O.kuhn_grid if et == H.SIMPLEX else O.cube_grid)(nx, ny, SPE10_LOWER, SPE10_UPPER)


@pytest.mark.parametrize("et,vx", [(H.SIMPLEX, True), (H.SIMPLEX, False), (H.CUBE, False)])
def test_flattop_channel_components(ctx, et, vx):
    """affine part 1 + channel and the component channel (the parametric structure, spe10.hh:160-172) in one
    call, with the SPE10 permeability tensor; ragged tiles (150 x 30 squares)."""
    import torch
    nx, ny = 150, 30
    boxes = _boxes()
    grid = H.Grid.structured(et, nx, ny, SPE10_LOWER, SPE10_UPPER)
    loc = grid.local()
    perm = O.spe10_synthetic_permeability()
    k = loc.checkerboard(SPE10_LOWER, SPE10_UPPER, 100, 20, perm)
    dm = H.DeviceMesh(loc, vertex_indexed=vx)
    dp = H.DevicePattern(loc)
    fns = [H.flattop_fn(boxes, 1.0, 1.0), H.flattop_fn(boxes, 0.0, 1.0)]
    vals = H.assemble(ctx, dm, dp, fns, H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(k).cuda()))
    torch.cuda.synchronize()
    og = O.Grid(*_mesh(et, nx, ny))
    A = O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k)
    for (c, b), v in zip([(1.0, 1.0), (0.0, 1.0)], vals):
        rp, col, ref = O.assemble(og, O.flattop(boxes, c, b), A, O.params())
        assert np.array_equal(dp.host[1], col)
        worst, ok = compare_rows(rp, v.cpu().numpy(), ref, RTOL, FLOOR)
        assert ok, (c, b, worst)
    # the channel is really there: the component is nonzero on a good part of the rows, zero elsewhere
    v1 = vals[1].cpu().numpy()
    assert 0.05 * v1.size < np.count_nonzero(v1) < 0.9 * v1.size


def test_flattop_layers_and_order(ctx):
    """a thin layer (sharp transitions) and integration order 2 (the caller's order picks the rules)"""
    import torch
    nx, ny = 64, 20
    boxes = _boxes(layer=(0.02, 0.01))
    grid = H.Grid.structured(H.SIMPLEX, nx, ny, SPE10_LOWER, SPE10_UPPER)
    loc = grid.local()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    og = O.Grid(*_mesh(H.SIMPLEX, nx, ny))
    for order in (3, 2):
        (v,) = H.assemble(ctx, dm, dp, [H.flattop_fn(boxes, 1.0, 0.9, order=order)], H.tensor_fn())
        torch.cuda.synchronize()
        rp, col, ref = O.assemble(og, O.flattop(boxes, 1.0, 0.9, order=order), O.tensor(), O.params())
        worst, ok = compare_rows(rp, v.cpu().numpy(), ref, RTOL, FLOOR)
        assert ok, (order, worst)


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_flattop_rhs_and_products(ctx, et):
    """the Dirichlet functional with a FlatTop kappa (g_D != 0) and the elliptic / penalty products, whose
    kappa is the affinely decomposed diffusion factor (swipdg.hh:251-347, 358-508)"""
    import torch
    nx, ny = 40, 12
    boxes = _boxes(layer=(0.3, 0.2))
    grid = H.Grid.structured(et, nx, ny, SPE10_LOWER, SPE10_UPPER)
    loc = grid.local()
    dm = H.DeviceMesh(loc)
    og = O.Grid(*_mesh(et, nx, ny))
    kap, okap = H.flattop_fn(boxes, 1.0, 1.0), O.flattop(boxes, 1.0, 1.0)
    g = H.scalar_fn(H.FN_SINUSOID, 0.5, b=0.25, kx=1.0, ky=2.0, order=3)
    og_d = O.scalar(O.FN_SINUSOID, 0.5, 0.25, 1.0, 2.0, order=3)
    b = H.rhs(ctx, dm, prm=H.params(), dirichlet=g, kappa=kap, tensor=H.tensor_fn())
    torch.cuda.synchronize()
    ref = O.rhs_swipdg(og, kappa=okap, dirichlet=og_d, A=O.tensor(), prm=O.params())
    assert np.max(np.abs(b.cpu().numpy() - ref)) <= 1e-12 * np.max(np.abs(ref))
    for kind in (H.PRODUCT_ELLIPTIC, H.PRODUCT_PENALTY):
        dp = H.DevicePattern(loc, volume=kind != H.PRODUCT_PENALTY)
        val = H.product(ctx, dm, kind, dp, kappa=kap, tensor=H.tensor_fn(), prm=H.params())
        torch.cuda.synchronize()
        rp, col, oval = O.product(og, kind, kappa=okap, A=O.tensor(), prm=O.params())
        worst, ok = compare_rows(rp, val.cpu().numpy(), oval, RTOL, FLOOR)
        assert ok, (kind, worst)


def test_flattop_rejected_on_hexahedra(ctx):
    g = H.Grid.structured3d((2, 2, 2), (0, 0, 0), (1, 1, 1), degree=1)
    loc = g.local()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    with pytest.raises(H.HddError):
        H.assemble(ctx, dm, dp, [H.flattop_fn(_boxes())], H.tensor_fn(dim=3))
