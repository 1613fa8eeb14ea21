"""Q1 half-image kernel (Q1PwcPolicy<.., H2>: the tile's two 32-element halves staged in turn through a 20 KB
LDS image, two waves per SIMD; the default on vertex-indexed meshes) == the whole-tile image kernel, bit for bit,
on vertex-indexed and on element-major geometry.

The two kernels run the same closed-form arithmetic (swipdg_device.hh, Q1PwcPolicy::compute) and differ only in
how a tile's row blocks reach HBM, so every value must be identical -- uniform, non-uniform and ragged tiles,
tile lists, the sharded step's SKIP launch, Neumann / Dirichlet, iso / symmetric tensors, per-element kappa.
The whole-tile kernel is itself pinned to the oracle (test_gpu_parity.py); the half-image kernel is checked
against the oracle directly here too.  Reference: block-swipdg.hh:1270-1326, swipdg.hh:485.
"""
import numpy as np
import pytest

import oracle as O
from cases import SPE10_LOWER, SPE10_UPPER, compare_rows
from mesh_tools import affine_quad_mesh, scrambled_quad_mesh

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu

# verification variants (swipdg_q1.hip): the default on vertex-indexed meshes is the half-image kernel
WHOLE = H.VARIANT_Q1_WHOLE_TILE                            # the whole-tile image kernel (round 3's default)
WHOLE_EM = H.VARIANT_Q1_WHOLE_TILE | H.VARIANT_ELEMENT_MAJOR   # ... on element-major coordinates


def _all(ctx, fn):
    """fn() under the whole-tile kernel on element-major and on vertex-indexed geometry, and the (default)
    half-image kernel -> [whole_em, whole_vx, half]"""
    import torch
    out = []
    for variant in (WHOLE_EM, WHOLE, 0):
        ctx.set_variant(variant)
        try:
            r = fn()
            torch.cuda.synchronize()
        finally:
            ctx.set_variant(0)
        out.append(r)
    return out


def _bits(a):
    return np.ascontiguousarray(a).view(np.int64)


@pytest.mark.parametrize("tk,bnd,kpe", [("iso", "dirichlet", False), ("iso", "dirichlet", True),
                                        ("sym", "dirichlet", True), ("sym", "neumann", False)])
def test_half_image_equals_whole_tile(ctx, tk, bnd, kpe):
    """203 x 91 quads over 4 x 3 subdomains: uniform / non-uniform / ragged tiles, and the oracle"""
    import torch
    rng = np.random.default_rng(5)
    nx, ny = 203, 91
    boundary = H.BOUNDARY_ALL_NEUMANN if bnd == "neumann" else H.BOUNDARY_ALL_DIRICHLET
    grid = H.Grid.structured(H.CUBE, nx, ny, (0, 0), (5, 1), px=4, py=3, boundary=boundary)
    ne = grid.ne
    a = rng.uniform(0.5, 2.0, ne); c = rng.uniform(0.5, 2.0, ne); b = rng.uniform(-0.3, 0.3, ne)
    kap = rng.uniform(0.1, 10.0, ne)
    t_np = np.stack([a, b, c], 0) if tk == "sym" else a
    tkind = H.TENSOR_SYM_PER_ELEM if tk == "sym" else H.TENSOR_ISO_PER_ELEM
    loc = grid.local()
    idx = loc.global_id
    ten = H.tensor_fn(tkind, per_elem=torch.from_numpy(np.ascontiguousarray(t_np[..., idx])).cuda())
    kf = [H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(np.ascontiguousarray(kap[idx])).cuda())
          if kpe else H.scalar_fn(H.FN_CONST, 1.7)]
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    whole, whole_vx, half = _all(ctx, lambda: H.assemble(ctx, dm, dp, kf, ten)[0].cpu().numpy())
    assert np.array_equal(_bits(whole), _bits(whole_vx))
    assert np.array_equal(_bits(whole), _bits(half))
    pc, pev, _ = grid.connectivity()
    og = O.Grid(O.cube_grid(1, 1, (0, 0), (1, 1))[0], pc, pev)
    okind = O.TENSOR_SYM_PER_ELEM if tk == "sym" else O.TENSOR_ISO_PER_ELEM
    oper = np.ascontiguousarray(t_np.T) if tk == "sym" else t_np
    okap = O.scalar(O.FN_PER_ELEM, per_elem=kap) if kpe else O.scalar(O.FN_CONST, 1.7)
    orp, _, oval = O.assemble(og, okap, O.tensor(okind, per_elem=oper),
                              O.params(O.BOUNDARY_NEUMANN if bnd == "neumann" else O.BOUNDARY_DIRICHLET))
    worst, ok = compare_rows(orp, half, oval, 1e-12)
    assert ok, worst


@pytest.mark.parametrize("nx,ny", [(1, 1), (1, 9), (9, 1), (8, 4), (32, 1), (33, 1), (16, 3), (65, 2), (200, 40)])
def test_half_image_edge_meshes(ctx, nx, ny):
    """tiles with <= 32 elements (empty second half), exactly 32 / 33 / 64 / 65, the SPE10 checkerboard"""
    import torch
    perm = O.spe10_synthetic_permeability()
    grid = H.Grid.structured(H.CUBE, nx, ny, SPE10_LOWER, SPE10_UPPER)
    loc = grid.local()
    k = torch.from_numpy(loc.checkerboard(SPE10_LOWER, SPE10_UPPER, 100, 20, perm)).cuda()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    kf, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    whole, whole_vx, half = _all(ctx, lambda: H.assemble(ctx, dm, dp, kf, ten)[0].cpu().numpy())
    assert np.isfinite(half).all()
    assert np.array_equal(_bits(whole), _bits(whole_vx))
    assert np.array_equal(_bits(whole), _bits(half))


@pytest.mark.parametrize("kind", ["parallelogram", "scrambled"])
def test_half_image_general_quads(ctx, kind):
    """sheared parallelograms (uniform tiles) and scrambled orientations (twin faces / reversals)"""
    import torch
    if kind == "parallelogram":
        et, coords, ev = affine_quad_mesh(200, 40, [[1.3, 0.45], [-0.2, 0.9]], (0.3, -0.1))
    else:
        et, coords, ev = scrambled_quad_mesh(130, 20, 5)
    grid = H.Grid.from_connectivity(et, coords, ev)
    loc = grid.local()
    x, y = loc.centers()
    k = torch.from_numpy(np.ascontiguousarray(10.0 ** np.sin(7 * x + 3 * y))).cuda()
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    kf, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    whole, whole_vx, half = _all(ctx, lambda: H.assemble(ctx, dm, dp, kf, ten)[0].cpu().numpy())
    assert np.array_equal(_bits(whole), _bits(whole_vx))
    assert np.array_equal(_bits(whole), _bits(half))


def test_half_image_tile_lists_and_element_fixup(ctx):
    """the sharded paths: interior / halo tile lists (TL launch) and every tile on poisoned ghosts followed by
    the ghost-adjacent element pass, both == the one-shot whole-tile assembly"""
    import torch
    grid = H.Grid.structured(H.CUBE, 1024, 6, (0, 0), (4, 1), px=4, py=1)
    local = grid.local(1, 3)
    dm, dp = H.DeviceMesh(local), H.DevicePattern(local)
    k = torch.from_numpy(local.checkerboard((0, 0), (4, 1), 100, 20, O.spe10_synthetic_permeability())).cuda()
    kf, ten = [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    ctx.set_variant(WHOLE)
    ref = H.assemble(ctx, dm, dp, kf, ten)[0]
    t_in, t_bd = H.halo_tiles(local)
    fix = np.random.default_rng(4).permutation(H.halo_elements(local)).astype(np.int32)
    ctx.set_variant(0)
    try:
        v = torch.full_like(ref, float("nan"))
        for tl in (t_in, t_bd):
            H.assemble_tiles(ctx, dm, dp, kf, ten, torch.from_numpy(tl).cuda(), [v])
        w = torch.full_like(ref, float("nan"))
        saved, saved_v = dm.coords.clone(), dm.vertex_coords.clone()
        ghosts = torch.ones(local.n_local, dtype=torch.bool, device="cuda")
        ghosts[local.own_begin:local.own_end] = False
        dm.coords[:, ghosts] = float("nan")
        ev = dm.elem_vertices.cpu().numpy()
        own_v = np.zeros(dm.vertex_coords.shape[0], bool)
        own_v[ev[:, local.own_begin:local.own_end].ravel()] = True
        dm.vertex_coords[torch.from_numpy(~own_v).cuda()] = float("nan")
        H.assemble(ctx, dm, dp, kf, ten, vals=[w])
        dm.coords.copy_(saved)
        dm.vertex_coords.copy_(saved_v)
        H.assemble_tiles(ctx, dm, dp, kf, ten, torch.from_numpy(fix).cuda(), [w], elements=True)
        torch.cuda.synchronize()
    finally:
        ctx.set_variant(0)
    assert torch.equal(v, ref)
    assert torch.equal(w, ref)
