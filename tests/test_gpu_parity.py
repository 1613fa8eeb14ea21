"""GPU parity: the HIP assembly (through the C ABI) against the CPU oracle, entry-wise.

Tolerance (fp64): per row, max_j |a_gpu - a_oracle| <= 1e-12 * max_j |a_oracle|.
The oracle is pinned by the reference's ESV2007 expectation tables (tests/test_oracle_pinning.py).
"""
import numpy as np
import pytest

import oracle as O
from cases import SPE10_LOWER, SPE10_UPPER, compare_rows, os2014_components
from mesh_tools import affine_quad_mesh as _affine_quad_mesh, scrambled_quad_mesh as _scrambled_quad_mesh

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu

RTOL = 1e-12


def _oracle_mesh(et, nx, ny, lower, upper):
    return (O.kuhn_grid if et == H.SIMPLEX else O.cube_grid)(nx, ny, lower, upper)


def _run_product(ctx, grid, kappa_fns, tensor, prm=None, s0=0, s1=None, dmesh=None):
    import torch
    local = grid.local(s0, s1)
    dm = dmesh or H.DeviceMesh(local)
    dp = H.DevicePattern(local)
    vals = H.assemble(ctx, dm, dp, kappa_fns, tensor, prm)
    torch.cuda.synchronize()
    return local, dp.host, [v.cpu().numpy() for v in vals]


def _torch():
    import torch
    return torch


@pytest.mark.parametrize("et,nx,ny", [(H.CUBE, 16, 16), (H.SIMPLEX, 8, 8), (H.SIMPLEX, 33, 17), (H.CUBE, 9, 13)])
def test_esv2007(ctx, et, nx, ny):
    """C1 (ESV2007 SGrid 16x16 Q1) and the Kuhn/P1 analogue: kappa = 1, A = I, AllDirichlet."""
    grid = H.Grid.structured(et, nx, ny, (-1, -1), (1, 1))
    local, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn())
    og = O.Grid(*_oracle_mesh(et, nx, ny, (-1, -1), (1, 1)))
    orp, ocol, oval = O.assemble(og, O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_CONST), O.params())
    assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("et,nx,ny", [(H.SIMPLEX, 200, 40), (H.CUBE, 200, 40), (H.SIMPLEX, 100, 20)])
def test_spe10_synthetic(ctx, et, nx, ny):
    """C2 / C4 coefficient structure: A = k_cell I on the 100x20 checkerboard, kappa = 1."""
    torch = _torch()
    perm = O.spe10_synthetic_permeability()
    grid = H.Grid.structured(et, nx, ny, SPE10_LOWER, SPE10_UPPER)
    local = grid.local()
    k = local.checkerboard(SPE10_LOWER, SPE10_UPPER, 100, 20, perm)
    tk = torch.from_numpy(k).cuda()
    _, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)],
                                           H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=tk))
    ot, oc, oev = _oracle_mesh(et, nx, ny, SPE10_LOWER, SPE10_UPPER)
    ok_ = O.checkerboard(O.element_centers(oc, oev), SPE10_LOWER, SPE10_UPPER, 100, 20, perm)
    assert np.array_equal(ok_, k)
    og = O.Grid(ot, oc, oev)
    orp, ocol, oval = O.assemble(og, O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=ok_),
                                 O.params())
    assert np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("et,n", [(H.SIMPLEX, 16), (H.CUBE, 12)])
def test_os2014_components(ctx, et, n):
    """C3: OS2014 affine part + mu-component, smooth kappa (integration order 3), two value arrays in one call."""
    grid = H.Grid.structured(et, n, n, (-1, -1), (1, 1))
    comps = os2014_components()
    fns = [H.scalar_fn(H.FN_SINUSOID, c, b, kx, ky, order=3) for (c, b, kx, ky) in comps]
    _, (rp, col, _), vals = _run_product(ctx, grid, fns, H.tensor_fn())
    og = O.Grid(*_oracle_mesh(et, n, n, (-1, -1), (1, 1)))
    for (c, b, kx, ky), val in zip(comps, vals):
        orp, ocol, oval = O.assemble(og, O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=3), O.tensor(O.TENSOR_CONST),
                                     O.params())
        worst, ok = compare_rows(rp, val, oval, RTOL)
        assert ok, worst


def test_sym_tensor_per_elem_and_kappa_per_elem(ctx):
    """Anisotropic SPD tensor per element and a per-element diffusion factor (general piecewise constants)."""
    torch = _torch()
    rng = np.random.default_rng(3)
    for et in (H.SIMPLEX, H.CUBE):
        grid = H.Grid.structured(et, 11, 7, (0, 0), (2, 1))
        ne = grid.ne
        a = rng.uniform(0.5, 2.0, ne); c = rng.uniform(0.5, 2.0, ne); b = rng.uniform(-0.3, 0.3, ne)
        sym = np.stack([a, b, c], 0)            # device layout [3][n]
        kap = rng.uniform(0.1, 10.0, ne)
        tsym = torch.from_numpy(np.ascontiguousarray(sym)).cuda()
        tkap = torch.from_numpy(kap).cuda()
        _, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_PER_ELEM, per_elem=tkap)],
                                               H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=tsym))
        og = O.Grid(*_oracle_mesh(et, 11, 7, (0, 0), (2, 1)))
        osym = np.ascontiguousarray(sym.T)
        orp, ocol, oval = O.assemble(og, O.scalar(O.FN_PER_ELEM, per_elem=kap),
                                     O.tensor(O.TENSOR_SYM_PER_ELEM, per_elem=osym), O.params())
        worst, ok = compare_rows(rp, val, oval, RTOL)
        assert ok, (et, worst)


def test_neumann_boundary(ctx):
    for et in (H.SIMPLEX, H.CUBE):
        grid = H.Grid.structured(et, 6, 5, (0, 0), (1, 1), boundary=H.BOUNDARY_ALL_NEUMANN)
        _, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 2.5)], H.tensor_fn())
        og = O.Grid(*_oracle_mesh(et, 6, 5, (0, 0), (1, 1)))
        orp, ocol, oval = O.assemble(og, O.scalar(O.FN_CONST, 2.5), O.tensor(), O.params(O.BOUNDARY_NEUMANN))
        worst, ok = compare_rows(rp, val, oval, RTOL)
        assert ok, worst
        # purely Neumann: constants are in the kernel (A 1 = 0 on every row)
        rows = np.repeat(np.arange(rp.shape[0] - 1), np.diff(rp))
        rs = np.zeros(rp.shape[0] - 1)
        np.add.at(rs, rows, val)
        assert np.max(np.abs(rs)) < 1e-10 * np.max(np.abs(val))


def test_unstructured_bisection_mesh(ctx):
    """Newest-vertex-bisection mesh (the ALU conforming ladder): reversed face orientations, general
    vertex order; built through hdd_grid_create_from_connectivity."""
    from mesh_tools import nvb_mesh
    et, coords, ev = nvb_mesh(4, 3)
    grid = H.Grid.from_connectivity(H.SIMPLEX, coords, ev)
    local = grid.local()
    assert np.any((local.face_info & 0x888) != 0), "expected reversed faces in a bisection mesh"
    _, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn())
    og = O.Grid(et, coords, ev)
    orp, ocol, oval = O.assemble(og, O.scalar(O.FN_CONST, 1.0), O.tensor(), O.params())
    assert np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("et,px,py", [(H.SIMPLEX, 2, 2), (H.CUBE, 4, 4), (H.SIMPLEX, 3, 1)])
def test_block_swipdg_numbering(ctx, et, px, py):
    """BlockSWIPDG: the product's subdomain-major monolithic assembly equals the oracle's restatement of the
    block algorithm (local all-Neumann + boundary + coupling, copied into the global block numbering)."""
    nx, ny = 12, 8
    grid = H.Grid.structured(et, nx, ny, (-1, -1), (1, 1), px=px, py=py)
    _, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn())
    ot, oc, oev = _oracle_mesh(et, nx, ny, (-1, -1), (1, 1))
    pc, pev, psd = grid.connectivity()
    key = {tuple(r): i for i, r in enumerate(oev)}
    perm = np.array([key[tuple(r)] for r in pev])          # product element -> oracle element
    sub = np.empty(len(perm), np.int32)
    sub[perm] = psd
    og = O.Grid(ot, oc, oev)
    ei, orp, ocol, oval = O.assemble_block(og, sub, px * py, O.scalar(O.FN_CONST, 1.0), O.tensor(), O.params())
    assert np.array_equal(ei[perm], np.arange(len(perm)))
    assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


def test_rank_local_rows_equal_global_slice(ctx):
    """Owner-computes sharding: assembling the rows of subdomains [s0, s1) on a rank-local mesh (owned +
    ghosts) gives exactly the corresponding slice of the global matrix."""
    grid = H.Grid.structured(H.SIMPLEX, 16, 6, (0, 0), (4, 1), px=4, py=1)
    _, (grp, gcol, _), (gval,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn())
    for s0, s1 in [(0, 1), (1, 3), (3, 4)]:
        local, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(),
                                                   s0=s0, s1=s1)
        a, b = grid.subdomain_range(s0, s1)
        lo, hi = grp[a * 3], grp[b * 3]
        assert np.array_equal(col, gcol[lo:hi])
        assert np.allclose(val, gval[lo:hi], rtol=0, atol=1e-13 * np.max(np.abs(gval)))


@pytest.mark.parametrize("tk,bnd", [("iso", "dirichlet"), ("sym", "dirichlet"), ("sym", "neumann")])
def test_q1_ragged_tiles_and_tile_lists(ctx, tk, bnd):
    """Q1 closed form (the C4 kernel) on 203 x 91 quads over 4 x 3 subdomains -- uniform and non-uniform
    tiles, a ragged last tile -- with per-element diffusion factor and tensor, Dirichlet or Neumann boundary,
    against the oracle on the grid's own (subdomain-major) element order; and a rank-local slice assembled
    through the sharded path's interior / halo tile lists == its one-shot assembly, bit for bit."""
    torch = _torch()
    rng = np.random.default_rng(21)
    nx, ny = 203, 91
    boundary = H.BOUNDARY_ALL_NEUMANN if bnd == "neumann" else H.BOUNDARY_ALL_DIRICHLET
    grid = H.Grid.structured(H.CUBE, nx, ny, (0, 0), (5, 1), px=4, py=3, boundary=boundary)
    ne = grid.ne
    a = rng.uniform(0.5, 2.0, ne); c = rng.uniform(0.5, 2.0, ne); b = rng.uniform(-0.3, 0.3, ne)
    kap = rng.uniform(0.1, 10.0, ne)
    t_np = np.stack([a, b, c], 0) if tk == "sym" else a
    tkind = H.TENSOR_SYM_PER_ELEM if tk == "sym" else H.TENSOR_ISO_PER_ELEM

    def run(s0=0, s1=None):
        loc = grid.local(s0, s1)
        idx = loc.global_id
        ten = H.tensor_fn(tkind, per_elem=torch.from_numpy(np.ascontiguousarray(t_np[..., idx])).cuda())
        kf = [H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(np.ascontiguousarray(kap[idx])).cuda())]
        dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
        (v,) = H.assemble(ctx, dm, dp, kf, ten)
        tiles = None
        if s1 is not None:   # the sharded path's interior / halo tile lists, assembled in two launches
            t_in, t_bd = H.halo_tiles(loc)
            tiles = torch.full_like(v, float("nan"))
            for tl in (t_in, t_bd):
                H.assemble_tiles(ctx, dm, dp, kf, ten, torch.from_numpy(tl).cuda(), [tiles])
        torch.cuda.synchronize()
        return dp.host[0], v.cpu().numpy(), (None if tiles is None else tiles.cpu().numpy())

    rp, val, _ = run()
    pc, pev, _ = grid.connectivity()
    og = O.Grid(_oracle_mesh(H.CUBE, 1, 1, (0, 0), (1, 1))[0], pc, pev)
    okind = O.TENSOR_SYM_PER_ELEM if tk == "sym" else O.TENSOR_ISO_PER_ELEM
    oper = np.ascontiguousarray(t_np.T) if tk == "sym" else t_np
    orp, _, oval = O.assemble(og, O.scalar(O.FN_PER_ELEM, per_elem=kap), O.tensor(okind, per_elem=oper),
                              O.params(O.BOUNDARY_NEUMANN if bnd == "neumann" else O.BOUNDARY_DIRICHLET))
    assert np.array_equal(rp, orp)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst
    _, lv, lt = run(5, 9)
    assert np.array_equal(lv, lt)


@pytest.mark.parametrize("mode", ["tiles", "elements"])
@pytest.mark.parametrize("et,smooth", [(H.SIMPLEX, False), (H.SIMPLEX, True), (H.CUBE, False), (H.CUBE, True)])
def test_tile_split_overlap(ctx, et, smooth, mode):
    """The two overlap schemes of the sharded step reproduce the one-shot assembly bit for bit:
    tiles     -- hdd_swipdg_assemble_tiles: interior tiles assembled while the ghost records are garbage (NaN),
                 the halo-boundary tiles after the ghosts are restored;
    elements  -- every tile assembled on the garbage ghosts (hdd_swipdg_assemble), then the ghost-adjacent
                 elements again (hdd_swipdg_assemble_elements, listed in shuffled order).
    Two components for the smooth case: the fused two-component P1 policy takes the element list too."""
    torch = _torch()
    grid = H.Grid.structured(et, 1024, 4, (0, 0), (4, 1), px=4, py=1)
    local = grid.local(1, 3)
    dm = H.DeviceMesh(local)
    dp = H.DevicePattern(local)
    kcell = torch.from_numpy(local.checkerboard((0, 0), (4, 1), 100, 20, O.spe10_synthetic_permeability())).cuda()
    kap = ([H.scalar_fn(H.FN_SINUSOID, 1.0, b=0.5, kx=3.0, ky=2.0, order=3),
            H.scalar_fn(H.FN_SINUSOID, 0.0, b=1.0, kx=3.0, ky=2.0, order=3)]
           if smooth else [H.scalar_fn(H.FN_CONST, 1.0)])
    ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=kcell)
    refs = H.assemble(ctx, dm, dp, kap, ten)
    t_in, t_bd = H.halo_tiles(local)
    fix = H.halo_elements(local)
    assert len(t_in) and len(t_bd)
    assert 0 < len(fix) < 64 * len(t_bd)
    fix = np.random.default_rng(3).permutation(fix).astype(np.int32)
    vals = [torch.full_like(r, float("nan")) for r in refs]
    saved = dm.coords.clone()
    ghosts = torch.ones(local.n_local, dtype=torch.bool, device="cuda")
    ghosts[local.own_begin:local.own_end] = False
    dm.coords[:, ghosts] = float("nan")
    # the vertex-indexed geometry the kernels read: poison the vertices only ghost elements touch
    assert dm.elem_vertices is not None
    ev = dm.elem_vertices.cpu().numpy()
    own_v = np.zeros(dm.vertex_coords.shape[0], bool)
    own_v[ev[:, local.own_begin:local.own_end].ravel()] = True
    ghost_only = torch.from_numpy(~own_v).cuda()
    assert bool(ghost_only.any())
    saved_v = dm.vertex_coords.clone()
    dm.vertex_coords[ghost_only] = float("nan")
    if mode == "tiles":
        H.assemble_tiles(ctx, dm, dp, kap, ten, torch.from_numpy(t_in).cuda(), vals)
    else:
        H.assemble(ctx, dm, dp, kap, ten, vals=vals)
        torch.cuda.synchronize()
        assert not all(torch.equal(v, r) for v, r in zip(vals, refs))   # the garbage ghosts reached some rows
    dm.coords.copy_(saved)
    dm.vertex_coords.copy_(saved_v)
    if mode == "tiles":
        H.assemble_tiles(ctx, dm, dp, kap, ten, torch.from_numpy(t_bd).cuda(), vals)
    else:
        H.assemble_tiles(ctx, dm, dp, kap, ten, torch.from_numpy(fix).cuda(), vals, elements=True)
    torch.cuda.synchronize()
    for v, r in zip(vals, refs):
        assert torch.equal(v, r)


def test_golden_fixtures(ctx):
    """Committed golden CSR fixtures (generated by tests/golden/make_golden.py with the pinned oracle)."""
    import glob
    import os
    torch = _torch()
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))
    assert files, "no golden fixtures committed"
    for fn in files:
        z = np.load(fn)
        et = int(z["elem_type"])
        grid = H.Grid.from_connectivity(et, z["coords"], z["elem_vert"], boundary=int(z["boundary"]))
        local = grid.local()
        tk = int(z["tensor_kind"])
        tper = torch.from_numpy(np.ascontiguousarray(z["tensor_per_elem"])).cuda() if tk != H.TENSOR_CONST else None
        tensor = H.tensor_fn(tk, tuple(z["tensor_c"]), per_elem=tper)
        fns = []
        for q in range(int(z["n_comp"])):
            kind, c, b, kx, ky, order = z["kappa_%d" % q]
            fns.append(H.scalar_fn(int(kind), c, b, kx, ky, order=int(order)))
        _, (rp, col, _), vals = _run_product(ctx, grid, fns, tensor)
        assert np.array_equal(rp, z["row_ptr"]) and np.array_equal(col, z["col"]), fn
        for q, v in enumerate(vals):
            worst, ok = compare_rows(rp, v, z["val_%d" % q], RTOL)
            assert ok, (fn, q, worst)


def test_bench_size_properties(ctx):
    """Full C2 size (3200 x 640 Kuhn, 4.1 M triangles, 147 M nnz): size-independent properties checked on
    the device -- symmetry a_ij = a_ji, zero row sums on rows without Dirichlet faces, positive
    diagonal.  The entry-wise full-size comparison with the oracle is tests/test_gpu_large.py."""
    torch = _torch()
    perm = O.spe10_synthetic_permeability()
    grid = H.Grid.structured(H.SIMPLEX, 3200, 640, SPE10_LOWER, SPE10_UPPER)
    local = grid.local()
    k = torch.from_numpy(local.checkerboard(SPE10_LOWER, SPE10_UPPER, 100, 20, perm)).cuda()
    dm = H.DeviceMesh(local)
    dp = H.DevicePattern(local)
    (val,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k))
    torch.cuda.synchronize()
    assert torch.isfinite(val).all()
    n = dp.row_ptr.numel() - 1
    rows = torch.repeat_interleave(torch.arange(n, device="cuda"), dp.row_ptr[1:] - dp.row_ptr[:-1])
    cols = dp.col.long()
    # symmetry: the transpose of a symmetric pattern sorted by (col, row) lines up with (row, col)
    order = torch.argsort(cols * n + rows)
    assert torch.equal(cols[order], rows) and torch.equal(rows[order], cols)
    scale = val.abs().max()
    assert (val[order] - val).abs().max() <= 1e-12 * scale
    # diagonal positive
    diag = val[rows == cols]
    assert (diag > 0).all()
    # A 1 = 0 on rows of elements without a Dirichlet face
    rs = torch.zeros(n, dtype=torch.float64, device="cuda").index_add_(0, rows, val)
    nb = torch.from_numpy(local.neighbors).cuda()
    interior_elem = (nb >= 0).all(dim=0)
    interior_rows = interior_elem.repeat_interleave(3)
    rel = rs[interior_rows].abs().max() / scale
    assert rel < 1e-12, float(rel)


@pytest.mark.parametrize("et,nx,ny", [(H.SIMPLEX, 1, 1), (H.CUBE, 1, 1), (H.CUBE, 1, 9), (H.SIMPLEX, 9, 1),
                                      (H.CUBE, 65, 2), (H.SIMPLEX, 33, 1), (H.CUBE, 64, 1)])
def test_edge_meshes(ctx, et, nx, ny):
    """Degenerate and ragged sizes: a single element (every face Dirichlet), one-element-wide strips, and
    owned ranges one past / exactly a multiple of the 64-element tile."""
    grid = H.Grid.structured(et, nx, ny, (0, 0), (1, 1))
    _, (rp, col, _), (val,) = _run_product(ctx, grid, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn())
    og = O.Grid(*_oracle_mesh(et, nx, ny, (0, 0), (1, 1)))
    orp, ocol, oval = O.assemble(og, O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_CONST), O.params())
    assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("smooth", [False, True])
def test_parallelogram_mesh_uniform_tiles(ctx, smooth):
    """Q1 on sheared/rotated parallelograms, large enough for tiles of 64 interior elements (the padded
    LDS image path) next to boundary tiles (the contiguous path); piecewise-constant SPD tensors, or the
    OS2014 sinusoid (quadrature policy)."""
    torch = _torch()
    M = [[1.3, 0.45], [-0.2, 0.9]]
    et, coords, ev = _affine_quad_mesh(200, 40, M, (0.3, -0.1))
    grid = H.Grid.from_connectivity(et, coords, ev)
    rng = np.random.default_rng(7)
    ne = ev.shape[0]
    a = rng.uniform(0.5, 2.0, ne); c = rng.uniform(0.5, 2.0, ne); b = rng.uniform(-0.3, 0.3, ne)
    sym = np.stack([a, b, c], 0)
    if smooth:
        fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, 4 * np.pi, 2 * np.pi, order=3)]
        ofn = O.scalar(O.FN_SINUSOID, 1.0, 0.75, 4 * np.pi, 2 * np.pi, order=3)
    else:
        kap = rng.uniform(0.1, 10.0, ne)
        fns = [H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(kap).cuda())]
        ofn = O.scalar(O.FN_PER_ELEM, per_elem=kap)
    tsym = torch.from_numpy(np.ascontiguousarray(sym)).cuda()
    local, (rp, col, _), (val,) = _run_product(ctx, grid, fns, H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=tsym))
    nb = local.neighbors[:, local.own_begin:local.own_end]
    full = (nb >= 0).all(axis=0)[: (local.n_own // 64) * 64].reshape(-1, 64).all(axis=1)
    assert full.any() and not full.all(), "expected both uniform and boundary tiles"
    og = O.Grid(et, coords, ev)
    orp, ocol, oval = O.assemble(og, ofn, O.tensor(O.TENSOR_SYM_PER_ELEM, per_elem=np.ascontiguousarray(sym.T)),
                                 O.params())
    assert np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("smooth", [False, True])
def test_scrambled_quad_orientations(ctx, smooth):
    """Q1 closed-form / quadrature policies against the oracle when faces meet under all twin-face ids and
    reversals (the role-slot mapping), with full tiles (padded image) present."""
    torch = _torch()
    et, coords, ev = _scrambled_quad_mesh(130, 20, 5)
    grid = H.Grid.from_connectivity(et, coords, ev)
    local = grid.local()
    assert np.any((local.face_info & 0x8888) != 0), "expected reversed faces"
    ne = ev.shape[0]
    rng = np.random.default_rng(9)
    t = rng.uniform(0.5, 3.0, ne)
    if smooth:
        fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.5, 3.0, 2.0, order=3)]
        ofn = O.scalar(O.FN_SINUSOID, 1.0, 0.5, 3.0, 2.0, order=3)
    else:
        kap = rng.uniform(0.2, 5.0, ne)
        fns = [H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(kap).cuda())]
        ofn = O.scalar(O.FN_PER_ELEM, per_elem=kap)
    local, (rp, col, _), (val,) = _run_product(ctx, grid, fns,
                                               H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(t).cuda()))
    og = O.Grid(et, coords, ev)
    orp, ocol, oval = O.assemble(og, ofn, O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=t), O.params())
    assert np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst


@pytest.mark.parametrize("coef", ["const", "per_elem_sym", "sinusoid", "os2014_two"])
@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_scrambled_numbering_full_tiles(ctx, et, coef):
    """Full interior tiles under a random element numbering and a random vertex order per element -- P1: the
    branch-free compute_full of P1PwcPolicy with its static image layout; Q1: the rotated (padded) image of the
    half-image kernel (rotations and reflections of the reference element, Dune vertex order kept valid): the row
    blocks' neighbour order, sorted by id, takes every permutation and the twin-face ids every value.  Interior
    elements first (shuffled), then the boundary elements (shuffled), so most tiles are full."""
    torch = _torch()
    simplex = et == H.SIMPLEX
    et, coords, ev = (O.kuhn_grid if simplex else O.cube_grid)(48, 40, (0, 0), (3, 2))
    rng = np.random.default_rng(11)
    sides = [[0, 1], [0, 2], [1, 2]] if simplex else [[0, 1], [2, 3], [0, 2], [1, 3]]
    edges = np.sort(np.stack([ev[:, e] for e in sides], 1), axis=2).reshape(-1, 2)
    _, inv, cnt = np.unique(edges, axis=0, return_inverse=True, return_counts=True)
    bnd = (cnt[inv.reshape(-1)].reshape(-1, len(sides)) == 1).any(axis=1)
    order = np.concatenate([rng.permutation(np.flatnonzero(~bnd)), rng.permutation(np.flatnonzero(bnd))])
    perms = np.array([[0, 1, 2], [1, 2, 0], [2, 0, 1], [0, 2, 1], [2, 1, 0], [1, 0, 2]] if simplex else
                     [[0, 1, 2, 3], [1, 3, 0, 2], [3, 2, 1, 0], [2, 0, 3, 1],     # the square's rotations
                      [1, 0, 3, 2], [2, 3, 0, 1], [0, 2, 1, 3], [3, 1, 2, 0]])    # and reflections
    pick = perms[rng.integers(0, len(perms), len(order))]
    ev = np.ascontiguousarray(np.take_along_axis(ev[order], pick, 1)).astype(np.int32)
    grid = H.Grid.from_connectivity(et, coords, ev)
    ne = ev.shape[0]
    ten, oten = H.tensor_fn(), O.tensor(O.TENSOR_CONST)
    if coef == "sinusoid":
        fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, 4 * np.pi, 2 * np.pi, order=3)]
        ofns = [O.scalar(O.FN_SINUSOID, 1.0, 0.75, 4 * np.pi, 2 * np.pi, order=3)]
    elif coef == "os2014_two":   # C3's two-component pass (P1SmoothFusedPolicy TWO)
        comps = os2014_components()
        fns = [H.scalar_fn(H.FN_SINUSOID, c, b, kx, ky, order=3) for (c, b, kx, ky) in comps]
        ofns = [O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=3) for (c, b, kx, ky) in comps]
    elif coef == "per_elem_sym":
        kap = rng.uniform(0.1, 10.0, ne)
        sym = np.stack([rng.uniform(0.5, 2.0, ne), rng.uniform(-0.3, 0.3, ne), rng.uniform(0.5, 2.0, ne)], 0)
        fns = [H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(kap).cuda())]
        ofns = [O.scalar(O.FN_PER_ELEM, per_elem=kap)]
        ten = H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=torch.from_numpy(np.ascontiguousarray(sym)).cuda())
        oten = O.tensor(O.TENSOR_SYM_PER_ELEM, per_elem=np.ascontiguousarray(sym.T))
    else:
        fns, ofns = [H.scalar_fn(H.FN_CONST, 1.0)], [O.scalar(O.FN_CONST, 1.0)]
    local, (rp, col, _), vals = _run_product(ctx, grid, fns, ten)
    nb = local.neighbors[:, local.own_begin:local.own_end]
    full = (nb >= 0).all(axis=0)[: (local.n_own // 64) * 64].reshape(-1, 64).all(axis=1)
    assert full.sum() >= len(full) - 4 and not full.all(), "expected mostly full tiles and some boundary tiles"
    og = O.Grid(et, coords, ev)
    for ofn, val in zip(ofns, vals):
        orp, ocol, oval = O.assemble(og, ofn, oten, O.params())
        assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
        worst, ok = compare_rows(rp, val, oval, RTOL)
        assert ok, worst


@pytest.mark.parametrize("case", ["kuhn_spe10", "quad_spe10", "kuhn_sinusoid_sym", "quad_sinusoid", "nvb", "scrambled"])
def test_vertex_indexed_geometry_equals_element_major(ctx, case):
    """hdd_mesh elem_vertices / vertex_coords (the default of DeviceMesh and of the shards): the P1 / Q1
    kernels read the element and neighbour vertices through vertex ids.  Same arithmetic on the same
    coordinates, so the values must equal those of the element-major coords path bit for bit -- on
    structured Kuhn / quad meshes (ragged tiles, 2 subdomains), the bisection mesh (reversed faces) and the
    scrambled quad mesh (every twin face id), piecewise-constant and sinusoid (C3) diffusion factors."""
    torch = _torch()
    rng = np.random.default_rng(17)
    if case in ("nvb", "scrambled"):
        if case == "nvb":
            from mesh_tools import nvb_mesh
            et, coords, ev = nvb_mesh(4, 3)
        else:
            et, coords, ev = _scrambled_quad_mesh(130, 20, 5)
        grid = H.Grid.from_connectivity(et, coords, ev)
    else:
        et = H.SIMPLEX if case.startswith("kuhn") else H.CUBE
        grid = H.Grid.structured(et, 157, 43, (0, 0), (5, 1), px=2, py=1)
    local = grid.local()
    ne = local.n_local
    if "sym" in case:
        t = np.stack([rng.uniform(0.5, 2.0, ne), rng.uniform(-0.3, 0.3, ne), rng.uniform(0.5, 2.0, ne)], 0)
        ten = H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=torch.from_numpy(np.ascontiguousarray(t)).cuda())
    else:
        ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(10.0 ** rng.uniform(-3, 3, ne)).cuda())
    if "sinusoid" in case:
        fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, 4 * np.pi, 2 * np.pi, order=3)]
    else:
        fns = [H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(rng.uniform(0.2, 5.0, ne)).cuda())]
    dp = H.DevicePattern(local)
    vals = []
    for vx in (True, False):
        dm = H.DeviceMesh(local, vertex_indexed=vx)
        assert (dm.elem_vertices is not None) == vx
        (v,) = H.assemble(ctx, dm, dp, fns, ten)
        torch.cuda.synchronize()
        vals.append(v)
    assert torch.equal(vals[0], vals[1])


@pytest.mark.parametrize("kind", ["l2", "h1_semi", "elliptic", "boundary_l2", "penalty"])
def test_vertex_indexed_products_equal_element_major(ctx, kind):
    """The products (swipdg.hh:358-508) on the vertex-indexed geometry equal the element-major ones bit for
    bit (bisection mesh: reversed faces; per-element tensor and diffusion factor)."""
    torch = _torch()
    from mesh_tools import nvb_mesh
    et, coords, ev = nvb_mesh(5, 3)
    grid = H.Grid.from_connectivity(et, coords, ev)
    local = grid.local()
    rng = np.random.default_rng(5)
    ne = local.n_local
    ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(10.0 ** rng.uniform(-2, 2, ne)).cuda())
    kap = H.scalar_fn(H.FN_PER_ELEM, per_elem=torch.from_numpy(rng.uniform(0.5, 2.0, ne)).cuda())
    k = {"l2": H.PRODUCT_L2, "h1_semi": H.PRODUCT_H1_SEMI, "elliptic": H.PRODUCT_ELLIPTIC,
         "boundary_l2": H.PRODUCT_BOUNDARY_L2, "penalty": H.PRODUCT_PENALTY}[kind]
    dp = H.DevicePattern(local, volume=kind != "penalty")
    vals = []
    for vx in (True, False):
        dm = H.DeviceMesh(local, vertex_indexed=vx)
        vals.append(H.product(ctx, dm, k, dp, kappa=kap, tensor=ten))
    torch.cuda.synchronize()
    assert torch.equal(vals[0], vals[1])


@pytest.mark.parametrize("nnz,n_comp,n_s,stride_pad", [(1001, 3, 90, 6), (75460608 // 64, 2, 130, 0), (4097, 8, 70, 0),
                                                        (7, 1, 1, 2)])
def test_affine_lincomb(ctx, nnz, n_comp, n_s, stride_pad):
    """theta-lincomb A(mu_s) = sum_q theta_q(mu_s) A_q (freeze_parameter, base.hh:338-361): 256 / n_comp samples
    per launch, so several launches here (90 = 85 + 5 samples of 3 components, 130 = 128 + 2 of 2, 70 = 32 + 32 +
    6 of 8), odd lengths (scalar tail), a padded output stride -- against numpy."""
    torch = _torch()
    rng = np.random.default_rng(nnz)
    comps = [torch.from_numpy(rng.standard_normal(nnz)).cuda() for _ in range(n_comp)]
    theta = rng.uniform(-2.0, 2.0, (n_s, n_comp))
    stride = nnz + (nnz & 1) + stride_pad
    out = torch.full((n_s, stride), np.nan, dtype=torch.float64, device="cuda")
    H.affine_lincomb(ctx, comps, theta, out=out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()[:, :nnz]
    ref = theta @ np.stack([c.cpu().numpy() for c in comps])
    assert np.max(np.abs(got - ref)) <= 1e-14 * np.max(np.abs(ref)) * n_comp


def test_affine_lincomb_odd_nnz_default_output(ctx):
    """out=None with odd nnz: the front-end pads the row stride (the kernel stores 16-byte pairs) and
    returns the (n_s, nnz) view."""
    torch = _torch()
    rng = np.random.default_rng(3)
    nnz = 1001
    comps = [torch.from_numpy(rng.standard_normal(nnz)).cuda() for _ in range(2)]
    theta = rng.uniform(-1.0, 1.0, (5, 2))
    out = H.affine_lincomb(ctx, comps, theta)
    torch.cuda.synchronize()
    assert tuple(out.shape) == (5, nnz)
    ref = theta @ np.stack([c.cpu().numpy() for c in comps])
    assert np.max(np.abs(out.cpu().numpy() - ref)) <= 1e-14 * np.max(np.abs(ref)) * 2


@pytest.mark.parametrize("et,smooth", [(H.SIMPLEX, False), (H.SIMPLEX, True), (H.CUBE, False)])
def test_penalty_exponent_beta(ctx, et, smooth):
    """beta != 1 (penalty |F|^-beta; 2d default 1/(d-1) = 1 is taken inline, other values through the
    out-of-line pow of the closed-form kernels) against the oracle with the same beta."""
    torch = _torch()
    grid = H.Grid.structured(et, 19, 13, (-1, -1), (1, 0.5))
    local = grid.local()
    beta = 0.5
    prm = H.Params(O.SIGMA_INNER_P1, O.SIGMA_BOUNDARY_P1, beta, -1, -1)
    if smooth:
        (c, b, kx, ky) = os2014_components()[0]
        fns, ofn = [H.scalar_fn(H.FN_SINUSOID, c, b, kx, ky, order=3)], O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=3)
    else:
        fns, ofn = [H.scalar_fn(H.FN_CONST, 1.0)], O.scalar(O.FN_CONST, 1.0)
    kc = 1.0 + np.arange(local.n_local) % 5.0
    ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(kc).cuda())
    _, (rp, col, _), (val,) = _run_product(ctx, grid, fns, ten, prm)
    og = O.Grid(*_oracle_mesh(et, 19, 13, (-1, -1), (1, 0.5)))
    orp, ocol, oval = O.assemble(og, ofn, O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=kc), O.params(beta=beta))
    assert np.array_equal(col, ocol)
    worst, ok = compare_rows(rp, val, oval, RTOL)
    assert ok, worst
    _, _, (v1,) = _run_product(ctx, grid, fns, ten)   # beta = 1 differs (the exponent is really applied)
    assert not np.allclose(v1, val)


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
def test_element_list_bitwise(ctx, et):
    """hdd_swipdg_assemble_elements over every owned element == hdd_swipdg_assemble, bit for bit, for every
    tensor kind x diffusion-factor kind of the persistent policies (the sharded step's fixup relies on it;
    -ffp-contract=on makes a formula round the same in both kernels, profiles/r03/fp_contract.log)"""
    torch = _torch()
    rng = np.random.default_rng(1)
    grid = H.Grid.structured(et, 96, 40, (0, 0), (5, 1), px=4, py=2)
    loc = grid.local(2, 6)
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    n = loc.n_local
    iso = torch.from_numpy(rng.uniform(0.5, 2, n)).cuda()
    sym = torch.from_numpy(np.stack([rng.uniform(1, 2, n), rng.uniform(-.3, .3, n), rng.uniform(1, 2, n)])).cuda()
    kpe = torch.from_numpy(rng.uniform(0.5, 2, n)).cuda()
    lst = torch.arange(loc.n_own, dtype=torch.int32, device="cuda")
    sin = lambda c, b: H.scalar_fn(H.FN_SINUSOID, c, b=b, kx=3.0, ky=2.0, order=3)
    for ten in [H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=iso), H.tensor_fn(H.TENSOR_SYM_PER_ELEM, per_elem=sym),
                H.tensor_fn()]:
        for kap in [[H.scalar_fn(H.FN_CONST, 1.0)], [H.scalar_fn(H.FN_PER_ELEM, per_elem=kpe)], [sin(1.0, 0.5)],
                    [sin(1.0, 0.5), sin(0.0, 1.0)]]:
            ref = H.assemble(ctx, dm, dp, kap, ten)
            vals = [torch.full_like(r, float("nan")) for r in ref]
            H.assemble_tiles(ctx, dm, dp, kap, ten, lst, vals, elements=True)
            torch.cuda.synchronize()
            for v, r in zip(vals, ref):
                assert torch.equal(v, r), (ten.kind, [k.kind for k in kap])
