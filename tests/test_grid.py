"""Host grids, rank-local views, halo plans and the sparsity pattern (product, C++) against the oracle's
independent grid walk (faces from element->vertex connectivity) -- CPU only."""
import numpy as np
import pytest

import hdd_amd as H
import oracle as O
from mesh_tools import nvb_mesh

MK = {H.SIMPLEX: O.kuhn_grid, H.CUBE: O.cube_grid}


@pytest.mark.parametrize("et", [H.SIMPLEX, H.CUBE])
@pytest.mark.parametrize("nx,ny", [(1, 1), (7, 5), (16, 3)])
def test_structured_matches_oracle(et, nx, ny):
    g = H.Grid.structured(et, nx, ny, (-1, -2), (3, 1))
    coords, ev, sd = g.connectivity()
    ot, oc, oev = MK[et](nx, ny, (-1, -2), (3, 1))
    assert np.array_equal(coords, oc) and np.array_equal(ev, oev) and not sd.any()
    og = O.Grid(ot, oc, oev)
    onb, onf = og.neighbors()
    loc = g.local()
    assert loc.n_local == g.ne and loc.own_begin == 0 and loc.n_ghost == 0
    nb = loc.neighbors.T.astype(np.int64)
    assert np.array_equal(np.where(onb < 0, H.NBR_DIRICHLET, onb), nb)
    tw = np.stack([(loc.face_info.astype(np.int64) >> (4 * f)) & 7 for f in range(g.nf)], 1)
    rev = np.stack([(loc.face_info.astype(np.int64) >> (4 * f + 3)) & 1 for f in range(g.nf)], 1)
    inner = onb >= 0
    assert np.array_equal(tw[inner], onf[inner]) and not rev.any()
    rp, col, ep = loc.pattern()
    orp, ocol = og.pattern()
    assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
    assert np.array_equal(ep, rp[::g.nb])


def test_connectivity_grid_bisection_mesh():
    et, c, ev = nvb_mesh(4, 3)
    g = H.Grid.from_connectivity(H.SIMPLEX, c, ev)
    og = O.Grid(et, c, ev)
    onb, onf = og.neighbors()
    loc = g.local()
    nb = loc.neighbors.T.astype(np.int64)
    assert np.array_equal(np.where(onb < 0, -1, onb), nb)
    fi = loc.face_info.astype(np.int64)
    inner = onb >= 0
    tw = np.stack([(fi >> (4 * f)) & 7 for f in range(3)], 1)
    assert np.array_equal(tw[inner], onf[inner])
    # reversal bit: my face vertex 0 is the neighbour's face vertex 1
    FV = [(0, 1), (0, 2), (1, 2)]
    for e in range(g.ne):
        for f in range(3):
            n = onb[e, f]
            if n < 0:
                continue
            r = (fi[e] >> (4 * f + 3)) & 1
            mine = ev[e, FV[f][0]]
            theirs = ev[n, FV[onf[e, f]][0]]
            assert r == int(mine != theirs)
    assert (fi & 0x888).any()


@pytest.mark.parametrize("et,px,py", [(H.SIMPLEX, 3, 2), (H.CUBE, 4, 4), (H.SIMPLEX, 5, 1)])
def test_partitioned_numbering_is_block_numbering(et, px, py):
    nx, ny = 13, 9
    g = H.Grid.structured(et, nx, ny, (0, 0), (1, 1), px=px, py=py)
    pc, pev, psd = g.connectivity()
    ot, oc, oev = MK[et](nx, ny, (0, 0), (1, 1))
    key = {tuple(r): i for i, r in enumerate(oev)}
    perm = np.array([key[tuple(r)] for r in pev])
    assert np.array_equal(np.sort(perm), np.arange(g.ne))
    assert np.all(np.diff(psd) >= 0)            # subdomain-major
    sub = np.empty(g.ne, np.int32)
    sub[perm] = psd
    og = O.Grid(ot, oc, oev)
    ei = O.block_numbering(og, sub, px * py)
    assert np.array_equal(ei[perm], np.arange(g.ne))
    rp, col, _ = g.local().pattern()
    orp, ocol = og.pattern(ei)
    assert np.array_equal(rp, orp) and np.array_equal(col, ocol)
    # rank-local slices
    nb = g.nb
    for s0, s1 in [(0, 1), (1, px * py - 1), (px * py - 1, px * py)]:
        if s0 >= s1:
            continue
        L = g.local(s0, s1)
        a, b = g.subdomain_range(s0, s1)
        lrp, lcol, _ = L.pattern()
        assert np.array_equal(lrp, rp[a * nb:b * nb + 1] - rp[a * nb])
        assert np.array_equal(lcol, col[rp[a * nb]:rp[b * nb]])
        # local order == global order
        assert np.all(np.diff(L.global_id) > 0)
        assert np.array_equal(L.global_id[L.own_begin:L.own_end], np.arange(a, b))


def test_halo_plan_consistency():
    g = H.Grid.structured(H.SIMPLEX, 24, 6, (0, 0), (4, 1), px=4, py=2)
    world = 4
    owner = np.repeat(np.arange(world, dtype=np.int32), 2)        # 2 subdomains (one column) per rank
    locs = [g.local(2 * r, 2 * r + 2) for r in range(world)]
    plans = [locs[r].halo_plan(owner, r) for r in range(world)]
    for r in range(world):
        peers = [p["peer"] for p in plans[r]]
        assert peers == sorted(set(peers)) and r not in peers
        for p in plans[r]:
            q = p["peer"]
            back = [x for x in plans[q] if x["peer"] == r][0]
            sent_gids = locs[r].global_id[p["send"]]
            recv_gids = locs[q].global_id[back["recv_offset"]:back["recv_offset"] + back["recv_count"]]
            assert np.array_equal(sent_gids, recv_gids)
        n_recv = sum(p["recv_count"] for p in plans[r])
        assert n_recv == locs[r].n_ghost


def test_checkerboard_matches_oracle():
    perm = O.spe10_synthetic_permeability()
    for et in (H.SIMPLEX, H.CUBE):
        g = H.Grid.structured(et, 100, 20, (0, 0), (5, 1))
        k = g.local().checkerboard((0, 0), (5, 1), 100, 20, perm)
        ot, oc, oev = MK[et](100, 20, (0, 0), (5, 1))
        assert np.array_equal(k, O.checkerboard(O.element_centers(oc, oev), (0, 0), (5, 1), 100, 20, perm))


def test_bench_size_counts():
    """C2 sizes quoted in SURVEY.md 8(a): 3200x640 Kuhn -> 4,096,000 triangles, 147,386,880 nnz."""
    g = H.Grid.structured(H.SIMPLEX, 3200, 640, (0, 0), (5, 1))
    assert g.ne == 4096000
    L = g.local()
    import ctypes as C
    nnz = C.c_int64()
    nb = np.ascontiguousarray(L.neighbors)
    H._check(H.lib().hdd_pattern_count(H.SIMPLEX, L.n_local, L.own_begin, L.own_end, nb.ctypes.data, C.byref(nnz)))
    assert nnz.value == 147386880
    g1 = H.Grid.structured(H.CUBE, 16, 16, (-1, -1), (1, 1))
    rp, col, _ = g1.local().pattern()
    assert col.shape[0] == 19456                                  # C1


def test_subdomain_range_errors():
    """An empty or out-of-range owned subdomain range is rejected with HDD_ERR_RANGE (the reference's
    Stuff::Exceptions::index_out_of_range, block-swipdg.hh:560-562), not silently assembled."""
    g = H.Grid.structured(H.CUBE, 8, 8, (0, 0), (1, 1), px=2, py=1)
    for s0, s1 in ((1, 1), (2, 1), (0, 3), (-1, 1)):
        with pytest.raises(H.HddError, match="status 5"):
            g.local(s0, s1)
    assert g.local(1, 2).n_own == 32


def test_connectivity_rejects_non_parallelogram_quads():
    """HDD_CUBE meshes carry Q1 on parallelograms only (affine geometry from vertices 0, 1, 2): a
    trapezoid must be refused, not assembled wrongly."""
    coords = np.array([[0.0, 0.0], [1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
    H.Grid.from_connectivity(H.CUBE, coords, np.array([[0, 1, 2, 3]]))          # square: accepted
    sheared = coords + np.array([[0.0, 0.0], [0.0, 0.0], [0.3, 0.0], [0.3, 0.0]])
    H.Grid.from_connectivity(H.CUBE, sheared, np.array([[0, 1, 2, 3]]))         # parallelogram: accepted
    trapezoid = coords.copy()
    trapezoid[3] = [0.8, 1.0]
    with pytest.raises(H.HddError, match="parallelogram"):
        H.Grid.from_connectivity(H.CUBE, trapezoid, np.array([[0, 1, 2, 3]]))


def test_indicator_first_closed_box():
    """hdd_indicator (dune-stuff Indicator at the element barycentre, problems/spe10.hh:144, 157) against the
    oracle-side numpy twin: first closed box containing the point, 0 outside."""
    rng = np.random.default_rng(5)
    pts = rng.uniform(0.0, 5.0, (2, 1000))
    pts[1] *= 0.2
    boxes = np.array([[0.95, 0.30, 1.10, 0.45, 2000.0], [3.00, 0.75, 3.15, 0.90, -1000.0],
                      [4.25, 0.25, 4.40, 0.40, -1000.0], [0.0, 0.0, 2.5, 0.5, 7.0]])
    pts[:, :4] = [[1.0, 3.1, 4.3, 1.1], [0.4, 0.8, 0.3, 0.45]]     # inside / on the closed edge
    got = H.indicator(pts, boxes)
    ref = O.indicator(pts.T, boxes)
    assert np.array_equal(got, ref)
    assert got[0] == 2000.0 and got[1] == -1000.0 and got[2] == -1000.0 and got[3] == 2000.0


@pytest.mark.parametrize("case", ["kuhn", "quad", "nvb", "kuhn_slice"])
def test_local_vertices_reproduce_element_coords(case):
    """hdd_local_vertices (ABI v3, the vertex-indexed geometry the P1 kernels read): every element's vertices
    through elem_vertices -> vertex_coords equal the element-major coords exactly, owned and ghost columns;
    the local vertex set is the distinct vertices of the local elements in ascending global id."""
    if case == "nvb":
        et, coords, ev = nvb_mesh(3, 2)
        g = H.Grid.from_connectivity(et, coords, ev)
        loc = g.local()
    else:
        et = H.CUBE if case == "quad" else H.SIMPLEX
        g = H.Grid.structured(et, 23, 9, (0, 0), (5, 1), px=3, py=1)
        loc = g.local(1, 2) if case == "kuhn_slice" else g.local()
    lev, lxy = loc.vertices()
    assert lev.shape == (loc.nvpe, loc.n_local) and lxy.shape[1] == 2
    for k in range(loc.nvpe):
        assert np.array_equal(lxy[lev[k], 0], loc.coords[2 * k])
        assert np.array_equal(lxy[lev[k], 1], loc.coords[2 * k + 1])
    used = np.zeros(lxy.shape[0], bool)
    used[lev.ravel()] = True
    assert used.all()                                                  # no unused vertex rows
    gcoords, gev, _ = g.connectivity()
    gids = np.unique(gev[loc.global_id].ravel())                       # ascending global ids
    assert np.array_equal(lxy, gcoords[gids])
    if case == "kuhn_slice":
        assert loc.n_ghost > 0


def test_hex_from_connectivity_reproduces_structured_3d():
    """hdd_grid_create_hex_from_connectivity (ABI v6, the 3d grid part of an oversampled local discretization,
    block-swipdg.hh:783-817): the connectivity of a structured 3d grid rebuilt explicitly (with its subdomain
    ids) has the same numbering, coordinates, neighbours, twin faces and subdomains -- subdomain by subdomain."""
    g = H.Grid.structured3d((4, 3, 5), (0, 0, 0), (1, 2, 3), degree=2, p=(2, 1, 2))
    coords, ev, sd = g.connectivity()
    e = H.Grid.from_connectivity(H.HEX, coords, ev, subdomain=sd, n_sub=4, degree=2)
    assert (e.nb, e.nf, e.nvpe, e.dim) == (27, 6, 8, 3)
    for s in range(4):
        a, b = g.local(s, s + 1), e.local(s, s + 1)
        for k in ("coords", "neighbors", "face_info", "global_id", "subdomain"):
            assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_hex_from_connectivity_subset_and_rejections():
    """A subset of a structured hex grid (subdomain 0 plus one ring of face neighbours, the oversampled grid
    part): neighbours inside the subset keep their parent pairing, faces leaving it become boundary faces;
    non-box elements and wrong vertex orders are refused with HDD_ERR_UNSUPPORTED."""
    g = H.Grid.structured3d((6, 4, 4), (0, 0, 0), (1, 1, 1), degree=1, p=(2, 2, 1))
    coords, ev, sd = g.connectivity()
    full = g.local()
    own = np.flatnonzero(sd == 0)
    ring = np.unique(full.neighbors[:, own][full.neighbors[:, own] >= 0])
    ids = np.union1d(own, ring)
    sub = H.Grid.from_connectivity(H.HEX, coords, ev[ids], degree=1)
    loc = sub.local()
    pos = {int(p): i for i, p in enumerate(ids)}
    for i, p in enumerate(ids):
        for f in range(6):
            n = full.neighbors[f, p]
            want = pos.get(int(n), H.NBR_DIRICHLET) if n >= 0 else H.NBR_DIRICHLET
            assert loc.neighbors[f, i] == want
    bad = coords.copy()
    bad[ev[0, 7]] += 0.01                                             # vertex 7 off the box
    with pytest.raises(H.HddError, match="axis-aligned box"):
        H.Grid.from_connectivity(H.HEX, bad, ev[:1], degree=1)
    with pytest.raises(H.HddError, match="axis-aligned box"):
        H.Grid.from_connectivity(H.HEX, coords, ev[:1, ::-1], degree=1)   # reversed vertex order
