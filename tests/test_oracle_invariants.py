"""Known-answer invariants of the assembled SWIPDG operator on the oracle, plus
the golden fixtures as a regression of the oracle itself."""
import glob
import os

import numpy as np
import pytest

import oracle as O
from cases import compare_rows


def _rows(rp):
    return np.repeat(np.arange(rp.shape[0] - 1), np.diff(rp))


@pytest.mark.parametrize("mk", [O.kuhn_grid, O.cube_grid])
def test_symmetry_rowsums_spd(mk):
    rng = np.random.default_rng(5)
    et, c, ev = mk(9, 7, (0, 0), (2, 1))
    g = O.Grid(et, c, ev)
    k = 10.0 ** rng.uniform(-2, 2, g.ne)
    rp, col, val = O.assemble(g, O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k), O.params())
    A = O.to_scipy(rp, col, val).toarray()
    assert np.max(np.abs(A - A.T)) <= 1e-13 * np.max(np.abs(A))
    nb, _ = g.neighbors()
    interior = np.repeat((nb >= 0).all(axis=1), g.nb)
    assert np.max(np.abs(A.sum(axis=1)[interior])) <= 1e-12 * np.max(np.abs(A))
    assert np.linalg.eigvalsh(A).min() > 0


def test_q1_volume_block_closed_form():
    """kappa = 1, A = I, one h x h square, exact (2x2) volume rule, all-Neumann (no faces): the Q1 stiffness
    (1/6)[[4,-1,-1,-2],...] in Dune vertex order (00, 10, 01, 11)."""
    et, c, ev = O.cube_grid(1, 1, (0, 0), (0.5, 0.5))
    g = O.Grid(et, c, ev)
    rp, col, val = O.assemble(g, O.scalar(), O.tensor(), O.params(O.BOUNDARY_NEUMANN, vol_order=2))
    A = O.to_scipy(rp, col, val).toarray()
    ref = np.array([[4, -1, -1, -2], [-1, 4, -2, -1], [-1, -2, 4, -1], [-2, -1, -1, 4]]) / 6.0
    assert np.allclose(A, ref, atol=1e-14)


def test_p1_volume_block_closed_form():
    et, c, ev = O.kuhn_grid(1, 1, (0, 0), (1, 1))
    g = O.Grid(et, c, ev)
    rp, col, val = O.assemble(g, O.scalar(), O.tensor(), O.params(O.BOUNDARY_NEUMANN))
    A = O.to_scipy(rp, col, val).toarray()
    # triangle (0,0),(1,0),(1,1): gradients (-1,0),(1,-1),(0,1), area 1/2 -- block of element 0
    ref = 0.5 * np.array([[1, -1, 0], [-1, 2, -1], [0, -1, 1]], float)
    # element 0 also couples to element 1 through the diagonal face: compare the volume part via a
    # single-element mesh instead
    g1 = O.Grid(O.SIMPLEX, np.array([[0, 0], [1, 0], [1, 1]], float), np.array([[0, 1, 2]], np.int32))
    rp1, col1, val1 = O.assemble(g1, O.scalar(), O.tensor(), O.params(O.BOUNDARY_NEUMANN))
    assert np.allclose(O.to_scipy(rp1, col1, val1).toarray(), ref, atol=1e-14)
    assert A.shape == (6, 6)


def test_block_equals_monolithic_permuted():
    rng = np.random.default_rng(2)
    et, c, ev = O.kuhn_grid(8, 6, (0, 0), (1, 1))
    g = O.Grid(et, c, ev)
    k = rng.uniform(0.5, 2, g.ne)
    ten = O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k)
    sub = rng.integers(0, 5, g.ne).astype(np.int32)       # arbitrary (even disconnected) subdomains
    ei, rp, col, val = O.assemble_block(g, sub, 5, O.scalar(), ten, O.params())
    mrp, mcol, mval = O.assemble(g, O.scalar(), ten, O.params(), elem_index=ei)
    assert np.array_equal(rp, mrp) and np.array_equal(col, mcol)
    worst, ok = compare_rows(rp, val, mval, 1e-13)
    assert ok, worst


def test_golden_fixtures_regression():
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))
    assert len(files) >= 5
    for fn in files:
        z = np.load(fn)
        et = int(z["elem_type"])
        g = O.Grid(et, z["coords"], z["elem_vert"])
        tk = int(z["tensor_kind"])
        if tk == O.TENSOR_CONST:
            T = O.tensor(O.TENSOR_CONST, tuple(z["tensor_c"]))
        elif tk == O.TENSOR_ISO_PER_ELEM:
            T = O.tensor(tk, per_elem=np.ascontiguousarray(z["tensor_per_elem"]))
        else:
            T = O.tensor(tk, per_elem=np.ascontiguousarray(z["tensor_per_elem"].T))
        for q in range(int(z["n_comp"])):
            kind, c, b, kx, ky, order = z["kappa_%d" % q]
            rp, col, val = O.assemble(g, O.scalar(int(kind), c, b, kx, ky, order=int(order)), T,
                                      O.params(int(z["boundary"])))
            assert np.array_equal(rp, z["row_ptr"]) and np.array_equal(col, z["col"])
            assert np.array_equal(val, z["val_%d" % q]), fn


def test_quadrature_exactness():
    from math import factorial
    for et, order in [(O.SIMPLEX, 1), (O.SIMPLEX, 2), (O.SIMPLEX, 4), (O.SIMPLEX, 7), (O.CUBE, 3), (O.CUBE, 5)]:
        x, w = O.quadrature(et, order)
        for a in range(order + 1):
            for b in range(order + 1 - a):
                num = np.sum(w * x[:, 0] ** a * x[:, 1] ** b)
                ex = factorial(a) * factorial(b) / factorial(a + b + 2) if et == O.SIMPLEX else 1 / ((a + 1) * (b + 1))
                assert abs(num - ex) < 1e-14, (et, order, a, b)
