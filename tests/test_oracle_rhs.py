"""Oracle right-hand sides (SWIPDG::init() functionals, swipdg.hh:251-347) -- CPU only.

L2Volume with the ESV2007 force is the functional the pinned expectation tables were reproduced with
(test_oracle_pinning.py), so or_rhs_swipdg(force) must equal it.  The Dirichlet functional
(DirichletBoundarySWIPDG) has no reference fixture (every BASELINE problem has g_D = 0): it is checked by a
manufactured non-homogeneous Dirichlet problem whose SWIPDG solution converges at O(h^2) in L2 (P1) --
wrong signs or penalty in the functional break the convergence.  L2Face and L2Volume also obey the
partition-of-unity sums sum_i b_i = int g."""
import numpy as np
import scipy.sparse.linalg as spla

import oracle as O


def test_force_functional_equals_pinned_rhs():
    for mk, n in [(O.kuhn_grid, 8), (O.cube_grid, 16)]:
        g = O.Grid(*mk(n, n, (-1, -1), (1, 1)))
        assert np.max(np.abs(O.rhs_swipdg(g, force=O.esv2007_force()) - O.rhs_esv2007(g))) < 1e-15


def test_partition_of_unity_sums():
    g = O.Grid(*O.kuhn_grid(6, 5, (0, 0), (3, 2)))
    b = O.rhs_swipdg(g, force=O.scalar(O.FN_CONST, 1.5))
    assert abs(b.sum() - 1.5 * 6.0) < 1e-12
    b = O.rhs_swipdg(g, neumann=O.scalar(O.FN_CONST, 2.0), prm=O.params(boundary=O.BOUNDARY_NEUMANN))
    assert abs(b.sum() - 2.0 * 10.0) < 1e-12
    q = O.QpGrid(3, 3, (2, 3, 2), (0, 0, 0), (1, 2, 3))
    b = O.qp_rhs_swipdg(q, neumann=O.scalar(O.FN_CONST, 0.5), prm=O.qp_params(q, boundary=O.BOUNDARY_NEUMANN))
    assert abs(b.sum() - 0.5 * 2 * (2 + 3 + 6)) < 1e-12
    q = O.QpGrid(3, 3, (3, 3, 3), (-0.5, -0.5, -0.5), (1, 1, 1))
    b = O.qp_rhs_swipdg(q, force=O.esv2007_force(3))
    k = np.pi / 2
    exact = 0.75 * np.pi ** 2 * ((np.sin(k) - np.sin(-0.5 * k)) / k) ** 3
    assert abs(b.sum() - exact) < 1e-6 * abs(exact)


def _p1_l2_error(coords, ev, u, exact):
    """L2 error of a DG P1 (vertex-Lagrange) function on triangles, Dunavant degree-4 rule."""
    a, b = 0.44594849091596488632, 0.091576213509770743460
    lam = np.array([[a, a, 1 - 2 * a], [1 - 2 * a, a, a], [a, 1 - 2 * a, a],
                    [b, b, 1 - 2 * b], [1 - 2 * b, b, b], [b, 1 - 2 * b, b]])
    w = np.array([0.22338158967801146570] * 3 + [0.10995174365532186764] * 3) * 0.5
    P = coords[ev]                                          # [ne, 3, 2]
    det = np.abs((P[:, 1, 0] - P[:, 0, 0]) * (P[:, 2, 1] - P[:, 0, 1]) - (P[:, 2, 0] - P[:, 0, 0]) * (P[:, 1, 1] - P[:, 0, 1]))
    U = u.reshape(-1, 3)
    err = 0.0
    for l, wk in zip(lam, w):
        # barycentric weights of the vertices (v0 = 1 - x - y, v1 = x, v2 = y)
        x = l[2] * P[:, 0] + l[0] * P[:, 1] + l[1] * P[:, 2]
        uh = l[2] * U[:, 0] + l[0] * U[:, 1] + l[1] * U[:, 2]
        err += np.sum(wk * det * (exact(x) - uh) ** 2)
    return np.sqrt(err)


def test_dirichlet_functional_manufactured_convergence():
    kx, ky = 1.3, 0.7
    exact = lambda x: 1.0 + 0.5 * np.sin(kx * x[:, 0] + ky * x[:, 1])
    f = O.scalar(O.FN_SINUSOID, 0.0, 0.5 * (kx * kx + ky * ky), kx, ky, order=3)
    gD = O.scalar(O.FN_SINUSOID, 1.0, 0.5, kx, ky, order=3)
    errs = []
    for n in (4, 8, 16):
        et, c, ev = O.kuhn_grid(n, n, (-1, -1), (1, 1))
        g = O.Grid(et, c, ev)
        rp, col, val = O.assemble(g, O.scalar(), O.tensor(), O.params())
        b = O.rhs_swipdg(g, force=f, kappa=O.scalar(), A=O.tensor(), dirichlet=gD)
        u = spla.spsolve(O.to_scipy(rp, col, val).tocsc(), b)
        errs.append(_p1_l2_error(c, ev, u, exact))
    rates = np.log2(np.array(errs[:-1]) / np.array(errs[1:]))
    assert errs[-1] < 2e-3 and (rates > 1.75).all(), (errs, rates)
