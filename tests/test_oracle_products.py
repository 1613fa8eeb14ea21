"""Oracle products (swipdg.hh:358-508) -- CPU known answers: 1^T M 1 = |Omega| (l2), 0 (h1_semi, elliptic:
gradients of constants), |boundary| (boundary_l2); symmetry; the penalty product is positive semi-definite
and, without boundary penalty, vanishes on globally continuous functions (jumps are zero)."""
import numpy as np

import oracle as O


def _sum(rp, col, val, n):
    M = O.to_scipy(rp, col, val, n)
    one = np.ones(n)
    return one @ (M @ one), M


def test_products_2d_known_answers():
    g = O.Grid(*O.kuhn_grid(5, 4, (0, 0), (2, 1)))
    n = g.ne * g.nb
    s, M = _sum(*O.product(g, O.PRODUCT_L2), n)
    assert abs(s - 2.0) < 1e-12 and abs(M - M.T).max() < 1e-14
    for k in (O.PRODUCT_H1_SEMI, O.PRODUCT_ELLIPTIC):
        s, M = _sum(*O.product(g, k), n)
        assert abs(s) < 1e-11 and abs(M - M.T).max() < 1e-12
    s, _ = _sum(*O.product(g, O.PRODUCT_BOUNDARY_L2), n)
    assert abs(s - 6.0) < 1e-12
    rp, col, val = O.product(g, O.PRODUCT_PENALTY)
    P = O.to_scipy(rp, col, val, n).toarray()
    assert abs(P - P.T).max() < 1e-12 * abs(P).max()
    assert np.linalg.eigvalsh(P).min() > -1e-10 * abs(P).max()
    # the inner-face penalty vanishes on globally continuous functions: with Neumann boundary (no boundary
    # penalty) the nodal interpolant of x + 2y has zero penalty energy
    rp, col, val = O.product(g, O.PRODUCT_PENALTY, prm=O.params(boundary=O.BOUNDARY_NEUMANN))
    P = O.to_scipy(rp, col, val, n)
    et, c, ev = O.kuhn_grid(5, 4, (0, 0), (2, 1))
    u = (c[ev][:, :, 0] + 2 * c[ev][:, :, 1]).reshape(-1)
    assert abs(u @ (P @ u)) < 1e-10


def test_products_qp_known_answers():
    q = O.QpGrid(3, 2, (2, 3, 2), (0, 0, 0), (1, 1.5, 2))
    n = q.ne * q.nb
    s, _ = _sum(*O.qp_product(q, O.PRODUCT_L2), n)
    assert abs(s - 3.0) < 1e-12
    s, _ = _sum(*O.qp_product(q, O.PRODUCT_H1_SEMI), n)
    assert abs(s) < 1e-10
    s, _ = _sum(*O.qp_product(q, O.PRODUCT_BOUNDARY_L2), n)
    assert abs(s - 2 * (1.5 + 2 + 3)) < 1e-12
    rp, col, val = O.qp_product(q, O.PRODUCT_PENALTY)
    P = O.to_scipy(rp, col, val, n).toarray()
    assert abs(P - P.T).max() < 1e-12 * abs(P).max()
    assert np.linalg.eigvalsh(P).min() > -1e-10 * abs(P).max()
