"""CPU checks of the restated dune-stuff FlatTop (oracle/swipdg_oracle.c: or_flattop) and of the summed
Indicator the Spe10::Model1 channel is at channel_boundary_layer == 0 (problems/spe10.hh:139-148):
  - the FlatTop against an independent numpy restatement of the same definition, its C^1 transitions
    (value / slope continuity at l - d, l + d, u - d, u + d) and its plateau / support;
  - a FlatTop box enclosing the whole domain is the constant c + b v: the oracle's FLATTOP assembly equals its
    constant-kappa assembly (integration order only changes the rules, not an exact constant integrand);
  - hdd_indicator_sum (the product's host evaluation) == the oracle's, and it differs from the first-match
    Indicator exactly where boxes overlap (the channel is make_sum, not one Indicator).
FlatTop itself is third-party (absent here): parity unpinned."""
import numpy as np
import pytest

import oracle as O
from cases import compare_rows


def _ft1(x, l, u, d):
    x = np.asarray(x, float)
    t_l = (x - (l + d)) / (2 * d)
    t_r = (x - (u - d)) / (2 * d)
    return np.where(x < l - d, 0.0, np.where(x < l + d, (1 + t_l) ** 2 * (1 - 2 * t_l),
                    np.where(x < u - d, 1.0, np.where(x < u + d, (1 - t_r) ** 2 * (1 + 2 * t_r), 0.0))))


BOX = np.array([0.2, 0.3, 0.6, 0.5, 0.05, 0.02, 2.0])


def test_flattop_matches_numpy_restatement():
    rng = np.random.default_rng(1)
    pts = np.column_stack([rng.uniform(0.0, 0.8, 400), rng.uniform(0.2, 0.6, 400)])
    got = np.array([O.flattop_at(BOX, x, y) for x, y in pts])
    ref = BOX[6] * _ft1(pts[:, 0], BOX[0], BOX[2], BOX[4]) * _ft1(pts[:, 1], BOX[1], BOX[3], BOX[5])
    assert np.max(np.abs(got - ref)) <= 1e-15 * BOX[6]
    assert np.any(got == 0.0) and np.any(got == BOX[6]) and np.any((got > 0) & (got < BOX[6]))


def test_flattop_c1_transitions_and_support():
    l, u, d = BOX[0], BOX[2], BOX[4]
    y = 0.4   # on the y plateau
    f = lambda x: O.flattop_at(BOX, x, y) / BOX[6]
    h = 1e-7
    for xk, val in [(l - d, 0.0), (l, 0.5), (l + d, 1.0), (u - d, 1.0), (u, 0.5), (u + d, 0.0)]:
        assert abs(f(xk - h) - val) < 1e-5 and abs(f(xk + h) - val) < 1e-5, xk   # slope <= 15 here
    for xk in (l - d, l + d, u - d, u + d):   # the slope is continuous (0) at the layer ends
        sl = (f(xk) - f(xk - h)) / h
        sr = (f(xk + h) - f(xk)) / h
        assert abs(sl) < 1e-3 and abs(sr) < 1e-3, xk   # vs the 15 of the mid-layer slope
    assert abs((f(l + 1e-6) - f(l - 1e-6)) / 2e-6 - 1.5 / (2 * d)) < 1e-3   # max slope 3/2 / (2d) at the face
    assert f(l - d - 1e-9) == 0.0 and f(u + d + 1e-9) == 0.0 and f(0.5 * (l + u)) == 1.0


@pytest.mark.parametrize("mesh", ["kuhn", "quad"])
def test_flattop_enclosing_box_is_constant(mesh):
    et, coords, ev = (O.kuhn_grid if mesh == "kuhn" else O.cube_grid)(12, 6, (0.0, 0.0), (2.0, 1.0))
    g = O.Grid(et, coords, ev)
    box = [[-1.0, -1.0, 3.0, 2.0, 0.1, 0.1, 0.75]]
    rp, col, ft = O.assemble(g, O.flattop(box, 1.0, 2.0), O.tensor(), O.params())
    # the same rules (order 3 kappa: volume order 3, faces 5; a constant kappa alone gets the reference's
    # 1-point volume rule, which is not exact for Q1 stiffness)
    _, _, cst = O.assemble(g, O.scalar(O.FN_CONST, 1.0 + 2.0 * 0.75), O.tensor(), O.params(vol_order=3, face_order=5))
    worst, ok = compare_rows(rp, ft, cst, 1e-13)
    assert ok, worst


def test_indicator_sum_matches_oracle_and_differs_on_overlaps():
    H = pytest.importorskip("hdd_amd")
    et, coords, ev = O.kuhn_grid(100, 20, (0.0, 0.0), (5.0, 1.0))
    cen = O.element_centers(coords, ev)
    ch, _ = O.spe10_channel_boxes()
    boxes = np.vstack([ch, [[1.7, 0.45, 1.8, 0.6, 5.0]]])   # plus one box overlapping the channel
    got = H.indicator(np.ascontiguousarray(cen.T), boxes, summed=True)
    assert np.array_equal(got, O.indicator_sum(cen, boxes))
    first = H.indicator(np.ascontiguousarray(cen.T), boxes)
    assert np.array_equal(first, O.indicator(cen, boxes))
    overlap = np.zeros(len(cen), int)
    for lx, ly, ux, uy, _ in boxes:
        overlap += (cen[:, 0] >= lx) & (cen[:, 0] <= ux) & (cen[:, 1] >= ly) & (cen[:, 1] <= uy)
    assert np.array_equal(got != first, overlap > 1) and (overlap > 1).any()
