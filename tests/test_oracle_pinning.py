"""Pins the CPU oracle against the reference's own expectation tables (the only numeric pins of the path):
solution-error norms of the ESV2007 EOC studies, 3 significant figures.

  SGrid<2,2>, Q1:  test/linearelliptic-swipdg-expectations_esv2007_2dsgrid.cxx:31-36
  ALUGrid<2,2,simplex,conforming>, P1:  test/linearelliptic-swipdg-expectations_esv2007_2daluconform.cxx:32-37
  BlockSWIPDG, partitions [1 1 1] [2 2 1] [4 4 1] [8 8 1]: identical values,
      test/linearelliptic-block-swipdg-expectations_esv2007_2daluconform.cxx:37-116

Pipeline restated from test/linearelliptic.hh:143-185 (assemble, solve, error vs the exact solution on
the refinement ladder of testcases/base.hh:92-103).  The ALU ladder is rebuilt by newest-vertex bisection
(tests/mesh_tools.py).  The matching also pins the unverifiable dune-gdt constants: sigma = 8 / 14, beta
= 1, and the order-0 (1-point) volume rule of Q1 -- the alternatives are shown NOT to match.
"""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import oracle as O
from mesh_tools import nvb_mesh

SGRID_L2 = [1.13e-02, 2.90e-03, 7.41e-04, 1.88e-04]
SGRID_H1 = [2.77e-01, 1.39e-01, 6.98e-02, 3.50e-02]
ALU_L2 = [1.83e-02, 4.53e-03, 1.12e-03, 2.78e-04]
ALU_H1 = [3.28e-01, 1.62e-01, 8.04e-02, 4.01e-02]


def sig3(x):
    return float("%.2e" % x)


def _sgrid_norms(prm, levels=4):
    out = []
    for lvl in range(levels):
        n = 8 * 2 ** lvl            # Cube(-1,1,4) + 1 global refine (SGrid), then 1 refine per level
        g = O.Grid(*O.cube_grid(n, n, (-1, -1), (1, 1)))
        out.append(O.esv2007_eoc(g, prm))
    return out


def _alu_norms(prm, levels=4):
    out = []
    for lvl in range(levels):
        g = O.Grid(*nvb_mesh(4, 2 + 2 * lvl))   # 128, 512, 2048, 8192 triangles
        out.append(O.esv2007_eoc(g, prm))
    return out


def test_sgrid_q1_table():
    norms = _sgrid_norms(O.params())
    assert [sig3(l2) for l2, _ in norms] == SGRID_L2
    assert [sig3(h1) for _, h1 in norms] == SGRID_H1


def test_alu_p1_table():
    norms = _alu_norms(O.params())
    assert [sig3(l2) for l2, _ in norms] == ALU_L2
    assert [sig3(h1) for _, h1 in norms] == ALU_H1


@pytest.mark.parametrize("alt", [dict(vol_order=2), dict(sigma_inner=10.0), dict(sigma_boundary=20.0),
                                 dict(sigma_inner=20.0, sigma_boundary=38.0)])
def test_alternative_constants_do_not_match(alt):
    """The tables discriminate: the exact 2x2 volume rule or other penalty constants miss them."""
    norms = _sgrid_norms(O.params(**alt), levels=2)
    got = [sig3(l2) for l2, _ in norms] + [sig3(h1) for _, h1 in norms]
    assert got != SGRID_L2[:2] + SGRID_H1[:2]


@pytest.mark.parametrize("p", [1, 2, 4, 8])
def test_block_swipdg_alu_table(p):
    """BlockSWIPDG (oracle restatement of block-swipdg.hh) reproduces the same table for every partition."""
    out = []
    for lvl in range(3):
        et, c, ev = nvb_mesh(4, 2 + 2 * lvl)
        g = O.Grid(et, c, ev)
        cen = O.element_centers(c, ev)
        sx = np.minimum(((cen[:, 0] + 1) / 2 * p).astype(int), p - 1)
        sy = np.minimum(((cen[:, 1] + 1) / 2 * p).astype(int), p - 1)
        sub = (sx * p + sy).astype(np.int32)
        ei, rp, col, val = O.assemble_block(g, sub, p * p, O.scalar(O.FN_CONST, 1.0), O.tensor(), O.params())
        A = O.to_scipy(rp, col, val)
        b = O.rhs_esv2007(g, ei)
        u = spla.spsolve(A.tocsc(), b)
        out.append(O.error_norms_esv2007(g, u, ei))
    assert [sig3(l2) for l2, _ in out] == ALU_L2[:3]
    assert [sig3(h1) for _, h1 in out] == ALU_H1[:3]
