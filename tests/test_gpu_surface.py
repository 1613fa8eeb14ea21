"""The header-only C++ operator surface (include/hdd_discretizations.hh: Discretizations::SWIPDG /
BlockSWIPDG) driven by examples/surface_main.cpp, checked against the oracle: block system matrix, local
operator A_00 and coupling operator A_0n (block-swipdg.hh:625-676), OS2014 affine part / mu-component and
freeze_parameter(0.3) = A_aff + 0.3 A_1 (base.hh:338-341), localize/globalize round trip, the reference's
error paths (non-neighbour coupling, parametric tensor)."""
import math
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle as O
from cases import compare_rows

H = pytest.importorskip("hdd_amd")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "bin", "surface_main")


def test_surface_example_is_built():
    assert os.access(EXE, os.X_OK), "examples/bin/surface_main missing: run make -C dune-hdd_amd"


@pytest.mark.gpu
def test_cpp_surface_against_oracle():
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([EXE, d], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "roundtrip 1" in r.stdout and "coupling(0,3) rejected" in r.stdout
        assert "rejected: The diffusion tensor must not be parametric!" in r.stdout
        assert "os2014 parametric 1 components 1" in r.stdout
        ld = lambda n, t: np.fromfile(os.path.join(d, n + ".bin"), dtype=t)
        brp, bcol, bval = ld("block_row_ptr", np.int64), ld("block_col", np.int32), ld("block_affine", np.float64)
        nbs = ld("neighbours0", np.int32)
        lrp, lcol, lval = ld("local0_row_ptr", np.int64), ld("local0_col", np.int32), ld("local0_affine", np.float64)
        crp, ccol, cval = ld("coupling0_row_ptr", np.int64), ld("coupling0_col", np.int32), ld("coupling0_affine", np.float64)
        osa, osc, osf = ld("os_affine", np.float64), ld("os_comp0", np.float64), ld("os_frozen_0.3", np.float64)
        brhs = ld("block_rhs", np.float64)
        pl2_rp, pl2 = ld("product_l2_row_ptr", np.int64), ld("product_l2", np.float64)
        ppen_rp, ppen = ld("product_penalty_row_ptr", np.int64), ld("product_penalty", np.float64)
        hrp, hcol, hval = ld("hex_row_ptr", np.int64), ld("hex_col", np.int32), ld("hex_affine", np.float64)
        hrhs = ld("hex_rhs", np.float64)
        assert "rhs components 0" in r.stdout and "product rejected: Product 'h2' not available!" in r.stdout
        assert "hex order 3 dofs 1728" in r.stdout
    # oracle: block-SWIPDG on the same multiscale grid
    g = H.Grid.structured(H.SIMPLEX, 16, 16, (-1, -1), (1, 1), px=2, py=2)
    pc, pev, psd = g.connectivity()
    et, oc, oev = O.kuhn_grid(16, 16, (-1, -1), (1, 1))
    key = {tuple(r): i for i, r in enumerate(oev)}
    perm = np.array([key[tuple(r)] for r in pev])
    sub = np.empty(g.ne, np.int32)
    sub[perm] = psd
    og = O.Grid(et, oc, oev)
    ei, rp, col, val = O.assemble_block(og, sub, 4, O.scalar(), O.tensor(), O.params())
    assert np.array_equal(brp, rp) and np.array_equal(bcol, col)
    assert compare_rows(rp, bval, val, 1e-12)[1]
    # right-hand side and products through the surface (block numbering = elem_index ei)
    b = O.rhs_swipdg(og, force=O.esv2007_force(), elem_index=ei)
    assert np.max(np.abs(brhs - b)) <= 1e-12 * np.max(np.abs(b))
    for prod_rp, prod, kind in [(pl2_rp, pl2, O.PRODUCT_L2), (ppen_rp, ppen, O.PRODUCT_PENALTY)]:
        orp, _, oval = O.product(og, kind, elem_index=ei)
        assert np.array_equal(prod_rp, orp)
        assert compare_rows(orp, prod, oval, 1e-12)[1]
    A = O.to_scipy(rp, col, val).tocsr()
    a0, b0 = g.subdomain_range(0, 1)
    n0 = int(nbs[0])
    an, bn = g.subdomain_range(n0, n0 + 1)
    L = A[a0 * 3:b0 * 3, a0 * 3:b0 * 3].tocsr()
    L.sort_indices()
    assert np.array_equal(lrp, L.indptr) and np.array_equal(lcol, L.indices)
    assert np.max(np.abs(lval - L.data)) <= 1e-12 * np.max(np.abs(L.data))
    Cm = A[a0 * 3:b0 * 3, an * 3:bn * 3].tocsr()    # keeps the pattern's explicit zeros: the coupling
    Cm.sort_indices()                                # pattern is the full element-block face coupling
    assert np.array_equal(crp, Cm.indptr) and np.array_equal(ccol, Cm.indices)
    assert np.max(np.abs(cval - Cm.data)) <= 1e-12 * np.max(np.abs(val))
    assert sorted(nbs.tolist()) == [1, 2]      # 2x2 partition: subdomain 0's face neighbours
    # OS2014 components and the frozen operator
    g2 = O.Grid(*O.kuhn_grid(8, 8, (-1, -1), (1, 1)))
    kx, ky = 4 * math.pi, 2 * math.pi
    rp2, col2, va = O.assemble(g2, O.scalar(O.FN_SINUSOID, 1.0, 0.75, kx, ky, order=3), O.tensor(), O.params())
    _, _, vc = O.assemble(g2, O.scalar(O.FN_SINUSOID, 0.0, -0.75, kx, ky, order=3), O.tensor(), O.params())
    assert compare_rows(rp2, osa, va, 1e-12)[1] and compare_rows(rp2, osc, vc, 1e-12)[1]
    assert compare_rows(rp2, osf, va + 0.3 * vc, 1e-12)[1]
    # C5 through the surface: Q3 hexahedra, matrix and right-hand side vs the Q_p oracle
    q = O.QpGrid(3, 3, (3, 3, 3), (-1, -1, -1), (1, 1, 1))
    orp, ocol, oval = O.qp_assemble(q, O.scalar(), O.qp_tensor(), O.qp_params(q))
    assert np.array_equal(hrp, orp) and np.array_equal(hcol, ocol)
    assert compare_rows(orp, hval, oval, 1e-12)[1]
    ob = O.qp_rhs_swipdg(q, force=O.esv2007_force(3))
    assert np.max(np.abs(hrhs - ob)) <= 1e-12 * np.max(np.abs(ob))
