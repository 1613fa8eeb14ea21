"""The full-size GPU tests (tests/test_gpu_large.py) check the C2 / C3 / C4 matrices against the oracle's
owner-computes OpenMP walk (`O.assemble_owner`, oracle/swipdg_oracle.c: or_assemble_swipdg_owner), because
the pinned primal walk (`O.assemble`, the restatement of SystemAssembler::walk over EllipticSWIPDG,
swipdg.hh:485; or_assemble_swipdg) is sequential and too slow at those sizes.  The owner variant evaluates
every interior face from both sides instead of once, so the two differ only in rounding.  This test closes
that link of the parity chain: owner == primal at <= 1e-13 per row on every small mesh / coefficient class
the GPU tests use (Kuhn, bisection, scrambled and sheared parallelogram quads; per-element iso / symmetric
tensors, sinusoid and per-element diffusion factors; Dirichlet and Neumann; 1 and 4 OpenMP threads)."""
import numpy as np
import pytest

import oracle as O
from cases import SPE10_LOWER, SPE10_UPPER, compare_rows, os2014_components
from mesh_tools import affine_quad_mesh, nvb_mesh, scrambled_quad_mesh

RTOL = 1e-13


def _mesh(name):
    if name == "kuhn":
        return O.kuhn_grid(33, 17, (-1, -1), (1, 1))
    if name == "quad":
        return O.cube_grid(29, 13, (-1, -1), (1, 1))
    if name == "kuhn_spe10":
        return O.kuhn_grid(100, 20, SPE10_LOWER, SPE10_UPPER)
    if name == "quad_spe10":
        return O.cube_grid(100, 20, SPE10_LOWER, SPE10_UPPER)
    if name == "nvb":
        return nvb_mesh(4, 3)
    if name == "scrambled":
        return scrambled_quad_mesh(40, 12, 5)
    if name == "parallelogram":
        return affine_quad_mesh(30, 10, [[1.3, 0.45], [-0.2, 0.9]], (0.3, -0.1))
    raise KeyError(name)


def _coefficients(name, grid, rng):
    ne = grid.ne
    if name == "const":
        return O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_CONST)
    if name == "spe10":
        et, coords, ev = grid.elem_type, grid.coords, grid.ev
        k = O.checkerboard(O.element_centers(coords, ev), SPE10_LOWER, SPE10_UPPER, 100, 20,
                           O.spe10_synthetic_permeability())
        return O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k)
    if name == "sinusoid":
        c, b, kx, ky = os2014_components()[0]
        return O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=3), O.tensor(O.TENSOR_CONST)
    if name == "sinusoid_comp":
        c, b, kx, ky = os2014_components()[1]
        return O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=3), O.tensor(O.TENSOR_CONST)
    if name == "per_elem_sym":
        sym = np.stack([rng.uniform(0.5, 2.0, ne), rng.uniform(-0.3, 0.3, ne), rng.uniform(0.5, 2.0, ne)], 1)
        kap = rng.uniform(0.1, 10.0, ne)
        return (O.scalar(O.FN_PER_ELEM, per_elem=kap),
                O.tensor(O.TENSOR_SYM_PER_ELEM, per_elem=np.ascontiguousarray(sym)))
    if name == "jump":
        return O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=10.0 ** rng.uniform(-6, 6, ne))
    raise KeyError(name)


CASES = [
    ("kuhn", "const", "dirichlet"), ("quad", "const", "dirichlet"),
    ("kuhn_spe10", "spe10", "dirichlet"), ("quad_spe10", "spe10", "dirichlet"),
    ("kuhn", "sinusoid", "dirichlet"), ("kuhn", "sinusoid_comp", "dirichlet"), ("quad", "sinusoid", "dirichlet"),
    ("kuhn", "per_elem_sym", "dirichlet"), ("quad", "per_elem_sym", "dirichlet"),
    ("kuhn", "per_elem_sym", "neumann"), ("quad", "const", "neumann"),
    ("nvb", "const", "dirichlet"), ("nvb", "per_elem_sym", "dirichlet"), ("nvb", "jump", "neumann"),
    ("scrambled", "per_elem_sym", "dirichlet"), ("scrambled", "sinusoid", "dirichlet"),
    ("parallelogram", "per_elem_sym", "dirichlet"), ("parallelogram", "sinusoid", "neumann"),
]


@pytest.mark.parametrize("mesh,coef,bnd", CASES)
@pytest.mark.parametrize("threads", [1, 4])
def test_owner_walk_equals_primal_walk(mesh, coef, bnd, threads):
    et, coords, ev = _mesh(mesh)
    grid = O.Grid(et, coords, ev)
    kappa, A = _coefficients(coef, grid, np.random.default_rng(11))
    prm = O.params(O.BOUNDARY_NEUMANN if bnd == "neumann" else O.BOUNDARY_DIRICHLET)
    pat = grid.pattern()
    rp, col, ref = O.assemble(grid, kappa, A, prm, pattern=pat)
    _, _, got = O.assemble_owner(grid, kappa, A, prm, pattern=pat, threads=threads)
    assert np.array_equal(rp, pat[0]) and np.array_equal(col, pat[1])
    worst, ok = compare_rows(rp, got, ref, RTOL)
    assert ok, worst
    assert np.count_nonzero(ref) > 0
