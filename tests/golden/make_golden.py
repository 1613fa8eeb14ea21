"""Generates tests/golden/*.npz: small golden CSR fixtures of the SWIPDG stiffness components.

The reference cannot be built or run here; the fixtures are produced by the CPU oracle
(oracle/), which is pinned against the reference's own expectation tables (ESV2007 SGrid Q1 and ALU P1
solution-error norms reproduced to all 3 significant figures, tests/test_oracle_pinning.py).  They freeze
the oracle's entry-wise output so the GPU path and later oracle edits are checked against fixed data.

Run:  python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "oracle"), os.path.join(HERE, "..")]
import oracle as O  # noqa: E402
from mesh_tools import nvb_mesh  # noqa: E402

SPE10 = ((0.0, 0.0), (5.0, 1.0))


def save(name, et, coords, ev, kappas, tensor_kind, tensor_c=(1.0, 0.0, 1.0), tensor_per_elem=None,
         boundary=O.BOUNDARY_DIRICHLET):
    g = O.Grid(et, coords, ev)
    prm = O.params(boundary)
    out = dict(elem_type=et, coords=coords, elem_vert=ev, boundary=boundary, n_comp=len(kappas),
               tensor_kind=tensor_kind, tensor_c=np.array(tensor_c, float),
               tensor_per_elem=np.zeros(1) if tensor_per_elem is None else tensor_per_elem)
    if tensor_kind == O.TENSOR_CONST:
        T = O.tensor(O.TENSOR_CONST, tensor_c)
    elif tensor_kind == O.TENSOR_ISO_PER_ELEM:
        T = O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=tensor_per_elem)
    else:
        T = O.tensor(O.TENSOR_SYM_PER_ELEM, per_elem=np.ascontiguousarray(tensor_per_elem.T))
    for q, (kind, c, b, kx, ky, order) in enumerate(kappas):
        rp, col, val = O.assemble(g, O.scalar(kind, c, b, kx, ky, order=order), T, prm)
        out["row_ptr"], out["col"] = rp, col
        out["val_%d" % q] = val
        out["kappa_%d" % q] = np.array([kind, c, b, kx, ky, order], float)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "nnz", out["col"].shape[0])


def main():
    one = (O.FN_CONST, 1.0, 0.0, 0.0, 0.0, 0)
    # C1: ESV2007 SGrid 16x16, Q1
    et, c, ev = O.cube_grid(16, 16, (-1, -1), (1, 1))
    save("c1_esv2007_sgrid16_q1", et, c, ev, [one], O.TENSOR_CONST)
    # ESV2007 on the ALU-conforming ladder level 0 (128 triangles, newest vertex bisection)
    et, c, ev = nvb_mesh(4, 2)
    save("esv2007_alu128_p1", et, c, ev, [one], O.TENSOR_CONST)
    # SPE10 (synthetic permeability) 100x20 quads and Kuhn triangles
    perm = O.spe10_synthetic_permeability()
    for name, mk in (("spe10_100x20_q1", O.cube_grid), ("spe10_100x20_p1", O.kuhn_grid)):
        et, c, ev = mk(100, 20, *SPE10)
        k = O.checkerboard(O.element_centers(c, ev), SPE10[0], SPE10[1], 100, 20, perm)
        save(name, et, c, ev, [one], O.TENSOR_ISO_PER_ELEM, tensor_per_elem=k)
    # OS2014: affine part + mu component on an 8x8 Kuhn grid (smooth kappa, integration order 3)
    et, c, ev = O.kuhn_grid(8, 8, (-1, -1), (1, 1))
    kx, ky = 4 * math.pi, 2 * math.pi
    save("os2014_kuhn8_p1", et, c, ev, [(O.FN_SINUSOID, 1.0, 0.75, kx, ky, 3), (O.FN_SINUSOID, 0.0, -0.75, kx, ky, 3)],
         O.TENSOR_CONST)


if __name__ == "__main__":
    main()
