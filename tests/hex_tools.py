"""Helpers for the Q_p hexahedral (C5) tests: map the product's subdomain-major element numbering onto the
oracle's lexicographic numbering of the same structured grid."""
import numpy as np


def lex_to_product(grid, n, lower, upper):
    """elem_index for the oracle: oracle element (lexicographic i + n0 (j + n1 k)) -> product global id."""
    coords, ev, _ = grid.connectivity()
    v0 = coords[ev[:, 0]]                                   # vertex 0 = lower corner of every hexahedron
    h = (np.asarray(upper, float) - np.asarray(lower, float)) / np.asarray(n, float)
    ijk = np.rint((v0 - np.asarray(lower, float)) / h).astype(np.int64)
    lex = ijk[:, 0] + n[0] * (ijk[:, 1] + n[1] * ijk[:, 2])
    elem_index = np.empty(grid.ne, np.int64)
    elem_index[lex] = np.arange(grid.ne)
    return elem_index
