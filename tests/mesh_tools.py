"""Test-side mesh builders that the product has no structured generator for."""
import numpy as np

import oracle as O


def nvb_mesh(n0, refines, lower=(-1.0, -1.0), upper=(1.0, 1.0)):
    """Newest-vertex bisection of the Kuhn triangulation of an n0 x n0 square grid (refinement edge of the
    initial triangles = the diagonal).  2 bisections per 'refineStepsForHalf' reproduce the ALUGrid
    conforming ladder the reference's ESV2007 ALU tests run on (testcases/ESV2007.hh:48-59, base.hh:92-103):
    with n0 = 4 and refines = 2 + 2k this gives the 128 / 512 / 2048 / 8192-triangle levels whose error
    norms match test/linearelliptic-swipdg-expectations_esv2007_2daluconform.cxx:32-37."""
    _, coords, q = O.cube_grid(n0, n0, lower, upper)
    coords = [tuple(c) for c in coords]
    idx = {c: i for i, c in enumerate(coords)}
    tris = []
    for v00, v10, v01, v11 in q:
        tris.append((v00, v11, v10))      # (a, b, newest): refinement edge a-b
        tris.append((v00, v11, v01))

    def mid(a, b):
        c = ((coords[a][0] + coords[b][0]) / 2, (coords[a][1] + coords[b][1]) / 2)
        if c not in idx:
            idx[c] = len(coords)
            coords.append(c)
        return idx[c]

    for _ in range(refines):
        new = []
        for a, b, c in tris:
            m = mid(a, b)
            new.append((a, c, m))
            new.append((c, b, m))
        tris = new
    return O.SIMPLEX, np.array(coords, dtype=np.float64), np.array(tris, dtype=np.int32)


def affine_quad_mesh(nx, ny, M, c):
    """Structured quads pushed through x -> M x + c: every element a general parallelogram (non-diagonal
    Jacobian), Dune vertex order kept."""
    et, coords, ev = O.cube_grid(nx, ny, (0, 0), (1, 1))
    return et, coords @ np.asarray(M, float).T + np.asarray(c, float), ev


def scrambled_quad_mesh(nx, ny, seed):
    """Structured quads whose elements are renumbered by random symmetries of the reference square (Dune
    cube vertex order kept valid: rotations and reflections), so neighbouring elements see each other's
    faces under every twin-face id and orientation; then a shear."""
    et, coords, ev = O.cube_grid(nx, ny, (0, 0), (1, 1))
    rng = np.random.default_rng(seed)
    # the 8 symmetries of the square as permutations of the lexicographic vertices (00, 10, 01, 11)
    syms = [(0, 1, 2, 3), (1, 3, 0, 2), (3, 2, 1, 0), (2, 0, 3, 1),     # rotations
            (1, 0, 3, 2), (2, 3, 0, 1), (0, 2, 1, 3), (3, 1, 2, 0)]     # reflections
    pick = rng.integers(0, 8, ev.shape[0])
    ev = np.stack([ev[k, list(syms[p])] for k, p in enumerate(pick)]).astype(np.int32)
    coords = coords @ np.array([[1.1, 0.3], [0.0, 0.8]]).T
    return et, coords, ev
