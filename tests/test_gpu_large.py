"""Full-size parity (BASELINE configurations at their quoted sizes): the HIP assembly against the CPU
oracle entry-wise on the whole C2 (3200 x 640 Kuhn P1, 147 M nnz) and C4 (3520 x 1200 Q1 in the 8 x 8
block numbering, 338 M nnz) matrices, plus the size-independent invariants on the device.  The oracle runs
its owner-computes OpenMP variant (same integrands and rules as the sequential walk the small-size tests
use; values equal up to summation order), so the comparison takes seconds.

Tolerance (fp64): per row, max_j |a_gpu - a_oracle| <= 1e-12 * max_j |a_oracle|."""
import os

import numpy as np
import pytest

import oracle as O
from cases import SPE10_LOWER, SPE10_UPPER, compare_rows_fast

H = pytest.importorskip("hdd_amd")
pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def _run(ctx, et, nx, ny, px, py):
    import torch
    perm = O.spe10_synthetic_permeability()
    grid = H.Grid.structured(et, nx, ny, SPE10_LOWER, SPE10_UPPER, px=px, py=py)
    local = grid.local()
    k = local.checkerboard(SPE10_LOWER, SPE10_UPPER, 100, 20, perm)
    dm = H.DeviceMesh(local)
    dp = H.DevicePattern(local)
    (val,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)],
                        H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=torch.from_numpy(k).cuda()))
    torch.cuda.synchronize()
    got = val.cpu().numpy()
    rp, col, _ = dp.host
    # the oracle on the product's own element order (block numbering) and pattern: coordinates and
    # element->vertex connectivity are rebuilt from the rank-local mesh
    coords, ev, _ = grid.connectivity()
    og = O.Grid(et, coords, ev)
    _, _, ref = O.assemble_owner(og, O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k), O.params(),
                           pattern=(rp, col), threads=THREADS)
    return rp, col, got, ref


@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_full_size_against_oracle(ctx, cfg):
    et, nx, ny, p = (H.SIMPLEX, 3200, 640, 1) if cfg == "c2" else (H.CUBE, 3520, 1200, 8)
    rp, col, got, ref = _run(ctx, et, nx, ny, p, p)
    assert col.shape[0] == (147386880 if cfg == "c2" else 337768960)
    worst, ok = compare_rows_fast(rp, got, ref, 1e-12)
    assert ok, worst


def test_full_size_os2014_components(ctx):
    """C3 at its quoted size (1024^2 Kuhn triangles, 75.5 M nnz per component): the affine part and the
    mu-component (sinusoid kappa, integration order 3) in one call, entry-wise against the oracle."""
    import torch
    from cases import os2014_components
    grid = H.Grid.structured(H.SIMPLEX, 1024, 1024, (-1, -1), (1, 1))
    local = grid.local()
    comps = os2014_components()
    dm, dp = H.DeviceMesh(local), H.DevicePattern(local)
    vals = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_SINUSOID, c, b, kx, ky, order=3) for c, b, kx, ky in comps],
                      H.tensor_fn())
    torch.cuda.synchronize()
    rp, col, _ = dp.host
    assert col.shape[0] == 75460608
    coords, ev, _ = grid.connectivity()
    og = O.Grid(H.SIMPLEX, coords, ev)
    for (c, b, kx, ky), v in zip(comps, vals):
        _, _, ref = O.assemble_owner(og, O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=3), O.tensor(O.TENSOR_CONST),
                                     O.params(), pattern=(rp, col), threads=THREADS)
        worst, ok = compare_rows_fast(rp, v.cpu().numpy(), ref, 1e-12)
        assert ok, worst
