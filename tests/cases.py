"""Shared test inputs: the BASELINE configurations at test sizes, built twice -- once through the oracle's
own grid builders (oracle/oracle.py) and once through the product (hdd_amd) -- plus comparison helpers.

Coefficients (reference files):
  ESV2007  kappa = 1, A = I                                    problems/ESV2007.hh:75-81
  SPE10    kappa = 1 (+0.9*channel, empty), A = k_cell * I,    problems/spe10.hh:141-179
           k_cell from perm_case1.dat -- ABSENT, synthetic log10 k ~ U(-3,3), seed 10
  OS2014   kappa_aff = 1 + 0.75 sin(4 pi (x + y/2)),           problems/OS2014.hh:63-76
           kappa_1 = -0.75 sin(4 pi (x + y/2)), theta_1 = mu, integration_order 3
"""
import math

import numpy as np

import oracle as O

SPE10_LOWER, SPE10_UPPER = (0.0, 0.0), (5.0, 1.0)
OS2014_KX, OS2014_KY = 4.0 * math.pi, 2.0 * math.pi


def os2014_components():
    """(c, b, kx, ky) of the affine part and the single mu-component."""
    return [(1.0, 0.75, OS2014_KX, OS2014_KY), (0.0, -0.75, OS2014_KX, OS2014_KY)]


def compare_rows(row_ptr, got, ref, rtol=1e-12, floor_frac=0.0):
    """max over rows of max_j |got - ref| / max_j |ref|  (SURVEY 8(c) tolerance: <= 1e-12).  floor_frac > 0:
    rows whose scale is below floor_frac * max|ref| are scaled by that floor instead -- for coefficients that
    vanish outside a support (FlatTop), where a row of entries ~1e-60 against exact zeros is rounding of
    where a quadrature point falls at the support's edge, not a wrong entry."""
    got = np.asarray(got); ref = np.asarray(ref)
    n = row_ptr.shape[0] - 1
    rows = np.repeat(np.arange(n), np.diff(row_ptr))
    scale = np.zeros(n)
    np.maximum.at(scale, rows, np.abs(ref))
    err = np.zeros(n)
    np.maximum.at(err, rows, np.abs(got - ref))
    if floor_frac > 0 and ref.size:
        scale = np.maximum(scale, floor_frac * np.max(np.abs(ref)))
    scale[scale == 0] = 1.0
    worst = float(np.max(err / scale)) if n else 0.0
    return worst, worst <= rtol


def oracle_kappa_const(c=1.0):
    return O.scalar(O.FN_CONST, c)


def oracle_sinusoid(c, b, kx, ky, order=3):
    return O.scalar(O.FN_SINUSOID, c, b, kx, ky, order=order)


def compare_rows_fast(row_ptr, got, ref, rtol=1e-12):
    """compare_rows for large matrices with non-empty rows: segment maxima by np.maximum.reduceat."""
    got = np.asarray(got); ref = np.asarray(ref)
    starts = np.asarray(row_ptr[:-1], np.int64)
    err = np.maximum.reduceat(np.abs(got - ref), starts)
    scale = np.maximum.reduceat(np.abs(ref), starts)
    scale[scale == 0] = 1.0
    worst = float(np.max(err / scale)) if starts.size else 0.0
    return worst, worst <= rtol
