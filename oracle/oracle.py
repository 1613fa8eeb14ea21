"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end of the CPU oracle (``swipdg_oracle.c``), a restatement of dune-hdd's SWIPDG /
BlockSWIPDG stiffness assembly (reference: dune/hdd/linearelliptic/discretizations/swipdg.hh:206-512,
block-swipdg.hh:262-551).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / timed CPU baseline.

Also holds the oracle-side structured grid builders (the reference's Stuff::Grid::Providers::Cube /
StructuredGridFactory meshes, testcases/ESV2007.hh:123-129, testcases/spe10.hh:301-307) and the problem
data of the BASELINE configs (problems/ESV2007.hh:75-81, problems/OS2014.hh:63-76, problems/spe10.hh:
141-179) so that tests can build inputs without touching the product.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

SIMPLEX, CUBE = 0, 1
FN_CONST, FN_PER_ELEM, FN_SINUSOID = 0, 1, 2
TENSOR_CONST, TENSOR_ISO_PER_ELEM, TENSOR_SYM_PER_ELEM = 0, 1, 2
BOUNDARY_DIRICHLET, BOUNDARY_NEUMANN = 0, 1

# dune-gdt LocalEvaluation::SWIPDG::internal defaults for p = 1 (restated)
SIGMA_INNER_P1 = 8.0
SIGMA_BOUNDARY_P1 = 14.0


class MeshT(C.Structure):
    _fields_ = [("elem_type", C.c_int32), ("pad", C.c_int32), ("n_vertices", C.c_int64),
                ("coords", C.c_void_p), ("n_elements", C.c_int64), ("elem_vert", C.c_void_p)]


class ScalarT(C.Structure):
    _fields_ = [("kind", C.c_int32), ("order", C.c_int32), ("c", C.c_double), ("b", C.c_double),
                ("kx", C.c_double), ("ky", C.c_double), ("per_elem", C.c_void_p), ("table", C.c_void_p),
                ("n_table", C.c_int32), ("pad", C.c_int32)]


class TensorT(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad", C.c_int32), ("c", C.c_double * 3), ("per_elem", C.c_void_p)]


class ParamsT(C.Structure):
    _fields_ = [("sigma_inner", C.c_double), ("sigma_boundary", C.c_double), ("beta", C.c_double),
                ("boundary_kind", C.c_int32), ("vol_order_override", C.c_int32),
                ("face_order_override", C.c_int32), ("pad", C.c_int32)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.or_grid_create.restype = C.c_void_p
        L.or_grid_create.argtypes = [C.POINTER(MeshT)]
        L.or_grid_destroy.argtypes = [C.c_void_p]
        L.or_grid_neighbor.restype = C.c_int64
        L.or_grid_neighbor.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        L.or_grid_neighbor_face.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        L.or_pattern_nnz.restype = C.c_int64
        L.or_pattern_nnz.argtypes = [C.c_void_p]
        L.or_pattern.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_assemble_swipdg.argtypes = [C.c_void_p, C.POINTER(ScalarT), C.POINTER(TensorT),
                                         C.POINTER(ParamsT), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_block_numbering.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.or_assemble_block_swipdg.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(ScalarT),
                                               C.POINTER(TensorT), C.POINTER(ParamsT), C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_rhs_l2.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.or_error_norms_esv2007.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                             C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.or_quadrature.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        _LIB = L
    return _LIB


def _ptr(a):
    return None if a is None else a.ctypes.data


# ----------------------------------------------------------------------------------------------------
# structured grids (oracle side)
# ----------------------------------------------------------------------------------------------------
def cube_grid(nx, ny, lower=(0.0, 0.0), upper=(1.0, 1.0)):
    """SGrid-like nx x ny quads, lexicographic elements, Dune cube vertex order (00,10,01,11)."""
    xs = np.linspace(lower[0], upper[0], nx + 1)
    ys = np.linspace(lower[1], upper[1], ny + 1)
    X, Y = np.meshgrid(xs, ys)                       # [ny+1][nx+1]
    coords = np.stack([X.ravel(), Y.ravel()], axis=1).copy()
    j, i = np.meshgrid(np.arange(ny), np.arange(nx), indexing="ij")
    v00 = (j * (nx + 1) + i).ravel()
    ev = np.stack([v00, v00 + 1, v00 + nx + 1, v00 + nx + 2], axis=1).astype(np.int32)
    return CUBE, coords, ev


def kuhn_grid(nx, ny, lower=(0.0, 0.0), upper=(1.0, 1.0)):
    """Kuhn triangulation (StructuredGridFactory::createSimplexGrid): per square (00,10,11),(00,01,11)."""
    _, coords, q = cube_grid(nx, ny, lower, upper)
    t0 = np.stack([q[:, 0], q[:, 1], q[:, 3]], axis=1)
    t1 = np.stack([q[:, 0], q[:, 2], q[:, 3]], axis=1)
    ev = np.stack([t0, t1], axis=1).reshape(-1, 3).astype(np.int32)
    return SIMPLEX, coords, ev


def element_centers(coords, ev):
    return coords[ev].mean(axis=1)


def checkerboard(centers, lower, upper, nxc, nyc, values):
    """dune-stuff Checkerboard: cell of the element centre (row-major x fastest)."""
    cx = np.clip(((centers[:, 0] - lower[0]) / (upper[0] - lower[0]) * nxc).astype(np.int64), 0, nxc - 1)
    cy = np.clip(((centers[:, 1] - lower[1]) / (upper[1] - lower[1]) * nyc).astype(np.int64), 0, nyc - 1)
    return values[cy * nxc + cx]


def indicator(points, boxes):
    """dune-stuff Indicator (playground/functions/indicator.hh, third-party: restated, unverifiable here) as
    problems/spe10.hh:144, 157 use it: per entity, the value of the first closed box [lower, upper] that
    contains the entity centre, 0 if none.  points [n][2], boxes [k][5] = lx, ly, ux, uy, value."""
    out = np.zeros(points.shape[0])
    done = np.zeros(points.shape[0], bool)
    for lx, ly, ux, uy, v in np.asarray(boxes, np.float64).reshape(-1, 5):
        m = ~done & (points[:, 0] >= lx) & (points[:, 0] <= ux) & (points[:, 1] >= ly) & (points[:, 1] <= uy)
        out[m] = v
        done |= m
    return out


def indicator_sum(points, boxes):
    """The Spe10 channel at channel_boundary_layer = 0 (problems/spe10.hh:139-148): make_sum of one-box
    Indicators, i.e. per entity the sum of the values of every closed box containing the entity centre."""
    out = np.zeros(points.shape[0])
    for lx, ly, ux, uy, v in np.asarray(boxes, np.float64).reshape(-1, 5):
        m = (points[:, 0] >= lx) & (points[:, 0] <= ux) & (points[:, 1] >= ly) & (points[:, 1] <= uy)
        out[m] += v
    return out


def spe10_channel_boxes():
    """The parametric SPE10 channel of testcases/spe10.hh:38-251 (105 boxes, channel_boundary_layer = 0, so
    Indicator functions: problems/spe10.hh:213-218) and the three force boxes (testcases/spe10.hh:31-37),
    from the committed fixture tests/golden/spe10_parametric_channel.json (make_spe10_channel.py).
    Returned as (channel [105][5], force [3][5])."""
    import json
    path = os.path.join(os.path.dirname(_HERE), "tests", "golden", "spe10_parametric_channel.json")
    d = json.load(open(path))
    return np.array(d["channel"], np.float64), np.array(d["force"], np.float64)


def spe10_synthetic_permeability(nxc=100, nyc=20, seed=10):
    """Stand-in for perm_case1.dat (absent): log10 k ~ U(-3, 3) on the 100x20 Model1 checkerboard."""
    rng = np.random.default_rng(seed)
    return 10.0 ** rng.uniform(-3.0, 3.0, size=nxc * nyc)


# ----------------------------------------------------------------------------------------------------
# oracle calls
# ----------------------------------------------------------------------------------------------------
class Grid:
    def __init__(self, elem_type, coords, ev):
        self.elem_type = int(elem_type)
        self.coords = np.ascontiguousarray(coords, dtype=np.float64)
        self.ev = np.ascontiguousarray(ev, dtype=np.int32)
        self.nb = 3 if self.elem_type == SIMPLEX else 4
        self.nf = self.nb
        self.ne = self.ev.shape[0]
        self._m = MeshT(self.elem_type, 0, self.coords.shape[0], _ptr(self.coords), self.ne, _ptr(self.ev))
        self.h = lib().or_grid_create(C.byref(self._m))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_grid_destroy(self.h)
            self.h = None

    def neighbors(self):
        L = lib()
        out = np.empty((self.ne, self.nf), np.int64)
        nf = np.empty((self.ne, self.nf), np.int64)
        for e in range(self.ne):
            for f in range(self.nf):
                out[e, f] = L.or_grid_neighbor(self.h, e, f)
                nf[e, f] = L.or_grid_neighbor_face(self.h, e, f)
        return out, nf

    def pattern(self, elem_index=None):
        L = lib()
        nnz = L.or_pattern_nnz(self.h)
        row_ptr = np.empty(self.ne * self.nb + 1, np.int64)
        col = np.empty(nnz, np.int32)
        ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
        L.or_pattern(self.h, _ptr(ei), _ptr(row_ptr), _ptr(col))
        return row_ptr, col


def scalar(kind=FN_CONST, c=1.0, b=0.0, kx=0.0, ky=0.0, per_elem=None, order=0, table=None):
    tab = None if table is None else np.ascontiguousarray(table, np.float64).reshape(-1, 7)
    s = ScalarT(kind, order, c, b, kx, ky, _ptr(per_elem), _ptr(tab), 0 if tab is None else tab.shape[0], 0)
    s._keep = (per_elem, tab)
    return s


def flattop(boxes, c=0.0, b=1.0, order=3):
    """c + b * sum of dune-stuff FlatTop functions (or_flattop; boxes [k][7] = lx, ly, ux, uy, dx, dy, value)."""
    return scalar(FN_FLATTOP, c, b, order=order, table=boxes)


def flattop_at(box, x, y):
    L = lib()
    L.or_flattop.restype = C.c_double
    L.or_flattop.argtypes = [C.c_void_p, C.c_double, C.c_double]
    b = np.ascontiguousarray(box, np.float64)
    return L.or_flattop(_ptr(b), float(x), float(y))


def tensor(kind=TENSOR_CONST, c=(1.0, 0.0, 1.0), per_elem=None):
    t = TensorT(kind, 0, (C.c_double * 3)(*c), _ptr(per_elem))
    t._keep = per_elem
    return t


def params(boundary=BOUNDARY_DIRICHLET, sigma_inner=SIGMA_INNER_P1, sigma_boundary=SIGMA_BOUNDARY_P1,
           beta=1.0, vol_order=-1, face_order=-1):
    return ParamsT(sigma_inner, sigma_boundary, beta, boundary, vol_order, face_order, 0)


def assemble(grid, kappa, A, prm, elem_index=None, pattern=None):
    """Monolithic SWIPDG component matrix (CSR arrays).  elem_index permutes element numbering."""
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    row_ptr, col = pattern if pattern is not None else grid.pattern(ei)
    val = np.empty(col.shape[0], np.float64)
    lib().or_assemble_swipdg(grid.h, C.byref(kappa), C.byref(A), C.byref(prm), _ptr(ei), _ptr(row_ptr),
                             _ptr(col), _ptr(val))
    return row_ptr, col, val


def assemble_owner(grid, kappa, A, prm, pattern=None, threads=1):
    """Owner-computes OpenMP variant of assemble() (same values up to summation order)."""
    L = lib()
    L.or_assemble_swipdg_owner.argtypes = [C.c_void_p] * 8 + [C.c_int]
    row_ptr, col = pattern if pattern is not None else grid.pattern()
    val = np.empty(col.shape[0], np.float64)
    L.or_assemble_swipdg_owner(grid.h, C.byref(kappa), C.byref(A), C.byref(prm), None, _ptr(row_ptr), _ptr(col),
                               _ptr(val), int(threads))
    return row_ptr, col, val


def block_numbering(grid, subdomain, n_sub):
    sd = np.ascontiguousarray(subdomain, np.int32)
    ei = np.empty(grid.ne, np.int64)
    lib().or_block_numbering(grid.h, _ptr(sd), int(n_sub), _ptr(ei))
    return ei


def assemble_block(grid, subdomain, n_sub, kappa, A, prm):
    """BlockSWIPDG global matrix in block numbering; returns (elem_index, row_ptr, col, val)."""
    sd = np.ascontiguousarray(subdomain, np.int32)
    ei = block_numbering(grid, sd, n_sub)
    row_ptr, col = grid.pattern(ei)
    val = np.empty(col.shape[0], np.float64)
    lib().or_assemble_block_swipdg(grid.h, _ptr(sd), int(n_sub), C.byref(kappa), C.byref(A), C.byref(prm),
                                   _ptr(ei), _ptr(row_ptr), _ptr(col), _ptr(val))
    return ei, row_ptr, col, val


def rhs_esv2007(grid, elem_index=None, force_order=3):
    b = np.empty(grid.ne * grid.nb, np.float64)
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    lib().or_rhs_l2(grid.h, 0, force_order, _ptr(ei), _ptr(b))
    return b


def error_norms_esv2007(grid, u, elem_index=None, order=10):
    u = np.ascontiguousarray(u, np.float64)
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    l2, h1 = C.c_double(), C.c_double()
    lib().or_error_norms_esv2007(grid.h, _ptr(u), _ptr(ei), order, C.byref(l2), C.byref(h1))
    return l2.value, h1.value


def quadrature(elem_type, order):
    x = np.empty((256, 2)); w = np.empty(256)
    n = lib().or_quadrature(elem_type, order, _ptr(x), _ptr(w))
    return x[:n].copy(), w[:n].copy()


def to_scipy(row_ptr, col, val, n=None):
    import scipy.sparse as sp
    n = n or (row_ptr.shape[0] - 1)
    return sp.csr_matrix((val, col, row_ptr), shape=(row_ptr.shape[0] - 1, n))


def esv2007_eoc(grid, prm, elem_index=None):
    """Assemble + solve ESV2007 (kappa=1, A=I, f = 1/2 pi^2 cos cos, AllDirichlet) and return the error
    norms (L2, H1 semi) -- the solution-level quantities test/linearelliptic-swipdg.hh:267-290 computes."""
    import scipy.sparse.linalg as spla
    rp, col, val = assemble(grid, scalar(FN_CONST, 1.0), tensor(TENSOR_CONST), prm, elem_index)
    A = to_scipy(rp, col, val)
    b = rhs_esv2007(grid, elem_index)
    u = spla.spsolve(A.tocsc(), b)
    return error_norms_esv2007(grid, u, elem_index)


# ------------------------------------------------------------------------------------------------------
# DG Q_p on structured 2D/3D cube grids (swipdg_oracle_qp.c): the C5 configuration (p = 3, 3D)
# ------------------------------------------------------------------------------------------------------
# dune-gdt LocalEvaluation::SWIPDG::internal::{inner,boundary}_sigma(p) (restated)
SIGMA_INNER = {0: 8.0, 1: 8.0, 2: 20.0, 3: 38.0}
SIGMA_BOUNDARY = {0: 14.0, 1: 14.0, 2: 38.0, 3: 74.0}


def sigma_inner(p):
    return SIGMA_INNER.get(p, 50.0)


def sigma_boundary(p):
    return SIGMA_BOUNDARY.get(p, 99.0)


class QpGridT(C.Structure):
    _fields_ = [("dim", C.c_int32), ("degree", C.c_int32), ("n", C.c_int64 * 3),
                ("lower", C.c_double * 3), ("upper", C.c_double * 3)]


class QpTensorT(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad", C.c_int32), ("c", C.c_double * 6), ("per_elem", C.c_void_p)]


def _qp_lib():
    L = lib()
    if not getattr(L, "_qp_ready", False):
        L.or_qp_num_elements.restype = C.c_int64
        L.or_qp_pattern_nnz.restype = C.c_int64
        for nm in ("or_qp_pattern", "or_qp_assemble", "or_qp_rhs_esv2007", "or_qp_error_esv2007"):
            getattr(L, nm).restype = C.c_int
        VP = C.c_void_p
        L.or_qp_num_elements.argtypes = [VP]
        L.or_qp_pattern_nnz.argtypes = [VP]
        L.or_qp_pattern.argtypes = [VP, VP, VP, VP]
        L.or_qp_assemble.argtypes = [VP, VP, VP, VP, VP, VP, VP, VP]
        L.or_qp_rhs_esv2007.argtypes = [VP, C.c_int, VP, VP]
        L.or_qp_error_esv2007.argtypes = [VP, VP, VP, C.c_int, VP, VP]
        L._qp_ready = True
    return L


class QpGrid:
    """Structured grid of n[0] x n[1] (x n[2]) axis-aligned cubes on [lower, upper] carrying DG Q_p;
    element id = i + n0 (j + n1 k) (lexicographic, x fastest)."""

    def __init__(self, dim, p, n, lower, upper):
        self.dim, self.p = int(dim), int(p)
        n = list(n) + [1] * (3 - len(n))
        lo = list(lower) + [0.0] * (3 - len(lower))
        up = list(upper) + [1.0] * (3 - len(upper))
        self.t = QpGridT(self.dim, self.p, (C.c_int64 * 3)(*n), (C.c_double * 3)(*lo), (C.c_double * 3)(*up))
        self.nb = (self.p + 1) ** self.dim
        self.ne = int(_qp_lib().or_qp_num_elements(C.byref(self.t)))
        if self.ne < 0:
            raise ValueError("invalid Q_p grid")

    def pattern(self, elem_index=None):
        L = _qp_lib()
        nnz = L.or_qp_pattern_nnz(C.byref(self.t))
        rp = np.empty(self.ne * self.nb + 1, np.int64)
        col = np.empty(nnz, np.int32)
        ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
        L.or_qp_pattern(C.byref(self.t), _ptr(ei), _ptr(rp), _ptr(col))
        return rp, col


def qp_tensor(kind=TENSOR_CONST, c=None, per_elem=None, dim=3):
    if c is None:
        c = (1.0, 0.0, 1.0) if dim == 2 else (1.0, 0.0, 0.0, 1.0, 0.0, 1.0)
    cc = list(c) + [0.0] * (6 - len(c))
    t = QpTensorT(kind, 0, (C.c_double * 6)(*cc), _ptr(per_elem))
    t._keep = per_elem
    return t


def qp_params(grid, boundary=BOUNDARY_DIRICHLET, vol_order=-1, face_order=-1):
    return ParamsT(sigma_inner(grid.p), sigma_boundary(grid.p), 1.0 / (grid.dim - 1), boundary, vol_order,
                   face_order, 0)


def qp_assemble(grid, kappa, A, prm, elem_index=None, pattern=None):
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    rp, col = pattern if pattern is not None else grid.pattern(ei)
    val = np.empty(col.shape[0], np.float64)
    rc = _qp_lib().or_qp_assemble(C.byref(grid.t), C.byref(kappa), C.byref(A), C.byref(prm), _ptr(ei), _ptr(rp),
                                  _ptr(col), _ptr(val))
    if rc:
        raise ValueError("or_qp_assemble failed")
    return rp, col, val


def qp_esv2007_errors(grid, elem_index=None):
    """Assemble + solve the d-dimensional ESV2007 problem (u = prod cos(pi x_a/2)) on the Q_p grid;
    returns (L2, H1-semi) errors."""
    import scipy.sparse.linalg as spla
    rp, col, val = qp_assemble(grid, scalar(FN_CONST, 1.0), qp_tensor(dim=grid.dim), qp_params(grid), elem_index)
    b = np.empty(grid.ne * grid.nb)
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    _qp_lib().or_qp_rhs_esv2007(C.byref(grid.t), 3 if grid.dim == 2 else 3, _ptr(ei), _ptr(b))
    u = spla.spsolve(to_scipy(rp, col, val).tocsc(), b)
    l2, h1 = C.c_double(), C.c_double()
    _qp_lib().or_qp_error_esv2007(C.byref(grid.t), _ptr(u), _ptr(ei), 2 * grid.p + 6, C.byref(l2), C.byref(h1))
    return l2.value, h1.value


# ------------------------------------------------------------------------------------------------------
# right-hand sides (SWIPDG::init() functionals, swipdg.hh:251-347)
# ------------------------------------------------------------------------------------------------------
FN_COS_PRODUCT = 3
FN_FLATTOP = 4


def esv2007_force(dim=2):
    """Testcase1Force (problems/ESV2007.hh:78), integration order 3; 3d: (d pi^2 / 4) prod cos(pi x_a / 2)."""
    k = 0.5 * np.pi
    return scalar(FN_COS_PRODUCT, 0.25 * dim * np.pi ** 2, k if dim == 3 else 0.0, k, k, order=3)


def rhs_swipdg(grid, force=None, kappa=None, A=None, dirichlet=None, neumann=None, prm=None, elem_index=None):
    L = lib()
    L.or_rhs_swipdg.argtypes = [C.c_void_p] + [C.c_void_p] * 5 + [C.c_void_p, C.c_void_p, C.c_void_p]
    b = np.empty(grid.ne * grid.nb, np.float64)
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    kappa = kappa or scalar()
    A = A or tensor()
    prm = prm or params()
    ref = lambda x: None if x is None else C.byref(x)
    L.or_rhs_swipdg(grid.h, ref(force), ref(kappa), ref(A), ref(dirichlet), ref(neumann), ref(prm), _ptr(ei),
                    _ptr(b))
    return b


def qp_rhs_swipdg(grid, force=None, kappa=None, A=None, dirichlet=None, neumann=None, prm=None, elem_index=None):
    L = _qp_lib()
    L.or_qp_rhs_swipdg.restype = C.c_int
    L.or_qp_rhs_swipdg.argtypes = [C.c_void_p] * 9
    b = np.empty(grid.ne * grid.nb, np.float64)
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    kappa = kappa or scalar()
    A = A or qp_tensor(dim=grid.dim)
    prm = prm or qp_params(grid)
    ref = lambda x: None if x is None else C.byref(x)
    L.or_qp_rhs_swipdg(C.byref(grid.t), ref(force), ref(kappa), ref(A), ref(dirichlet),
                       ref(neumann), ref(prm), _ptr(ei), _ptr(b))
    return b


# ------------------------------------------------------------------------------------------------------
# products (swipdg.hh:358-508)
# ------------------------------------------------------------------------------------------------------
PRODUCT_L2, PRODUCT_H1_SEMI, PRODUCT_ELLIPTIC, PRODUCT_BOUNDARY_L2, PRODUCT_PENALTY = 0, 1, 2, 3, 4


def volume_pattern(ne, nb, elem_index=None):
    """Block-diagonal (volume) pattern of the l2 / h1_semi / elliptic / boundary_l2 products."""
    rp = np.arange(ne * nb + 1, dtype=np.int64) * nb
    blk = np.arange(ne, dtype=np.int64)                     # row block k holds element k's DoFs
    col = (blk[:, None, None] * nb + np.arange(nb)[None, None, :]).repeat(nb, axis=1).reshape(-1).astype(np.int32)
    return rp, col


def product(grid, kind, kappa=None, A=None, prm=None, elem_index=None):
    L = lib()
    L.or_product.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 7
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    rp, col = volume_pattern(grid.ne, grid.nb) if kind != PRODUCT_PENALTY else grid.pattern(ei)
    val = np.empty(col.shape[0])
    ref = lambda x: C.byref(x)
    L.or_product(grid.h, kind, ref(kappa or scalar()), ref(A or tensor()), ref(prm or params()), _ptr(ei), _ptr(rp),
                 _ptr(col), _ptr(val))
    return rp, col, val


def qp_product(grid, kind, kappa=None, A=None, prm=None, elem_index=None):
    L = _qp_lib()
    L.or_qp_product.restype = C.c_int
    L.or_qp_product.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 7
    ei = None if elem_index is None else np.ascontiguousarray(elem_index, np.int64)
    rp, col = volume_pattern(grid.ne, grid.nb) if kind != PRODUCT_PENALTY else grid.pattern(ei)
    val = np.empty(col.shape[0])
    ref = lambda x: C.byref(x)
    L.or_qp_product(C.byref(grid.t), kind, ref(kappa or scalar()),
                    ref(A or qp_tensor(dim=grid.dim)), ref(prm or qp_params(grid)), _ptr(ei), _ptr(rp), _ptr(col),
                    _ptr(val))
    return rp, col, val
