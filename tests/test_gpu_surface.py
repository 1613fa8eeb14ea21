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
# HDD_EXAMPLES_BIN: another build of the examples, e.g. examples/bin_asan (make -C dune-hdd_amd asan)
EXE = os.path.join(os.environ.get("HDD_EXAMPLES_BIN") or os.path.join(ROOT, "examples", "bin"), "surface_main")


def test_surface_example_is_built():
    assert os.access(EXE, os.X_OK), "examples/bin/surface_main missing: run make -C dune-hdd_amd"


@pytest.fixture(scope="module")
def surface_run(tmp_path_factory):
    """one run of examples/surface_main; the parametric SPE10 channel / force boxes (testcases/spe10.hh) are
    handed over as a binary file"""
    d = str(tmp_path_factory.mktemp("surface"))
    ch, fo = O.spe10_channel_boxes()
    np.concatenate([[len(ch), len(fo)], ch.ravel(), fo.ravel()]).astype(np.float64).tofile(
        os.path.join(d, "spe10_boxes.bin"))
    r = subprocess.run([EXE, d], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r, d


@pytest.mark.gpu
def test_cpp_surface_against_oracle(surface_run):
    r, d = surface_run
    if True:
        assert "roundtrip 1" in r.stdout and "coupling(0,3) rejected" in r.stdout
        assert "batched operators 12 same 1" in r.stdout, r.stdout
        # the *_and_return_ptr / pb_get_* variants (block-swipdg.hh:602-690, 770-831): equal, own values, deletable
        assert "caller-owned copies 1" in r.stdout, r.stdout
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


def _ld(d, n, t=np.float64):
    return np.fromfile(os.path.join(d, n + ".bin"), dtype=t)


@pytest.mark.gpu
def test_cpp_reference_ctor_init_products(surface_run):
    """SWIPDG(grid_provider, boundary_cfg, problem, level, only_these_products) + init(out, prefix)
    (swipdg.hh:159-163, 206-217, 486): level 1 of the provider, the timing line, only the requested products
    available, the reference's error paths (base.hh:282-291, 370-377)."""
    r, d = surface_run
    out = r.stdout
    assert "  [swipdg] assembling... done (took " in out
    assert "available products: l2 penalty" in out
    assert "not requested: Product 'h1_semi' not available!" in out
    assert "before init: The user has to call init() before calling any other method!" in out
    assert "no products: Do not call get_product() if available_products() is empty!" in out
    assert "bad level: level 5 not in [0, 2)" in out
    assert "  [block] walking subdomains for the first time (block pattern, built at construction)... done (took " in out
    assert "  [block] walking subdomains for the second time... done (took " in out
    og = O.Grid(*O.kuhn_grid(16, 16, (-1, -1), (1, 1)))
    rp, col, val = O.assemble(og, O.scalar(), O.tensor(), O.params())
    assert np.array_equal(_ld(d, "lvl1_row_ptr", np.int64), rp)
    assert compare_rows(rp, _ld(d, "lvl1_affine"), val, 1e-12)[1]
    b = O.rhs_swipdg(og, force=O.esv2007_force())
    assert np.max(np.abs(_ld(d, "lvl1_rhs") - b)) <= 1e-12 * np.max(np.abs(b))


@pytest.mark.gpu
def test_cpp_block_local_discretization_product_functional(surface_run):
    """BlockSWIPDG::get_local_discretization(0) (block-swipdg.hh:761-768: SWIPDG on the local grid part,
    AllNeumann, ZeroBoundary), get_local_product(0, "l2") (612-618) and get_local_functional(0) (678-685)
    against the oracle on the subdomain's elements with an all-Neumann boundary."""
    r, d = surface_run
    assert "local discretization 0: layer local 1, dofs 384, purely neumann 1" in r.stdout
    assert "local functional 0: size 384 components 0" in r.stdout
    assert "local discretization 4 rejected" in r.stdout
    g = H.Grid.structured(H.SIMPLEX, 16, 16, (-1, -1), (1, 1), px=2, py=2)
    pc, pev, psd = g.connectivity()
    a0, b0 = g.subdomain_range(0, 1)
    sg = O.Grid(O.SIMPLEX, pc, pev[a0:b0])
    neu = O.params(boundary=O.BOUNDARY_NEUMANN)
    rp, col, val = O.assemble(sg, O.scalar(), O.tensor(), neu)
    assert np.array_equal(_ld(d, "ld0_row_ptr", np.int64), rp) and np.array_equal(_ld(d, "ld0_col", np.int32), col)
    assert compare_rows(rp, _ld(d, "ld0_affine"), val, 1e-12)[1]
    prp, _, pval = O.product(sg, O.PRODUCT_L2, prm=neu)
    assert np.array_equal(_ld(d, "lp0_row_ptr", np.int64), prp)
    assert compare_rows(prp, _ld(d, "lp0_l2"), pval, 1e-12)[1]
    b = O.rhs_swipdg(sg, force=O.esv2007_force(), prm=neu)
    lf = _ld(d, "lf0")
    assert np.max(np.abs(lf - b)) <= 1e-12 * np.max(np.abs(b))
    assert np.array_equal(lf, _ld(d, "lf0_from_ld"))     # the local discretization's rhs, bit for bit


@pytest.mark.gpu
def test_cpp_parametric_spe10(surface_run):
    """Parametric SPE10 Model1 (problems/spe10.hh:160-172, channel / force boxes of testcases/spe10.hh:31-251):
    affine part (1 + channel) and component channel with theta = -1.0*mu, the rhs with the kappa_1 x g_D,aff
    component, the elliptic product; GPU vs oracle at 1e-12.  freeze_parameter(0.5) is the reference's
    theta-lincomb; it equals a frozen-mu assembly exactly on rows whose element and neighbours lie outside the
    channel (inside, the penalty's kappa^- kappa^+ is assembled per component, as the reference does)."""
    r, d = surface_run
    assert "spe10 parametric 1 components 1 coefficient -1.0*mu rhs components 1 coefficient -1.0*mu" in r.stdout
    et, c, ev = O.kuhn_grid(100, 20, (0, 0), (5, 1))
    og = O.Grid(et, c, ev)
    cen = O.element_centers(c, ev)
    ch, fo = O.spe10_channel_boxes()
    chan = O.indicator_sum(cen, ch)     # make_sum of one-box Indicators (problems/spe10.hh:139-148)
    k_aff, k_1 = 1.0 + chan, chan
    perm = _ld(d, "spe10_perm")
    A = O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=O.checkerboard(cen, (0, 0), (5, 1), 100, 20, perm))
    pe = lambda v: O.scalar(O.FN_PER_ELEM, per_elem=np.ascontiguousarray(v))
    rp, col, va = O.assemble(og, pe(k_aff), A, O.params())
    _, _, v1 = O.assemble(og, pe(k_1), A, O.params())
    assert (k_1 != 0).sum() > 100
    assert compare_rows(rp, _ld(d, "spe10_affine"), va, 1e-12)[1]
    assert compare_rows(rp, _ld(d, "spe10_comp0"), v1, 1e-12)[1]
    fr = _ld(d, "spe10_frozen_0.5")
    assert compare_rows(rp, fr, va - 0.5 * v1, 1e-12)[1]
    _, _, vf = O.assemble(og, pe(k_aff - 0.5 * k_1), A, O.params())
    nb, _ = og.neighbors()
    quiet = (k_1 == 0) & np.all((nb < 0) | (k_1[np.maximum(nb, 0)] == 0), axis=1)
    rows = np.repeat(quiet, 3)
    for i in np.nonzero(rows)[0][::37]:
        s = slice(rp[i], rp[i + 1])
        assert np.array_equal(fr[s], vf[s]) or np.max(np.abs(fr[s] - vf[s])) <= 1e-12 * np.max(np.abs(vf[s]))
    assert not np.allclose(fr, vf)        # the channel rows differ: component-wise penalty
    b = O.rhs_swipdg(og, force=pe(O.indicator(cen, fo)), kappa=pe(k_aff), A=A, dirichlet=O.scalar(O.FN_CONST, 0.0))
    assert np.max(np.abs(_ld(d, "spe10_rhs") - b)) <= 1e-12 * np.max(np.abs(b))
    assert not _ld(d, "spe10_rhs_comp0").any()       # kappa_1 x (g_D = 0)
    _, _, e1 = O.product(og, O.PRODUCT_ELLIPTIC, kappa=pe(k_1), A=A)
    assert np.max(np.abs(_ld(d, "spe10_elliptic_comp0") - e1)) <= 1e-12 * np.max(np.abs(e1))


@pytest.mark.gpu
def test_cpp_spe10_flattop_channel(surface_run):
    """Spe10Model1 with the reference's default channel_boundary_layer (problems/spe10.hh:86: FlatTop's
    default, restated as 0.1): the channel is a sum of FlatTop functions (213-222) -- 1 + 0.9 channel, and the
    parametric split 1 + channel / channel -- against the oracle's FlatTop restatement at 1e-12 (parity
    unpinned: FlatTop is third-party)."""
    r, d = surface_run
    assert "spe10 flattop channel: components 1 order 3" in r.stdout
    et, c, ev = O.kuhn_grid(97, 21, (0, 0), (5, 1))   # mesh lines off the FlatTop discontinuities (surface_main)
    og = O.Grid(et, c, ev)
    cen = O.element_centers(c, ev)
    ch, _ = O.spe10_channel_boxes()
    boxes = np.column_stack([ch[:, :4], np.full((len(ch), 2), 0.1), ch[:, 4]])
    A = O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=O.checkerboard(cen, (0, 0), (5, 1), 100, 20, _ld(d, "spe10_perm")))
    for name, (cc, bb) in [("spe10ft_affine", (1.0, 0.9)), ("spe10ftp_affine", (1.0, 1.0)), ("spe10ftp_comp0", (0.0, 1.0))]:
        rp, col, ref = O.assemble(og, O.flattop(boxes, cc, bb), A, O.params())
        assert compare_rows(rp, _ld(d, name), ref, 1e-12, floor_frac=1e-10)[1], name
    assert np.count_nonzero(_ld(d, "spe10ftp_comp0")) > 0.05 * _ld(d, "spe10ftp_comp0").size   # the channel is there


@pytest.mark.gpu
def test_cpp_parametric_rhs_cross_terms(surface_run):
    """swipdg.hh:251-356 component structure: with kappa = kappa_aff + mu kappa_1 and g_D = g_aff + mu g_1 the
    rhs holds affine = L2Volume(f) + Dirichlet(kappa_aff, g_aff) and the components Dirichlet(kappa_aff, g_1)
    [mu], Dirichlet(kappa_1, g_aff) [mu], Dirichlet(kappa_1, g_1) [(mu)*(mu)]; b(0.7) = sum theta b."""
    r, d = surface_run
    assert "parametric rhs components 3 coefficients mu;mu;(mu)*(mu);" in r.stdout
    og = O.Grid(*O.kuhn_grid(8, 8, (-1, -1), (1, 1)))
    kx, ky = 4 * math.pi, 2 * math.pi
    k_aff = O.scalar(O.FN_SINUSOID, 1.0, 0.75, kx, ky, order=3)
    k_1 = O.scalar(O.FN_SINUSOID, 0.0, -0.75, kx, ky, order=3)
    g_aff = O.scalar(O.FN_SINUSOID, 0.25, 0.5, 1.0, 2.0, order=3)
    g_1 = O.scalar(O.FN_COS_PRODUCT, 0.7, 0.0, 1.5, 0.5, order=3)
    ref = [O.rhs_swipdg(og, force=O.esv2007_force(), kappa=k_aff, dirichlet=g_aff),
           O.rhs_swipdg(og, kappa=k_aff, dirichlet=g_1), O.rhs_swipdg(og, kappa=k_1, dirichlet=g_aff),
           O.rhs_swipdg(og, kappa=k_1, dirichlet=g_1)]
    got = [_ld(d, "prhs_affine")] + [_ld(d, "prhs_comp%d" % q) for q in range(3)]
    for g_, r_ in zip(got, ref):
        assert np.max(np.abs(g_ - r_)) <= 1e-12 * np.max(np.abs(r_))
    mu = 0.7
    frozen = ref[0] + mu * ref[1] + mu * ref[2] + mu * mu * ref[3]
    assert np.max(np.abs(_ld(d, "prhs_frozen_0.7") - frozen)) <= 1e-12 * np.max(np.abs(frozen))


@pytest.mark.gpu
def test_cpp_block_oversampled_discretization(surface_run):
    """BlockSWIPDG::get_oversampled_discretization(0, "dirichlet" / "neumann") (block-swipdg.hh:783-817) with
    oversampling_layers = 1 (testcases/base.hh:169): SWIPDG on subdomain 0 plus one ring of face neighbours,
    the whole boundary of that grid part Dirichlet / Neumann, ZeroBoundary(ESV2007) -- against the oracle on
    the same element set."""
    r, d = surface_run
    ids = _ld(d, "os0_ids", np.int64)
    assert "oversampled 0: %d elements (layers 1)" % ids.size in r.stdout and "oversampled robin rejected" in r.stdout
    g = H.Grid.structured(H.SIMPLEX, 16, 16, (-1, -1), (1, 1), px=2, py=2)
    pc, pev, psd = g.connectivity()
    a0, b0 = g.subdomain_range(0, 1)
    assert ids.size > b0 - a0 and np.array_equal(ids[ids < b0][:b0 - a0], np.arange(a0, b0))
    # one ring: every added element shares a face with subdomain 0
    loc = g.local()
    nb = loc.neighbors.T
    added = ids[(ids < a0) | (ids >= b0)]
    assert all(np.any((nb[e] >= a0) & (nb[e] < b0)) for e in added)
    sg = O.Grid(O.SIMPLEX, pc, pev[ids])
    for bt, kind in (("dirichlet", O.BOUNDARY_DIRICHLET), ("neumann", O.BOUNDARY_NEUMANN)):
        prm = O.params(boundary=kind)
        rp, col, val = O.assemble(sg, O.scalar(), O.tensor(), prm)
        assert np.array_equal(_ld(d, "os0_%s_row_ptr" % bt, np.int64), rp)
        assert np.array_equal(_ld(d, "os0_%s_col" % bt, np.int32), col)
        assert compare_rows(rp, _ld(d, "os0_%s_affine" % bt), val, 1e-12)[1]
        b = O.rhs_swipdg(sg, force=O.esv2007_force(), prm=prm)
        assert np.max(np.abs(_ld(d, "os0_%s_rhs" % bt) - b)) <= 1e-12 * np.max(np.abs(b))


@pytest.mark.gpu
def test_cpp_block_oversampled_discretization_3d(surface_run):
    """get_oversampled_discretization in 3d (block-swipdg.hh:783-817 is dimension-generic; VERDICT r02 missing
    #2): ESV2007 3d, Q2 on 4 x 3 x 3 hexahedra of [-1,1]^3, 2 x 1 x 1 subdomains, one oversampling layer.  The
    grid part is subdomain 0 (x-columns 0, 1) plus the face-neighbour x-column 2 -- a 3 x 3 x 3 box, so the Q_p
    oracle on that box (Dirichlet / Neumann on its whole boundary, ZeroBoundary(ESV2007)) is the reference."""
    r, d = surface_run
    ids = _ld(d, "os3_ids", np.int64)
    assert "oversampled 3d 0: 27 elements (layers 1)" in r.stdout
    g = H.Grid.structured3d((4, 3, 3), (-1, -1, -1), (1, 1, 1), p=(2, 1, 1), degree=2)
    coords, ev, _ = g.connectivity()
    lo, up, n = (-1.0, -1.0, -1.0), (0.5, 1.0, 1.0), (3, 3, 3)
    v0 = coords[ev[ids, 0]]
    ijk = np.rint((v0 - np.asarray(lo)) / (2.0 / np.array([4, 3, 3]))).astype(np.int64)
    assert ijk[:, 0].max() == 2
    lex = ijk[:, 0] + 3 * (ijk[:, 1] + 3 * ijk[:, 2])
    ei = np.empty(27, np.int64)
    ei[lex] = np.arange(27)
    q = O.QpGrid(3, 2, n, lo, up)
    for bt, kind in (("dirichlet", O.BOUNDARY_DIRICHLET), ("neumann", O.BOUNDARY_NEUMANN)):
        prm = O.qp_params(q, boundary=kind)
        rp, col, val = O.qp_assemble(q, O.scalar(), O.qp_tensor(), prm, elem_index=ei)
        assert np.array_equal(_ld(d, "os3_%s_row_ptr" % bt, np.int64), rp)
        assert np.array_equal(_ld(d, "os3_%s_col" % bt, np.int32), col)
        assert compare_rows(rp, _ld(d, "os3_%s_affine" % bt), val, 1e-12)[1]
        b = O.qp_rhs_swipdg(q, force=O.esv2007_force(3), prm=prm, elem_index=ei)
        assert np.max(np.abs(_ld(d, "os3_%s_rhs" % bt) - b)) <= 1e-12 * np.max(np.abs(b))


def _checksum(t):
    """sum_k bits[k] * (2k + 1) mod 2^64 over a device tensor (examples/surface_main.cpp: checksum)"""
    import torch
    bits = t.contiguous().view(torch.int64) if t.dtype == torch.float64 else t.to(torch.int64)
    h, chunk = 0, 1 << 26
    for k0 in range(0, bits.numel(), chunk):
        b = bits[k0:k0 + chunk]
        w = torch.arange(k0, k0 + b.numel(), device=b.device, dtype=torch.int64) * 2 + 1
        h = (h + int((b * w).sum().item())) % (1 << 64)
    return h


def _big(which, *extra):
    r = subprocess.run([EXE, "big", which, *extra], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("big ")][-1]
    f = line.split()
    kv = {f[i]: f[i + 1] for i in range(2, len(f) - 1, 2)}
    return kv


@pytest.mark.gpu
def test_cpp_full_size_c2_swipdg_device_pattern():
    """The reference-signature SWIPDG (swipdg.hh:159-163) at the full C2 size (3200 x 640 Kuhn, SPE10 checkerboard
    tensor): pattern built on the device, never downloaded; pattern and values bit-identical to the Python
    front-end's device pattern + assembly (checksums of the bit patterns)."""
    import torch
    kv = _big("c2")
    grid = H.Grid.structured(H.SIMPLEX, 3200, 640, (0, 0), (5, 1))
    loc = grid.local()
    perm = np.array([math.pow(10.0, -3.0 + 6.0 * math.fmod(0.618033988749895 * i, 1.0)) for i in range(2000)])
    k = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
    ctx = H.Context(0)
    dm = H.DeviceMesh(loc)
    dp = H.DevicePattern(loc, ctx=ctx, dmesh=dm, on_device=True)
    (v,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k))
    torch.cuda.synchronize()
    assert int(kv["nnz"]) == dp.nnz == 147386880
    assert int(kv["col_hash"]) == _checksum(dp.col)
    assert int(kv["val_hash"]) == _checksum(v)


@pytest.mark.gpu
def test_cpp_full_size_hex_q3_swipdg_device_pattern():
    """The same surface on ESV2007 3d, Q3 on 32^3 hexahedra (940 M nnz: the pattern exists only on the device)."""
    import torch
    n = 32
    kv = _big("hex", str(n))
    g = H.Grid.structured3d((n, n, n), (-1, -1, -1), (1, 1, 1), degree=3)
    loc = g.local()
    ctx = H.Context(0)
    dm = H.DeviceMesh(loc)
    dp = H.DevicePattern(loc, ctx=ctx, dmesh=dm, on_device=True)
    (v,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(dim=3))
    torch.cuda.synchronize()
    assert int(kv["order"]) == 3 and int(kv["nnz"]) == dp.nnz
    assert int(kv["col_hash"]) == _checksum(dp.col)
    assert int(kv["val_hash"]) == _checksum(v)


@pytest.mark.gpu
def test_cpp_c4_block_operators_batched():
    """BlockSWIPDG at C4's size and decomposition (3520 x 1200 Q1, 8 x 8 subdomains): all 288 local / coupling
    operators one by one and through extract_operators() (one batched device extraction), equal by checksums of
    row pointers, columns and values; the times go to the log (< 10 ms batched)."""
    r = subprocess.run([EXE, "big", "c4ops"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    print(r.stdout)
    line = [l for l in r.stdout.splitlines() if l.startswith("c4 ops batched")][-1]
    assert "288 operators" in line and line.endswith("equal 1"), line
