#!/usr/bin/env python3
"""Measured runs of the other BASELINE configurations (the driver's bench line is C2 in bench.py):

  c3  OS2014 parametric, [-1,1]^2, 1024^2 Kuhn triangles (2.10 M elements, 6.29 M DoFs, 75.5 M nnz per
      component): (i) assembly of the affine part + the mu-component (smooth kappa, integration order 3,
      problems/OS2014.hh:63-76) and (ii) 128 theta-lincombs A(mu_s) = A_aff + mu_s A_1, mu ~ U(0.1, 1)
      (seed 14), materialised in HBM.
  c4  SPE10-like 3520 x 1200 Q1 quads on [0,5]x[0,1], 8x8 subdomains (block numbering), synthetic
      permeability, single GPU (the 8-GPU sharded form is bench.py --gpus 8 on the strip workload).
  c5  ESV2007 3d structured, n^3 axis-aligned hexahedra on [-1,1]^3 (default n = 64: 262,144 elements,
      16.8 M DoFs, 7.4 G nnz, 59 GB of values resident in HBM), DG Q3 (64 basis functions), kappa = 1, A = I,
      AllDirichlet; f64 MFMA kernel (hex_qp.hip).  The device pattern build is timed separately (the
      reference builds its pattern outside init(), swipdg.hh:169).
  c5s ESV2007 3d 256^3 (16.8 M hexahedra, 1.07 G DoFs, 4.8e11 nnz = 3.8 TB of values: larger than HBM), Q3,
      streamed-slab mode: the grid is cut into x-slabs (rank-local meshes with face ghosts)
      whose row blocks are assembled in turn into one rotating value buffer; the time is one pass over all
      slabs (values of earlier slabs are overwritten -- a throughput measurement, nothing is skipped).
  f   the SURVEY.md 8(f) rows on the C2 mesh (3200 x 640 Kuhn P1, synthetic SPE10 tensor): device pattern
      build (hdd_pattern_elem_ptr_device + hdd_pattern_fill_device), the SWIPDG right-hand side
      (L2Volume(ESV2007 force, order 3) + DirichletBoundarySWIPDG(g_D = 1)), and the products l2 / h1_semi /
      elliptic (element-diagonal volume pattern) and the SWIPDG penalty (full pattern).  Bytes per call are
      the algorithmic ones: outputs written once + the element records read.
  ops BlockSWIPDG operator extraction (get_local_operator / get_coupling_operator, block-swipdg.hh:612-690)
      on the C4 layout (Q1, 8 x 8 subdomains; --n sets nx, default 3520): every local and every coupling
      operator extracted on the device from the assembled global matrix (hdd_block_operator_map_device +
      hdd_block_operator_values_device), end to end; the round-2 host maps timed beside it.
Prints one JSON line per config."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))


def timed(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e-3


def c3(args):
    import torch
    import hdd_amd as H
    n = args.n or 1024
    grid = H.Grid.structured(H.SIMPLEX, n, n, (-1, -1), (1, 1))
    loc = grid.local()
    ctx = H.Context(0)
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    kx, ky = 4 * math.pi, 2 * math.pi
    fns = [H.scalar_fn(H.FN_SINUSOID, 1.0, 0.75, kx, ky, order=3), H.scalar_fn(H.FN_SINUSOID, 0.0, -0.75, kx, ky, order=3)]
    vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda") for _ in range(2)]
    t_asm = timed(lambda: H.assemble(ctx, dm, dp, fns, H.tensor_fn(), vals=vals), args.steps, args.warmup)
    mus = np.random.default_rng(14).uniform(0.1, 1.0, args.samples)
    theta = np.stack([np.ones_like(mus), mus], 1)          # A(mu) = A_aff + mu A_1 (ParameterFunctional "mu")
    out = torch.empty((args.samples, dp.nnz), dtype=torch.float64, device="cuda")
    t_lc = timed(lambda: H.affine_lincomb(ctx, vals, theta, out=out), max(1, args.steps // 4), 1)
    dofs = 3 * loc.n_own
    nif = int((loc.neighbors[:, :] >= 0).sum()) // 2
    alg = 8 * dp.nnz * 2 + loc.n_own * (84 + 16) + 12 * nif
    lc_bytes = args.samples * 8 * dp.nnz + 2 * 8 * dp.nnz * math.ceil(args.samples / 32)   # 32 samples per pass
    return dict(config="c3_os2014_multiquery_kuhn%dx%d" % (n, n), dofs=dofs, nnz_per_component=dp.nnz,
                components=2, assembly_ms=t_asm * 1e3, assembled_dofs_per_s=dofs / t_asm,
                assembly_alg_GBps=alg / t_asm / 1e9, samples=args.samples, lincomb_ms=t_lc * 1e3,
                lincomb_matrices_per_s=args.samples / t_lc, lincomb_GBps=lc_bytes / t_lc / 1e9)


def c4(args):
    import torch
    import hdd_amd as H
    nx, ny = (args.n or 3520), (args.n and args.n * 1200 // 3520) or 1200
    grid = H.Grid.structured(H.CUBE, nx, ny, (0, 0), (5, 1), px=8, py=8)
    loc = grid.local()
    rng = np.random.default_rng(10)
    k = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, 10.0 ** rng.uniform(-3, 3, 2000))).cuda()
    ctx = H.Context(0)
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
    fn = lambda: H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k), vals=vals)
    t = timed(fn, args.steps, args.warmup)
    nif = int((loc.neighbors >= 0).sum()) // 2
    alg = 8 * dp.nnz + loc.n_own * (104 + 8) + 12 * nif
    dofs = 4 * loc.n_own
    return dict(config="c4_spe10_q1_%dx%d_block8x8" % (nx, ny), dofs=dofs, nnz=dp.nnz, assembly_ms=t * 1e3,
                assembled_dofs_per_s=dofs / t, alg_GBps=alg / t / 1e9, roofline_frac=alg / t / 8e12)


def f(args):
    import torch
    import hdd_amd as H
    nx, ny = (args.n or 3200), (args.n and args.n // 5) or 640
    grid = H.Grid.structured(H.SIMPLEX, nx, ny, (0, 0), (5, 1))
    loc = grid.local()
    rng = np.random.default_rng(10)
    k = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, 10.0 ** rng.uniform(-3, 3, 2000))).cuda()
    ctx = H.Context(0)
    dm = H.DeviceMesh(loc)
    ne, N = loc.n_own, 3 * loc.n_own
    res = dict(config="f_rows_spe10_kuhn%dx%d" % (nx, ny), dofs=N)
    # device pattern (timed by wall clock around the synchronising builder)
    gid = torch.from_numpy(loc.global_id).cuda()
    ep = torch.empty(ne + 1, dtype=torch.int64, device="cuda")
    nnz = H.C.c_int64()
    s = torch.cuda.current_stream().cuda_stream

    def pattern():
        H._check(H.lib().hdd_pattern_elem_ptr_device(ctx.h, H.C.byref(dm.t), 3, ep.data_ptr(), H.C.byref(nnz),
                                                    H.C.c_void_p(s)))
        H._check(H.lib().hdd_pattern_fill_device(ctx.h, H.C.byref(dm.t), 3, gid.data_ptr(), ep.data_ptr(),
                                                 rp.data_ptr(), col.data_ptr(), H.C.c_void_p(s)))
    pattern_probe = H.DevicePattern(loc, ctx=ctx, dmesh=dm, on_device=True)
    rp = torch.empty(N + 1, dtype=torch.int64, device="cuda")
    col = torch.empty(pattern_probe.nnz, dtype=torch.int32, device="cuda")
    t = timed(pattern, args.steps, args.warmup)
    pb = 8 * (N + 1) + 4 * pattern_probe.nnz + 8 * (ne + 1) + ne * (12 + 8)
    res.update(pattern_ms=t * 1e3, pattern_GBps=pb / t / 1e9, pattern_nnz=pattern_probe.nnz)
    # right-hand side
    ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
    out = torch.empty(N, dtype=torch.float64, device="cuda")
    fn = lambda: H.rhs(ctx, dm, force=H.esv2007_force(), kappa=H.scalar_fn(H.FN_CONST, 1.0), tensor=ten,
                       dirichlet=H.scalar_fn(H.FN_CONST, 1.0), out=out)
    t = timed(fn, args.steps, args.warmup)
    rb = 8 * N + ne * (48 + 12 + 8)
    res.update(rhs_ms=t * 1e3, rhs_GBps=rb / t / 1e9)
    # products
    dpv = H.DevicePattern(loc, volume=True)
    dpf = H.DevicePattern(loc)
    # products read the vertex-indexed geometry (12 B of vertex ids per triangle + each 16-byte vertex row
    # once); the elliptic / penalty products the tensor (8 B), the penalty product the neighbour ids + face
    # info (16 B); values written once
    nv = dm.vertex_coords.shape[0] if dm.vertex_coords is not None else 0
    for name, kind, dp in (("l2", H.PRODUCT_L2, dpv), ("h1_semi", H.PRODUCT_H1_SEMI, dpv),
                           ("elliptic", H.PRODUCT_ELLIPTIC, dpv), ("penalty", H.PRODUCT_PENALTY, dpf)):
        o = torch.empty(dp.nnz, dtype=torch.float64, device="cuda")
        fn = lambda: H.product(ctx, dm, kind, dp, kappa=H.scalar_fn(H.FN_CONST, 1.0), tensor=ten, out=o)
        t = timed(fn, args.steps, args.warmup)
        per_elem = 12 + (8 if kind in (H.PRODUCT_ELLIPTIC, H.PRODUCT_PENALTY) else 0) + \
            (16 if kind == H.PRODUCT_PENALTY else 0)
        b = 8 * dp.nnz + ne * per_elem + 16 * nv
        res.update({name + "_ms": t * 1e3, name + "_GBps": b / t / 1e9, name + "_values_GBps": 8 * dp.nnz / t / 1e9,
                    name + "_nnz": dp.nnz})
    return res


def ops(args):
    """all local + coupling operators of the C4 layout: (i) the device path -- hdd_block_operator_map_device +
    hdd_block_operator_values_device per operator from the device pattern, end to end (every launch, the nnz
    read-back of each map included), and with the nnz known in advance (block_operator_nnz, one host pass per
    mesh, timed separately): no synchronisation inside; (ii) the round-2 host maps (hdd_block_operator_map)
    for comparison, timed once."""
    import torch
    import hdd_amd as H
    nx = args.n or 3520
    ny = nx * 1200 // 3520
    grid = H.Grid.structured(H.CUBE, nx, ny, (0, 0), (5, 1), px=8, py=8)
    loc = grid.local()
    ctx = H.Context(0)
    dm, dp = H.DeviceMesh(loc), H.DevicePattern(loc)
    rng = np.random.default_rng(10)
    k = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, 10.0 ** rng.uniform(-3, 3, 2000))).cuda()
    (vals,) = H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k))
    pairs = []
    for ss in range(64):
        sx, sy = divmod(ss, 8)
        pairs += [(ss, nn) for nn in [ss] + [(sx + dx) * 8 + sy + dy for dx, dy in ((-1, 0), (1, 0), (0, -1), (0, 1))
                                             if 0 <= sx + dx < 8 and 0 <= sy + dy < 8]]
    t0 = time.perf_counter()
    nnz_of = H.block_operator_nnz(loc)
    t_nnz = time.perf_counter() - t0

    def run(known):
        out = [H.block_operator(ctx, grid, dp, [vals], ss, nn, nnz=nnz_of[(ss, nn)] if known else None)
               for ss, nn in pairs]
        torch.cuda.synchronize()
        return out

    res = {}
    for known in (False, True):
        run(known)   # warm-up (allocator, scan scratch)
        ts = []
        for _ in range(max(3, args.steps // 4)):
            t0 = time.perf_counter()
            out = run(known)
            ts.append(time.perf_counter() - t0)
        res["device_ms_" + ("known_nnz" if known else "sync_nnz")] = float(np.median(ts)) * 1e3
    n = sum(int(o[1].numel()) for o in out)
    assert n == sum(nnz_of[p] for p in pairs)
    # (iii) all operators in one batched call (hdd_block_operators_map_device / _values_device)
    for known in (False, True):
        H.block_operators(ctx, grid, dp, [vals], pairs, nnz=nnz_of if known else None)
        torch.cuda.synchronize()
        ts = []
        for _ in range(max(3, args.steps // 4)):
            t0 = time.perf_counter()
            b = H.block_operators(ctx, grid, dp, [vals], pairs, nnz=nnz_of if known else None)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res["batched_ms_" + ("known_nnz" if known else "sync_nnz")] = float(np.median(ts)) * 1e3
    for p, o in zip(pairs, out):
        assert all(torch.equal(x, y) for x, y in zip(b[p][:2], o[:2])) and torch.equal(b[p][2][0], o[2][0])
    rp, col, _ = dp.host
    t0 = time.perf_counter()
    for ss, nn in pairs:
        c = H.C.c_int64()
        H._check(H.lib().hdd_block_operator_map(grid.h, ss, nn, H._p(rp), H._p(col), None, None, None, H.C.byref(c)))
        src = np.empty(c.value, np.int64)
        ocol = np.empty(c.value, np.int32)
        orp = np.empty(4 * grid.ne + 1, np.int64)
        H._check(H.lib().hdd_block_operator_map(grid.h, ss, nn, H._p(rp), H._p(col), H._p(orp), H._p(ocol), H._p(src),
                                                H.C.byref(c)))
    t_host = time.perf_counter() - t0
    return dict(config="ops_block_swipdg_q1_%dx%d_8x8" % (nx, ny), operators=len(pairs), values=n, global_nnz=dp.nnz,
                nnz_host_pass_s=t_nnz, host_map_s=t_host, **res,
                device_GBps_known_nnz=(8 + 8 + 4) * n / (res["device_ms_known_nnz"] * 1e-3) / 1e9,
                batched_GBps_known_nnz=(8 + 8 + 4) * n / (res["batched_ms_known_nnz"] * 1e-3) / 1e9)


def c5(args):
    import torch
    import hdd_amd as H
    n, deg = (args.n or 64), args.degree
    grid = H.Grid.structured3d((n, n, n), (-1, -1, -1), (1, 1, 1), degree=deg)
    loc = grid.local()
    ctx = H.Context(0)
    dm = H.DeviceMesh(loc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dp = H.DevicePattern(loc, ctx=ctx, dmesh=dm, on_device=True)
    torch.cuda.synchronize()
    t_pat = time.perf_counter() - t0
    vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
    prm = H.params_for(deg, 3)
    fn = lambda: H.assemble(ctx, dm, dp, [H.scalar_fn(H.FN_CONST, 1.0)], H.tensor_fn(dim=3), prm, vals=vals)
    t = timed(fn, args.steps, args.warmup)
    nb = grid.nb
    nbr = loc.neighbors
    n_inner = int((nbr >= 0).sum())                 # interior (element, face) pairs = 2 nif
    nif, nbf = n_inner // 2, int((nbr == H.NBR_DIRICHLET).sum())
    nq1v, nq1f = deg, deg + 1                        # reference integrand orders 2(p-1) / 2p
    nq, nqf = nq1v ** 3, nq1f ** 2
    # F = ne 2 nb^2 nq d + nif 24 nb^2 nqf + nbf 6 nb^2 nqf (reference quadrature)
    alg_flops = loc.n_own * 2 * nb * nb * nq * 3 + nif * 24 * nb * nb * nqf + nbf * 6 * nb * nb * nqf
    # executed MFMA work (v_mfma_f64_16x16x4: 2048 flop).  hex_q3_kernel (HDD_VARIANT=32), whole element = 4 waves:
    # volume 27 k-steps x 4 row tiles per wave; every face runs its rows in the layout rotated to its normal,
    # so the [V] part takes 1 row tile (4 k-steps) per wave; the [N] part 4 tiles x 4 k-steps in every wave
    # on x / y faces and in one wave only on z faces (column skip) -> x/y: 80 (S) + 80 (E, inner) per face,
    # z: 32 (S) + 32 (E)
    nbr_own = nbr[:, loc.own_begin:loc.own_end]
    xy_inner = int((nbr_own[:4] >= 0).sum()); xy_dir = int((nbr_own[:4] == H.NBR_DIRICHLET).sum())
    z_inner = int((nbr_own[4:] >= 0).sum()); z_dir = int((nbr_own[4:] == H.NBR_DIRICHLET).sum())
    # (HDD_VARIANT selects the register kernel only in the ablation build, HDD_AMD_LIB=.../libhdd_abl.so)
    legacy = ("abl" in os.path.basename(H.LIB_PATH)
              and int(os.environ.get("HDD_VARIANT", "0") or 0, 0) & H.VARIANT_HEX_Q3_REGISTER)
    if deg != 3:
        n_mfma = 0
    elif legacy:
        n_mfma = (loc.n_own * 4 * 108 + (xy_inner + xy_dir) * 80 + xy_inner * 80 + (z_inner + z_dir) * 32
                  + z_inner * 32)
    else:
        # hex_q3g_kernel: per 16-element group, each of the 64 row waves runs 8 x 4 (self, 32 terms) +
        # 6 x 2 x 4 (face blocks, 8 terms) MFMAs, boundary faces included (zero coefficients)
        n_mfma = (loc.n_own + 15) // 16 * 64 * 80
    mfma_flops = 2048 * n_mfma
    alg_bytes = 8 * dp.nnz + loc.n_own * (24 * 8 + 8 + 6 * 4)
    dofs = nb * loc.n_own
    # roofline: the EXECUTED f64 MFMA work against the 78.6 TF/s MFMA peak and the value stream against the HBM
    # peak.  The 8(d) reference-quadrature count is only a count here: the closed-form rows skip work the
    # reference's quadrature does, so a rate built from it can exceed the peak and is not roofline evidence.
    return dict(config="c5_esv2007_3d_q%d_%d^3" % (deg, n), dofs=dofs, nnz=dp.nnz, values_GB=8 * dp.nnz / 1e9,
                pattern_build_s=t_pat, assembly_ms=t * 1e3, assembled_dofs_per_s=dofs / t,
                alg_GBps=alg_bytes / t / 1e9, hbm_frac=alg_bytes / t / 8e12,
                values_written_GBps=8 * dp.nnz / t / 1e9, hbm_write_frac=8 * dp.nnz / t / 8e12,
                mfma_exec_TFLOPs=mfma_flops / t / 1e12, fp64_mfma_peak_TF=78.6, mfma_frac=mfma_flops / t / 78.6e12,
                ref_quadrature_TFLOP_count=alg_flops / 1e12)


def c5s(args):
    import torch
    import hdd_amd as H
    n, deg, slabs = (args.n or 256), args.degree, args.slabs
    grid = H.Grid.structured3d((n, n, n), (-1, -1, -1), (1, 1, 1), p=(slabs, 1, 1), degree=deg)
    ctx = H.Context(0)
    prm = H.params_for(deg, 3)
    t0 = time.perf_counter()
    parts = []
    for sl in range(slabs):
        loc = grid.local(sl, sl + 1)
        dm = H.DeviceMesh(loc)
        ep = torch.empty(loc.n_own + 1, dtype=torch.int64, device="cuda")
        nnz = H.C.c_int64()
        H._check(H.lib().hdd_pattern_elem_ptr_device(ctx.h, H.C.byref(dm.t), grid.nb, ep.data_ptr(),
                                                    H.C.byref(nnz), None), "hdd_pattern_elem_ptr_device")
        csr = H.CsrT(grid.nb * loc.n_own, grid.ne * grid.nb, nnz.value, None, None, ep.data_ptr())
        nbr = loc.neighbors[:, loc.own_begin:loc.own_end]
        parts.append(dict(dm=dm, ep=ep, csr=csr, nnz=nnz.value, n_own=loc.n_own,
                          inner=int((nbr >= 0).sum()), dirichlet=int((nbr == H.NBR_DIRICHLET).sum())))
        loc.coords = loc.neighbors = None   # host copies no longer needed
    t_setup = time.perf_counter() - t0
    vals = torch.empty(max(p["nnz"] for p in parts), dtype=torch.float64, device="cuda")
    kap = H.ScalarFn(H.FN_CONST, 0, 1.0, 0.0, 0.0, 0.0, None)
    ten = H.tensor_fn(dim=3)
    ptrs = (H.C.c_void_p * 1)(vals.data_ptr())
    s = torch.cuda.current_stream().cuda_stream

    def sweep():
        for p in parts:
            H._check(H.lib().hdd_swipdg_assemble(ctx.h, H.C.byref(p["dm"].t), H.C.byref(kap), 1, H.C.byref(ten),
                                                 H.C.byref(prm), H.C.byref(p["csr"]), ptrs, H.C.c_void_p(s)),
                     "hdd_swipdg_assemble")
    t = timed(sweep, max(1, args.steps // 5), 1)
    nnz = sum(p["nnz"] for p in parts)
    dofs = grid.ne * grid.nb
    n_own = sum(p["n_own"] for p in parts)
    inner = sum(p["inner"] for p in parts)
    nif, nbf = inner // 2, sum(p["dirichlet"] for p in parts)
    nq, nqf, nb = deg ** 3, (deg + 1) ** 2, grid.nb
    alg_flops = n_own * 2 * nb * nb * nq * 3 + nif * 24 * nb * nb * nqf + nbf * 6 * nb * nb * nqf
    return dict(config="c5s_esv2007_3d_q%d_%d^3_streamed_%d_slabs" % (deg, n, slabs), dofs=dofs, nnz=nnz,
                values_TB=8 * nnz / 1e12, rotating_buffer_GB=8 * vals.numel() / 1e9, setup_s=t_setup,
                assembly_s=t, assembled_dofs_per_s=dofs / t, values_written_GBps=8 * nnz / t / 1e9,
                hbm_write_frac=8 * nnz / t / 8e12, ref_quadrature_TFLOP_count=alg_flops / 1e12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c3", "c4"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--degree", type=int, default=3)
    ap.add_argument("--slabs", type=int, default=64)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    for c in args.configs:
        print(json.dumps(dict(c3=c3, c4=c4, c5=c5, c5s=c5s, f=f, ops=ops)[c](args)), flush=True)


if __name__ == "__main__":
    main()
