#!/usr/bin/env python3
"""bench.py -- assembled DoFs/s of the SWIPDG global stiffness (BASELINE.json metric) on MI355X.

Workload (BASELINE.json configs[1]): SPE10 model1, SWIPDG p=1 on a Kuhn-triangulated
3200 x 640 grid over [0,5]x[0,1] (ALUConform-like simplices): 4,096,000 triangles, 12,288,000 DoFs,
147,386,880 nnz; A = k_cell I on the 100x20 Model1 checkerboard with a SYNTHETIC permeability
(perm_case1.dat is absent: log10 k ~ U(-3,3), seed 10), diffusion factor 1, AllDirichlet.

A "step" = one assembly of the global stiffness values (Q+1 = 1 value array) on the pre-built pattern, from
mesh + coefficient arrays resident in HBM (the reference times the same region: SWIPDG::init()'s walk, the
pattern being built in the constructor, swipdg.hh:169, 216-217, 485-486).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): weak scaling, block-SWIPDG strip
partition -- rank r owns the r-th 3200 x 640 strip of a (3200 N) x 640 grid over [0,5N]x[0,1] (the
checkerboard widened to 100N x 20 cells) and assembles its own rows (owner-computes, no reduction); the
face-halo records (vertex coordinates + tensor of the ghost elements) are exchanged with RCCL send/recv
inside every step.

--workload c4 (BASELINE.json configs[3], not the metric's line): SPE10 3520 x 1200 Q1 quads on [0,5]x[0,1]
with 8 x 8 subdomains (block numbering), strong scaling -- rank r of N owns subdomains [64 r / N, 64 (r+1) / N)
(columns of the 8 x 8 layout) and assembles its rows; same halo exchange.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=["c2", "c4"],
                    help="c2 (default, the metric's line): SPE10 P1 Kuhn strips, weak scaling; c4: SPE10 "
                         "3520x1200 Q1 with 8x8 subdomains sharded over the ranks in subdomain columns "
                         "(BASELINE.json configs[3]), strong scaling")
    ap.add_argument("--nx", type=int, default=0, help="c2: squares per strip in x per rank (3200); c4: 3520")
    ap.add_argument("--ny", type=int, default=0, help="c2: 640; c4: 1200")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU work of the baseline sample")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06", "traffic.json"),
                    help="PMC traffic summary (scripts/traffic_summary.py); used only when its build_id matches the "
                         "timed libhdd_amd.so")
    ap.add_argument("--kernel-times-json", default=os.path.join(ROOT, "profiles", "r06", "kernel_times.json"),
                    help="rocprofv3 kernel durations per workload (scripts/kernel_times.py); used only when its build_id "
                         "matches the timed libhdd_amd.so and its kernel the dispatched one")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearsal of the N-rank path on one GPU (host-staged halo)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: exchange the halo before the whole assembly instead of overlapping it "
                         "with the interior tiles")
    ap.add_argument("--probe-last", action="store_true",
                    help="run the attainable-bandwidth probe after the timed steps (default: before the warmup)")
    ap.add_argument("--halo", default="step", choices=["step", "once"],
                    help="N>1: exchange the face halo in every step (default) or once at setup -- the mesh and "
                         "the coefficients are static, so a re-assembly needs no exchange (SURVEY.md 8(e))")
    return ap.parse_args()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(nx_full, ny, target_s, cube=False):
    """The CPU oracle timed on a bounded strip of the same workload (nxs x ny Kuhn squares over
    [0, 5 nxs/nx_full] x [0,1], checkerboard of the full domain), SURVEY.md 8(d) protocol: 1 warm-up, median
    of 5.  `value`: the sequential element walk with per-entry CSR binary search, 1 thread -- the reference's
    walk() runs without TBB (swipdg.hh:485).  `omp_value`: the owner-computes OpenMP variant of the same
    integrands on the host cores this process may use (16 on the GPU box's share)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    perm = O.spe10_synthetic_permeability()
    lower = (0.0, 0.0)
    # The OpenMP leg uses this job's CPU share, not the node: the GPU box exports OMP_NUM_THREADS (16 = the
    # host cores allotted to one GPU of the node; nproc / the affinity set show the whole machine's CPUs there,
    # and the pool rules forbid sizing worker pools by them).  Without OMP_NUM_THREADS: the affinity set.
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS") or 0) or affinity)

    def run(nxs, reps=5, omp=0):
        upper = (5.0 * nxs / nx_full, 1.0)
        et, c, ev = (O.cube_grid if cube else O.kuhn_grid)(nxs, ny, lower, upper)
        k = O.checkerboard(O.element_centers(c, ev), (0.0, 0.0), (5.0, 1.0), 100, 20, perm)
        g = O.Grid(et, c, ev)
        rp, col = g.pattern()
        kap, ten, prm = O.scalar(O.FN_CONST, 1.0), O.tensor(O.TENSOR_ISO_PER_ELEM, per_elem=k), O.params()
        fn = (lambda: O.assemble_owner(g, kap, ten, prm, pattern=(rp, col), threads=omp)) if omp else \
             (lambda: O.assemble(g, kap, ten, prm, pattern=(rp, col)))
        fn()                                                    # warm-up
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return float(np.median(ts)), g.ne * (4 if cube else 3)

    t_cal, _ = run(25, reps=1)
    per_rep = target_s / 6.0                                   # warm-up + 5 timed runs ~ target_s
    nxs = int(min(nx_full, max(25, 25 * per_rep / max(t_cal, 1e-6))))
    t, dofs = run(nxs)
    t_omp, _ = run(nxs, omp=threads)
    return dict(value=dofs / t, unit="DoFs/s", cores=1, kind="port",
                sample="CPU oracle (oracle/swipdg_oracle.c, sequential element walk + per-entry CSR binary "
                       "search, 1 thread, median of 5 after 1 warm-up) on a %d x %d %s strip of the %s "
                       "workload = %d DoFs (%.3f s per assembly)"
                       % (nxs, ny, "Q1 quad" if cube else "Kuhn", "C4" if cube else "C2", dofs, t),
                omp_value=dofs / t_omp, omp_cores=threads,
                omp_sample="owner-computes OpenMP variant of the same integrands, %d threads (OMP_NUM_THREADS=%s: "
                           "the job's host-core share; %d CPUs in the affinity set), same strip, median of 5 "
                           "(%.3f s per assembly)" % (threads, os.environ.get("OMP_NUM_THREADS", "unset"), affinity,
                                                      t_omp),
                cpu_model=_cpu_model(), host_cpus=os.cpu_count())


def attainable_hbm(torch, nbytes=1 << 30, reps=None):
    """Attainable HBM bandwidth on this box, measured in the same run ('also report attainable
    BW from a device copy kernel'): a device-to-device copy (reads + writes) and a fill (writes only) of a
    1 GiB buffer, HIP events around `reps` back-to-back launches after one warm-up; GB/s of bytes moved."""
    reps = reps or int(os.environ.get("HDD_BENCH_PROBE_REPS", "25"))
    a = torch.empty(nbytes // 8, dtype=torch.float64, device="cuda").fill_(1.0)
    b = torch.empty_like(a)
    out = {}
    for name, fn, moved in (("copy", lambda: b.copy_(a), 2 * nbytes), ("fill", lambda: b.fill_(2.0), nbytes)):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_gbs"] = moved * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    return out


def lib_build_id():
    """sha256 prefix of the timed libhdd_amd.so: PMC traffic files are stamped with it, and a traffic figure
    measured on another build is not reported."""
    import hashlib
    import hdd_amd as H
    try:
        return hashlib.sha256(open(H.LIB_PATH, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import hdd_amd as H
    from hdd_amd.halo import gloo_host_comm, rccl_comm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    gpu = local_rank if args.backend == "nccl" else 0
    torch.cuda.set_device(gpu)
    # N > 1: every device synchronisation runs under this deadline (hdd_amd.watchdog): a lost or stalled peer ends the
    # rank with a report of the step stage that did not complete instead of a hang
    deadline = float(os.environ.get("HDD_BENCH_DEADLINE", "60"))
    if world > 1:
        import datetime
        # control plane only (barriers, the max-over-ranks timing, the RCCL id broadcast); the halo itself is
        # moved by the library (hdd_comm: RCCL send/recv, or the host-staged rehearsal transport)
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(120.0, 2 * deadline)))

    c4 = args.workload == "c4"
    if c4:   # strong scaling: one 3520 x 1200 Q1 mesh, 8 x 8 subdomains, rank r owns a subdomain-column range
        nx, ny = (args.nx or 3520), (args.ny or 1200)
        lower, upper = (0.0, 0.0), (5.0, 1.0)
        grid = H.Grid.structured(H.CUBE, nx, ny, lower, upper, px=8, py=8)
        if world > grid.n_sub:
            raise SystemExit("c4 shards 64 subdomains: at most 64 ranks")
        ncx = 100
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=2000)
    else:    # weak scaling: rank r owns the r-th (nx x ny) Kuhn strip of a (nx N) x ny grid
        nx, ny = (args.nx or 3200) * world, (args.ny or 640)
        lower, upper = (0.0, 0.0), (5.0 * world, 1.0)
        grid = H.Grid.structured(H.SIMPLEX, nx, ny, lower, upper, px=world, py=1)
        ncx = 100 * world
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=100 * world * 20)   # == oracle field at N=1
    # the structured grid is implicit (O(subdomains) host memory); the shard holds the rank's owned elements
    # + face ghosts only (C ABI hdd_shard_create: mesh, halo plan, tile lists on the device)
    ctx = H.Context(gpu)
    shard = H.Shard(ctx, grid, world, rank)
    kcell = shard.checkerboard(lower, upper, ncx, 20, perm)
    # every rank evaluates its OWNED coefficients only; the ghost columns arrive through the halo
    kcell[:shard.own_begin] = np.nan
    kcell[shard.own_end:] = np.nan
    tens = torch.from_numpy(kcell).cuda()
    _, _, _, pat_t = pat = shard.pattern(ctx, gpu)
    kappa = [H.scalar_fn(H.FN_CONST, 1.0)]
    tensor = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=tens)
    nnz = shard.info.nnz
    vals = [torch.empty(nnz, dtype=torch.float64, device="cuda")]
    comm = None
    rccl_init_s = None
    if world > 1:
        t_init = time.perf_counter()
        comm = rccl_comm(rank, world, gpu) if args.backend == "nccl" else gloo_host_comm(gpu)
        rccl_init_s = time.perf_counter() - t_init
        sys.stderr.write("[bench] rank %d/%d on GPU %d: %s communicator in %.3f s, halo peers %s\n"
                         % (rank, world, gpu, "RCCL (ncclCommInitRank)" if args.backend == "nccl" else "gloo host",
                            rccl_init_s, [int(p) for p in shard.halo_lists()[0]]))
        sys.stderr.flush()
    flags = H.SHARD_NO_OVERLAP if args.no_overlap else 0

    def gpu_sync(what):
        if world > 1:
            from hdd_amd.watchdog import guarded_sync
            guarded_sync(torch, shard, rank, what, deadline, stream=stream.cuda_stream)
        else:
            torch.cuda.synchronize()

    n_own = shard.n_own
    nbf = 4 if c4 else 3
    dofs_rank = nbf * n_own
    qp1 = 1
    b_elem = (104 if c4 else 84) + 8 * qp1                                  # quad / triangle record
    # interior faces touched by the owned rows: nnz / nb^2 = n_own + 2 (owned-owned faces) + (owned-ghost faces)
    sides = nnz // (nbf * nbf) - n_own
    nif = (sides + shard.info.halo_faces) // 2
    alg_bytes = 8 * nnz * qp1 + n_own * b_elem + 12 * nif                  # SURVEY.md 8(d) formula

    stream = torch.cuda.current_stream()

    def step(f=flags):
        H.assemble_sharded(ctx, shard, comm, kappa, tensor, pat_t, vals, flags=f)

    # The attainable-bandwidth probe (1 GiB torch copy / fill, ~6 ms of HBM streaming) runs before the
    # warmup on every rank: sustained HBM streaming on MI355X goes through a power-management transient
    # (C2 launches 11-30 of a back-to-back run take 225-260 us, before and after 200-215 us:
    # profiles/r02/s3/long/), and with the probe first the timed steps sit nearer the steady state.
    att = None if args.probe_last else attainable_hbm(torch)
    # the first step fills the ghost columns (NaN until then); --halo once keeps them for the timed steps
    step()
    gpu_sync("the first step")
    if args.halo == "once":
        flags = H.SHARD_NO_HALO
    for _ in range(args.warmup):
        step(flags)
    # Kernel time: one event pair brackets the K back-to-back steps on the assembly stream, so kernel_ms is the
    # average step duration including the dispatch gaps (and, with N > 1, the sharded step's pack / exchange /
    # element pass).  Per-step event records would add ~9 us of queue work per step on ROCm (scripts/study/gap.py
    # -> profiles/r01/s2/gap.log) inside the timed region, so they are not used at any N.
    per_step = False
    sharded_step = world > 1 and args.halo == "step"   # (the kernel label below: the SKIP / split launches)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps if per_step else 1)]
    if world > 1:
        gpu_sync("the warmup steps")
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if per_step:
        for k in range(args.steps):
            events[k][0].record(stream)
            step(flags)
            events[k][1].record(stream)
    else:
        events[0][0].record(stream)
        for k in range(args.steps):
            step(flags)
        events[0][1].record(stream)
    gpu_sync("the timed steps")
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_label = H.last_tile_kernel()
    # at N > 1 the ranks may dispatch different kernels (P1 middle ranks split their tiles: tile-list kernels; end
    # ranks the SKIP launch): every rank's label, grouped
    kernels_by_rank = None
    if world > 1:
        labels = [None] * world
        dist.all_gather_object(labels, kernel_label)
        kernels_by_rank = {}
        for r_, lab in enumerate(labels):
            kernels_by_rank.setdefault(lab, []).append(r_)
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in events])) / (1 if per_step else args.steps)
    # max over ranks: wall time, event-timed step; sum over ranks: algorithmic bytes (every rank assembles its own rows)
    t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64)
    per_rank = torch.tensor([[float(alg_bytes), kernel_ms]], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gathered = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(gathered, per_rank)
        per_rank = torch.cat(gathered)
    elapsed, kernel_ms_max = float(t[0]), float(t[1])
    if not np.isfinite(vals[0][:1024].cpu().numpy()).all():
        raise SystemExit("non-finite values: a ghost column was not filled by the halo")
    total_dofs = nbf * grid.ne if c4 else dofs_rank * world
    value = total_dofs * args.steps / elapsed

    if rank == 0:
        # roofline of the whole job: every rank's algorithmic bytes / the slowest rank's event-timed step, against N x
        # the per-GPU peak (at N = 1: this rank's bytes / its step); slowest_rank: that rank's own bytes / its step
        all_bytes = float(per_rank[:, 0].sum())
        achieved = all_bytes / (kernel_ms_max * 1e-3) / 1e9
        peak = HBM_PEAK_GBS * world
        slow = int(torch.argmax(per_rank[:, 1]))
        slowest = {"rank": slow, "step_ms_event": float(per_rank[slow, 1]),
                   "algorithmic_bytes": float(per_rank[slow, 0]),
                   "frac": float(per_rank[slow, 0]) / (float(per_rank[slow, 1]) * 1e-3) / 1e9 / HBM_PEAK_GBS}
        traffic, traffic_src = None, None
        bid = lib_build_id()
        # the stamped profile figures are per-GPU launches of one workload: the C2 strip is the same at every N (weak
        # scaling); the C4 rank piece shrinks with N, so at N > 1 its N = 1 figures do not describe the timed launches
        same_launch = world == 1 or not c4
        wl_key = ("spe10_block_swipdg_q1_%dx%d_8x8_subdomains" % (nx, ny) if c4
                  else "spe10_swipdg_p1_kuhn_%dx%d" % (nx // world, ny))
        if os.path.exists(args.traffic_json) and same_launch:
            try:
                tj = json.load(open(args.traffic_json))
                tw = tj.get("workloads", {}).get(wl_key)
                # the counters' kernel in hdd_last_tile_kernel()'s form (rocprof's demangled name, namespaces dropped)
                tk = (tw or {}).get("kernel", "").split("(")[0].replace("void ", "").replace("hdd::dev::", "")
                if tj.get("build_id") != bid:
                    traffic_src = "n/a: %s measured on build %s, timed build %s" % (
                        os.path.relpath(args.traffic_json, ROOT), tj.get("build_id"), bid)
                elif tw is None:
                    traffic_src = "n/a: workload %s not in %s" % (wl_key, os.path.relpath(args.traffic_json, ROOT))
                elif tk != kernel_label:
                    traffic_src = "n/a: the timed launch (%s) is not the counted kernel (%s)" % (kernel_label, tk)
                else:
                    traffic = tw["hbm_bytes_per_launch"]
                    traffic_src = os.path.relpath(args.traffic_json, ROOT)
            except (OSError, ValueError, KeyError):
                traffic = None
        rocprof_ms, rocprof_src = None, None
        if os.path.exists(args.kernel_times_json) and same_launch:
            try:
                kj = json.load(open(args.kernel_times_json))
                ent = kj.get("workloads", {}).get("c4" if c4 else "c2", {})
                if kj.get("build_id") != bid:
                    rocprof_src = "n/a: %s profiled build %s, timed build %s" % (
                        os.path.relpath(args.kernel_times_json, ROOT), kj.get("build_id"), bid)
                elif ent.get("kernel") != kernel_label:
                    rocprof_src = "n/a: the timed launch (%s) is not the profiled kernel (%s)" % (kernel_label,
                                                                                             ent.get("kernel"))
                else:
                    # the launches of the bench command's timed window (scripts/kernel_times.py), else the all-launch
                    # average of an older file
                    rocprof_ms = ent.get("window_avg_ns", ent["avg_ns"]) * 1e-6
                    rocprof_src = os.path.relpath(args.kernel_times_json, ROOT) + (
                        " (timed-window launches %d-%d of the profiled bench command)"
                        % (ent["window_first_launch"], ent["window_last_launch"]) if "window_avg_ns" in ent else
                        " (all launches)")
            except (OSError, ValueError, KeyError):
                rocprof_ms = None
        if not same_launch:
            traffic_src = rocprof_src = "n/a: the C4 rank piece at N > 1 is not the profiled N = 1 launch"
        halo_desc = ""
        if world > 1 and args.halo == "once":
            halo_desc = ", face halo exchanged once at setup (static mesh and coefficients)"
        elif world > 1:
            # the library's default schedule: Q1 (c4) exchange first, then every tile; P1 (c2) overlapped
            overlapped = not args.no_overlap and not c4
            halo_desc = ", %s face halo%s" % ("RCCL" if args.backend == "nccl" else "gloo host-staged (rehearsal)",
                                              " overlapped with the tiles" if overlapped else ", then every tile")
        if att is None:
            att = attainable_hbm(torch)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(nx // world, ny, args.cpu_seconds, cube=c4)
        out = {
            "metric": "assembled DoFs/sec (global stiffness), SPE10 SWIPDG p=1",
            "value": value,
            "unit": "DoFs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if c4 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SPE10 Model1 stand-in permeability: perm_case1.dat absent)",
            "config": ({"workload": "spe10_block_swipdg_q1_%dx%d_8x8_subdomains" % (nx, ny),
                        "elements": grid.ne, "elements_rank0": n_own, "total_dofs": total_dofs,
                        "nnz_rank0": nnz, "components": qp1,
                        "parallelism": "subdomain columns x%d, owner-computes%s" % (world, halo_desc)}
                       if c4 else
                       {"workload": "spe10_swipdg_p1_kuhn_%dx%d_per_gpu" % (nx // world, ny),
                        "elements_per_gpu": n_own, "dofs_per_gpu": dofs_rank, "nnz_per_gpu": nnz,
                        "total_dofs": total_dofs, "components": qp1,
                        "parallelism": "block-swipdg strips x%d, owner-computes%s" % (world, halo_desc)
                        if world > 1 else "single GPU"}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": traffic,
                         # the physical figure: HBM bytes the kernel really moves (PMC, same build) per second,
                         # over the same peak -- below `frac` because the layout reads less than SURVEY 8(d) prices
                         "traffic_frac": (traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "traffic_gbs": (traffic / (kernel_ms * 1e-3) / 1e9) if traffic else None,
                         # N > 1: frac = all ranks' bytes / the slowest rank's step / (N x peak); the slowest rank alone
                         "slowest_rank": slowest if world > 1 else None,
                         "peak_per_gpu": HBM_PEAK_GBS,
                         "traffic_source": traffic_src, "build_id": bid,
                         # the dominant kernel as the library's dispatch picked it in the last timed step
                         # (hdd_last_tile_kernel, rank 0)
                         "kernel": kernel_label,
                         "kernels_by_rank": kernels_by_rank,
                         # event-timed average step on the assembly stream (one event pair around the K steps, so
                         # dispatch gaps -- and at N > 1 the step's pack / exchange / element pass -- are included)
                         "step_ms_event": kernel_ms, "step_ms_event_max_rank": kernel_ms_max,
                         # the same kernel's average duration from a rocprofv3 --kernel-trace run of this build
                         # (profiles/*/kernel_times.json, build-stamped like the traffic), else null
                         "kernel_ms_rocprof": rocprof_ms, "kernel_ms_rocprof_source": rocprof_src,
                         # the same roofline over the profiled kernel duration (per GPU: rank 0's bytes)
                         "frac_rocprof": (alg_bytes / (rocprof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if rocprof_ms else None,
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "algorithmic_bytes_all_ranks": all_bytes,
                         # measured on this box in this run: device copy (read + write) and fill (write)
                         "attainable": dict(att, source="torch copy_ / fill_ of 1 GiB, HIP events"),
                         "frac_of_torch_copy": achieved / att["copy_gbs"],
                         "frac_note": "frac = SURVEY 8(d) algorithmic bytes (element-major coordinates, 48 B per "
                                      "triangle) / kernel time; traffic_frac = PMC-measured HBM bytes of this build "
                                      "(the vertex-indexed layout reads less) / kernel time, the physical rate"},
            "cpu_baseline": cpu,
        }
        out["config"]["entry"] = "hdd_block_assemble_sharded (C ABI)"
        # any HDD_* variable of this process (the release library reads none but the tests' HDD_DEBUG_FLAGS error
        # injection; recorded so that an inherited environment is visible in the line)
        out["config"]["hdd_env"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith("HDD_")}
        if world > 1:
            out["config"]["comm_init_s_rank0"] = rccl_init_s
            out["config"]["halo"] = args.halo
            out["config"]["halo_elements_rank0"] = [int(shard.info.halo_send), int(shard.info.halo_recv)]
        print(json.dumps(out), flush=True)
    if world > 1:
        del comm
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
