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
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01s2d.json"))
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearsal of the N-rank path on one GPU (host-staged halo)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: exchange the halo before the whole assembly instead of overlapping it "
                         "with the interior tiles")
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
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))

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
                omp_sample="owner-computes OpenMP variant of the same integrands, %d threads, same strip, "
                           "median of 5 (%.3f s per assembly)" % (threads, t_omp),
                cpu_model=_cpu_model(), host_cpus=os.cpu_count())


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import hdd_amd as H
    from hdd_amd.halo import HaloExchange, strip_owner

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    gpu = local_rank if args.backend == "nccl" else 0
    torch.cuda.set_device(gpu)
    local_rank = gpu
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")

    c4 = args.workload == "c4"
    if c4:   # strong scaling: one 3520 x 1200 Q1 mesh, 8 x 8 subdomains, rank r owns a subdomain-column range
        nx, ny = (args.nx or 3520), (args.ny or 1200)
        lower, upper = (0.0, 0.0), (5.0, 1.0)
        grid = H.Grid.structured(H.CUBE, nx, ny, lower, upper, px=8, py=8)
        if world > grid.n_sub:
            raise SystemExit("c4 shards 64 subdomains: at most 64 ranks")
        s0, s1 = (rank * grid.n_sub) // world, ((rank + 1) * grid.n_sub) // world
        local = grid.local(s0, s1)
        ncx = 100
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=2000)
    else:    # weak scaling: rank r owns the r-th (nx x ny) Kuhn strip of a (nx N) x ny grid
        nx, ny = (args.nx or 3200) * world, (args.ny or 640)
        lower, upper = (0.0, 0.0), (5.0 * world, 1.0)
        grid = H.Grid.structured(H.SIMPLEX, nx, ny, lower, upper, px=world, py=1)
        local = grid.local(rank, rank + 1)
        ncx = 100 * world
        perm = 10.0 ** np.random.default_rng(10).uniform(-3.0, 3.0, size=100 * world * 20)   # == oracle field at N=1
    kcell = local.checkerboard(lower, upper, ncx, 20, perm)
    ctx = H.Context(local_rank)
    dmesh = H.DeviceMesh(local, local_rank, zero_ghosts=world > 1)
    tens = torch.from_numpy(kcell).cuda()
    if world > 1:
        tens[:local.own_begin] = 0
        tens[local.own_end:] = 0
    dpat = H.DevicePattern(local, local_rank)
    kappa = [H.scalar_fn(H.FN_CONST, 1.0)]
    tensor = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=tens)
    vals = [torch.empty(dpat.nnz, dtype=torch.float64, device="cuda")]
    halo = None
    if world > 1:
        halo = HaloExchange(ctx, local, [(dmesh.coords, dmesh.coords.shape[0]), (tens.view(1, -1), 1)],
                            strip_owner(grid.n_sub, world), rank, host_staging=args.backend == "gloo")

    n_own = local.n_own
    nbf = 4 if c4 else 3
    dofs_rank = nbf * n_own
    nbr = local.neighbors[:, local.own_begin:local.own_end]
    interior = nbr >= 0
    owned_pair = interior & (nbr >= local.own_begin) & (nbr < local.own_end)
    nif = int(owned_pair.sum()) // 2 + int((interior & ~owned_pair).sum())
    qp1 = 1
    b_elem = (104 if c4 else 84) + 8 * qp1                                  # quad / triangle record
    alg_bytes = 8 * dpat.nnz * qp1 + n_own * b_elem + 12 * nif             # SURVEY.md 8(d) formula

    stream = torch.cuda.current_stream()
    if halo is not None and args.halo == "once":
        halo.exchange()
        torch.cuda.synchronize()
        halo = None
    overlap = halo is not None and not args.no_overlap
    if overlap:
        t_in, t_bd = H.halo_tiles(local)
        tiles_in = torch.from_numpy(t_in).cuda()
        tiles_bd = torch.from_numpy(t_bd).cuda()

    def step(ev=None):
        if overlap:
            # interior tiles (no ghost face neighbour) run while the face halo is in flight
            halo.start()
            if ev is not None:
                ev[0].record(stream)
            H.assemble_tiles(ctx, dmesh, dpat, kappa, tensor, tiles_in, vals)
            halo.finish()
            H.assemble_tiles(ctx, dmesh, dpat, kappa, tensor, tiles_bd, vals)
            if ev is not None:
                ev[1].record(stream)
            return
        if halo is not None:
            halo.exchange()
        if ev is not None:
            ev[0].record(stream)
        H.assemble(ctx, dmesh, dpat, kappa, tensor, vals=vals)
        if ev is not None:
            ev[1].record(stream)

    for _ in range(args.warmup):
        step()
    # Kernel time: with a per-step halo, events bracket the assembly launches of every step (on the
    # assembly stream); otherwise one event pair brackets the K back-to-back launches (per-step event records
    # add ~9 us of queue work per launch on ROCm: scripts/study/gap.py -> profiles/r01/s2/gap.log), so
    # kernel_ms is the average launch duration including the dispatch gaps between launches (conservative).
    per_step = halo is not None
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps if per_step else 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if per_step:
        for k in range(args.steps):
            step(events[k])
    else:
        events[0][0].record(stream)
        for k in range(args.steps):
            step()
        events[0][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in events])) / (1 if per_step else args.steps)
    t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cuda" if args.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms_max = float(t[0]), float(t[1])
    total_dofs = nbf * grid.ne if c4 else dofs_rank * world
    value = total_dofs * args.steps / elapsed

    if rank == 0:
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if not c4 and world == 1 and tj.get("workload") == "spe10_swipdg_p1_kuhn_%dx%d" % (nx // world, ny):
                    traffic = tj.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        halo_desc = ""
        if world > 1 and args.halo == "once":
            halo_desc = ", face halo exchanged once at setup (static mesh and coefficients)"
        elif world > 1:
            halo_desc = ", %s face halo%s" % ("RCCL" if args.backend == "nccl" else "gloo host-staged (rehearsal)",
                                              " overlapped with interior tiles" if overlap else "")
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
                        "nnz_rank0": dpat.nnz, "components": qp1,
                        "parallelism": "subdomain columns x%d, owner-computes%s" % (world, halo_desc)}
                       if c4 else
                       {"workload": "spe10_swipdg_p1_kuhn_%dx%d_per_gpu" % (nx // world, ny),
                        "elements_per_gpu": n_own, "dofs_per_gpu": dofs_rank, "nnz_per_gpu": dpat.nnz,
                        "total_dofs": total_dofs, "components": qp1,
                        "parallelism": "block-swipdg strips x%d, owner-computes%s" % (world, halo_desc)
                        if world > 1 else "single GPU"}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "swipdg_persistent_kernel<%s<1, 0, false>, %s>"
                                   % ("Q1PwcPolicy" if c4 else "P1PwcPolicy", "true" if overlap else "false"),
                         "kernel_ms_avg": kernel_ms, "kernel_ms_avg_max_rank": kernel_ms_max,
                         "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        if halo is not None:
            out["config"]["halo_bytes_per_step_rank0"] = halo.halo_bytes
        if world > 1:
            out["config"]["halo"] = args.halo
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
