#!/usr/bin/env python3
"""kernel_times.py -- build-stamped kernel durations of the bench workloads from rocprofv3 --kernel-trace --stats runs.

usage: kernel_times.py OUT.json WORKLOAD=PROF_DIR [WORKLOAD=PROF_DIR ...] [--lib PATH] [--steps K] [--warmup W]

For every workload (c2, c4) reads the kernel_stats.csv and kernel_trace.csv under PROF_DIR (scripts/gpu.sh "prof" step:
bench.py under rocprofv3, default --steps 20 --warmup 5), takes the persistent tile kernel with the largest total time
and writes {build_id, workloads: {wl: {kernel, avg_ns, calls, window_*, ...}}}:
  - avg_ns / min_ns / max_ns / calls: rocprof's own statistics over every launch of the command (the cold first launch
    -- the ghost-filling first step -- included);
  - window_*: the launches of bench.py's timed region only.  bench.py launches the kernel once for the first step, W
    times for the warmup and K times timed, so the timed window is launches W + 2 .. W + K + 1 (1-based, in dispatch
    order); window_avg_ns / window_median_ns over them, window_launches_us the per-launch durations.
build_id = sha256 prefix of the library the profile ran (the in-tree libhdd_amd.so unless --lib); bench.py reports
`kernel_ms_rocprof` (the window average) only when the timed library has the same id and dispatched the same kernel.
"""
import csv
import glob
import hashlib
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def label(name):
    """rocprof's demangled kernel name -> hdd_last_tile_kernel()'s format"""
    m = re.search(r"swipdg_persistent_kernel<(.*)>\(", name)
    if not m:
        return name
    return "swipdg_persistent_kernel<" + m.group(1).replace("hdd::dev::", "") + ">"


def window(trace_csv, name, steps, warmup):
    """per-launch durations (ns) of kernel `name` in dispatch order, and the bench's timed window of them"""
    rows = [r for r in csv.DictReader(open(trace_csv)) if r["Kernel_Name"] == name]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    lo, hi = warmup + 1, warmup + 1 + steps          # 0-based [lo, hi) = 1-based launches W + 2 .. W + K + 1
    return dur, dur[lo:hi] if len(dur) >= hi else []


def main():
    args = sys.argv[1:]
    opts = {"--lib": os.path.join(ROOT, "dune-hdd_amd", "lib", "libhdd_amd.so"), "--steps": "20", "--warmup": "5"}
    for k in list(opts):
        if k in args:
            i = args.index(k)
            opts[k] = args[i + 1]
            del args[i:i + 2]
    lib, steps, warmup = opts["--lib"], int(opts["--steps"]), int(opts["--warmup"])
    out, pairs = args[0], args[1:]
    bid = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    res = {"build_id": bid, "library": os.path.relpath(lib, ROOT), "bench_steps": steps, "bench_warmup": warmup,
           "workloads": {}}
    for p in pairs:
        wl, d = p.split("=", 1)
        files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not files:
            sys.exit("no kernel_stats.csv under %s" % d)
        rows = list(csv.DictReader(open(files[0])))
        rows = [r for r in rows if "swipdg_persistent_kernel" in r["Name"]]
        if not rows:
            sys.exit("no persistent tile kernel in %s" % files[0])
        r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
        ent = {"kernel": label(r["Name"]), "avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]),
               "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]), "source": os.path.relpath(files[0], ROOT)}
        traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if traces:
            dur, win = window(traces[0], r["Name"], steps, warmup)
            if win:
                ent.update(window_first_launch=warmup + 2, window_last_launch=warmup + steps + 1,
                           window_avg_ns=statistics.fmean(win), window_median_ns=statistics.median(win),
                           window_launches_us=[round(x / 1e3, 1) for x in win],
                           avg_ns_without_first=statistics.fmean(dur[1:]),
                           trace_source=os.path.relpath(traces[0], ROOT))
        # the profiled bench command's own JSON line (gpu.sh "prof" writes it to PROF_DIR.log): its step time brackets
        # the same launches the window averages
        blog = d.rstrip("/") + ".log"
        if os.path.exists(blog):
            for line in open(blog):
                if line.startswith("{"):
                    b = json.loads(line)
                    ent.update(profiled_run_ms_per_step=b["ms_per_step"],
                               profiled_run_step_ms_event=b["roofline"]["step_ms_event"],
                               profiled_run_log=os.path.relpath(blog, ROOT))
        res["workloads"][wl] = ent
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
