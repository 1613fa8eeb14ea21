#!/usr/bin/env python3
"""kernel_times.py -- build-stamped kernel durations of the bench workloads from rocprofv3 --kernel-trace --stats runs.

usage: kernel_times.py OUT.json WORKLOAD=PROF_DIR [WORKLOAD=PROF_DIR ...] [--lib PATH]

For every workload (c2, c4) reads the kernel_stats.csv under PROF_DIR (scripts/gpu.sh "prof" step), takes the
persistent tile kernel with the largest total time and writes {build_id, workloads: {wl: {kernel, avg_ns, calls,
source}}}.  build_id = sha256 prefix of the library the profile ran (the in-tree libhdd_amd.so unless --lib); bench.py
reports `kernel_ms_rocprof` only when the timed library has the same id and dispatched the same kernel.
"""
import csv
import glob
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def label(name):
    """rocprof's demangled kernel name -> hdd_last_tile_kernel()'s format"""
    m = re.search(r"swipdg_persistent_kernel<(.*)>\(", name)
    if not m:
        return name
    return "swipdg_persistent_kernel<" + m.group(1).replace("hdd::dev::", "") + ">"


def main():
    args = sys.argv[1:]
    lib = os.path.join(ROOT, "dune-hdd_amd", "lib", "libhdd_amd.so")
    if "--lib" in args:
        i = args.index("--lib")
        lib = args[i + 1]
        del args[i:i + 2]
    out, pairs = args[0], args[1:]
    bid = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    res = {"build_id": bid, "library": os.path.relpath(lib, ROOT), "workloads": {}}
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
        res["workloads"][wl] = {"kernel": label(r["Name"]), "avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]),
                                "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                "source": os.path.relpath(files[0], ROOT)}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
