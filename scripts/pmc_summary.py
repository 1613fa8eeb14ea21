"""Per-kernel PMC summary of rocprofv3 --pmc passes: mean counter value per dispatch, by kernel name.

usage: python scripts/pmc_summary.py <dir> [kernel-substring ...]
Walks <dir> for *counter_collection.csv (one per pass) and *kernel_stats.csv; prints a markdown table.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    want = sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        with open(path) as f:
            for r in csv.DictReader(f):
                per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
    print("| kernel | counter | dispatches | mean per dispatch |")
    print("|---|---|---|---|")
    for k in sorted(vals):
        if want and not any(w in k for w in want):
            continue
        short = k.split("(")[0]
        for c in sorted(vals[k]):
            v = vals[k][c]
            print("| %s | %s | %d | %.4g |" % (short, c, len(v), sum(v) / len(v)))
    for path in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
        print("\nkernel stats: %s" % os.path.relpath(path, root))
        with open(path) as f:
            for r in csv.DictReader(f):
                if want and not any(w in r["Name"] for w in want):
                    continue
                print("  %-60s calls %4s  avg %.3f ms" % (r["Name"].split("(")[0], r["Calls"],
                                                            float(r["AverageNs"]) / 1e6))


if __name__ == "__main__":
    main()
