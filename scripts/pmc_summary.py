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
    # wave-cycle accounting (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, disjoint;
    # ACTIVE_INST_* by instruction class may overlap each other)
    for k in sorted(vals):
        if want and not any(w in k for w in want):
            continue
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        wc = m.get("SQ_WAVE_CYCLES")
        if not wc or not all(c in m for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")):
            continue
        print("\nwave-cycle accounting, %s (SQ_WAVE_CYCLES %.4g per dispatch):" % (k.split("(")[0], wc))
        parts = ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
        for c in parts:
            print("  %-22s %6.1f %%" % (c, 100 * m[c] / wc))
        print("  %-22s %6.1f %%" % ("sum", 100 * sum(m[c] for c in parts) / wc))
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA",
                  "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_FLAT", "SQ_WAIT_INST_LDS"):
            if c in m:
                print("    %-20s %6.1f %%" % (c, 100 * m[c] / wc))
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
