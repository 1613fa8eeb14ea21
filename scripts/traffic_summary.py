"""Summarise the PMC traffic passes (scripts/traffic.sh) into profiles/<tag>/traffic.json and the
bench-readable profiles/traffic_<tag>.json: HBM bytes per launch of the hot kernel, corrected with the
factors measured on calibration kernels of known byte counts (MI355X_MICROARCH.md HBM section: FETCH_SIZE
reads 1/2 of wide coalesced reads on gfx950; other widths must be calibrated)."""
import csv, glob, hashlib, json, os, sys, collections
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
LIB = os.path.join(ROOT, "dune-hdd_amd", "lib", "libhdd_amd.so")
# the build the counters were taken on (bench.py reports traffic only for the same build id)
build_id = hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16]
src = os.path.join(ROOT, "gpurun_out", "traffic_" + tag)

def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc

KB = 1024.0
cal_bytes = 1200 * 2 ** 20      # stream.hip: every calibration kernel moves 1200 MiB
f = per_kernel(os.path.join(src, "cal_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
w = per_kernel(os.path.join(src, "cal_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
def med(v):
    v = sorted(v); return v[len(v) // 2]
cal = {}
for k, v in f.items():
    if k.startswith("rd8"): cal["read_8B_lane"] = cal_bytes / (med(v) * KB)
    elif k.startswith("rd("): cal["read_16B_lane"] = cal_bytes / (med(v) * KB)
for k, v in w.items():
    if k.startswith("wr8"): cal["write_8B_lane"] = cal_bytes / (med(v) * KB)
    elif k.startswith("wr("): cal["write_16B_lane"] = cal_bytes / (med(v) * KB)
def kernel_traffic(prefix):
    bf = per_kernel(os.path.join(src, prefix + "_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    bw = per_kernel(os.path.join(src, prefix + "_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    kname = [k for k in bf if "swipdg_persistent" in k][0]
    fetch_kb, write_kb = med(bf[kname]), med([v for k, vs in bw.items() if "swipdg_persistent" in k for v in vs])
    # the kernel's reads are 8-byte lanes (coalesced SoA) + gathers; its writes are 16-byte lanes
    read_bytes = fetch_kb * KB * cal.get("read_8B_lane", 2.0)
    write_bytes = write_kb * KB * cal.get("write_16B_lane", 1.0)
    return dict(kernel=kname, fetch_size_kb=fetch_kb, write_size_kb=write_kb, read_bytes=read_bytes,
                write_bytes=write_bytes, hbm_bytes_per_launch=read_bytes + write_bytes)


workloads = {"spe10_swipdg_p1_kuhn_3200x640": kernel_traffic("bench")}
if os.path.exists(os.path.join(src, "c4_FETCH_SIZE")):
    workloads["spe10_block_swipdg_q1_3520x1200_8x8_subdomains"] = kernel_traffic("c4")
out = dict(build_id=build_id, calibration_factors=cal, workloads=workloads,
           note="FETCH_SIZE/WRITE_SIZE medians over the profiled launches; factors = known bytes / counter "
                "bytes measured on stream.hip kernels of the same lane width")
os.makedirs(os.path.join(ROOT, "profiles", tag), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "profiles", tag, "traffic.json"), "w"), indent=1)
json.dump(out, open(os.path.join(src, "traffic.json"), "w"), indent=1)   # gpurun_out travels back from the box
print(json.dumps(out, indent=1))
