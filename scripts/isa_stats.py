#!/usr/bin/env python3
"""isa_stats.py -- static instruction census of one kernel in a hipcc `-S` (device-only) assembly file.

usage: isa_stats.py FILE.s SYMBOL_SUBSTRING [--loops] [--dump OUT.s]

Prints, for the first kernel whose symbol contains SYMBOL_SUBSTRING: the register / LDS / spill metadata and an
instruction tally by class (f64 VALU, other VALU, SALU, LDS, VMEM loads / stores, waits, branches), for the whole
kernel and -- with --loops -- per basic block that is the target of a backward branch (the loop bodies), so a
kernel variant's per-tile instruction count can be read before spending GPU time on it.
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        if "_f64" in op or op in ("v_rcp_f64", "v_rsq_f64"):
            return "valu_f64"
        if op.startswith("v_accvgpr"):
            return "accvgpr"
        if op.startswith("v_readlane") or op.startswith("v_readfirstlane"):
            return "v_readlane"
        return "valu_other"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "lds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "lds_write"
    if op.startswith("ds_"):
        return "lds_other"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_load" if not op.startswith("scratch") else "scratch_load"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store")):
        return "vmem_store" if not op.startswith("scratch") else "scratch_store"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    loops = "--loops" in sys.argv
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        head = l.split(";")[0].rstrip()
        if head.endswith(":") and not l.startswith((".", "\t", " ")) and sub in head and "kernel" in head:
            start = i
            name = head[:-1]
            break
    if start is None:
        sys.exit("no kernel matching %r" % sub)
    body = []
    for l in lines[start + 1:]:
        if l.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", l):
            break
        body.append(l)
    meta = {}
    for l in lines[start:]:
        m = re.match(r"\s*; (NumVgprs|NumAgprs|TotalNumVgprs|ScratchSize|Occupancy|LDSByteSize|NumSgprs): (\S+)", l)
        if m:
            meta.setdefault(m.group(1), m.group(2))
        if ".end_amdhsa_kernel" in l:
            break
    if "--dump" in sys.argv:
        with open(sys.argv[sys.argv.index("--dump") + 1], "w") as fh:
            fh.write("\n".join(body))
    print(name[:160])
    print("  ", meta)
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = Counter()
    back_targets = set()
    order = [cur]
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\d+_\d+:", s):
                cur = s[:-1]
                blocks[cur] = Counter()
                order.append(cur)
            continue
        op = s.split()[0]
        blocks[cur][classify(op)] += 1
        blocks[cur]["total"] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in blocks:   # already seen -> backward branch
                back_targets.add(tgt)
    tot = Counter()
    for c in blocks.values():
        tot.update(c)
    keys = ["total", "valu_f64", "valu_other", "v_readlane", "accvgpr", "salu", "smem", "lds_write", "lds_read",
            "vmem_load", "vmem_store", "scratch_load", "scratch_store", "s_waitcnt", "branch", "mfma"]
    print("   kernel:", " ".join("%s=%d" % (k, tot[k]) for k in keys if tot[k]))
    if loops:
        for t in back_targets:
            i0 = order.index(t)
            # the loop body: blocks from the target up to the block holding the backward branch (last such)
            seg = Counter()
            for b in order[i0:]:
                seg.update(blocks[b])
            print("   from %s to end:" % t, " ".join("%s=%d" % (k, seg[k]) for k in keys if seg[k]))


if __name__ == "__main__":
    main()
