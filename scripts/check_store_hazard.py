#!/usr/bin/env python3
"""check_store_hazard.py -- scan the gfx950 code objects inside a built library for the VMEM store-data hazard.

A buffer / global store of more than 8 bytes (dwordx3 / dwordx4) reads its data VGPRs after issue; a VALU
instruction that overwrites one of them in the very next slot needs a wait state in between.  hipcc inserts that
`s_nop` only when the store's soffset is not a register, and gfx950 then writes the stale first dword (round 5:
wrong low words on the sharded SKIP tiles of the Q1 half-image kernel).  This scan flags every
store of > 8 bytes whose next instruction is a VALU writing one of its data registers, whatever the soffset.

usage: check_store_hazard.py [LIB.so ...]      (default: dune-hdd_amd/lib/libhdd_amd.so); exit 1 on a finding
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# the data operand: first for buffer stores, second (after the address) for global stores
STORE = re.compile(r"^\s*(?:buffer_store_dwordx[34]\s+|global_store_dwordx[34]\s+v(?:\[\d+:\d+\]|\d+),\s*)"
                   r"v\[(\d+):(\d+)\]")
VDST = re.compile(r"^\s*v_\w+\s+v(?:\[(\d+):(\d+)\]|(\d+))\s*,")
SYM = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def code_objects(lib):
    """the gfx950 ELF code objects of every offload bundle in the library's .hip_fatbin section"""
    data = open(lib, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if "gfx950" in triple and size > 0:
                yield data[pos + off:pos + off + size]
        pos = data.find(MAGIC, pos + 32)


def scan_text(lines):
    """-> [(symbol, store line, next line)] for every hazard in one disassembly.

    Window: the ONE instruction right after the store.  That is the hazard's extent on gfx950 (the VALU write
    conflicts with the store's read of its data registers only in the slot immediately following the issue; one
    wait state -- an s_nop or any other instruction -- resolves it, which is how hipcc pads the soffset-free form),
    so a register overwritten two or more instructions later is not a hazard."""
    out, sym, pend = [], "?", None
    for line in lines:
        m = SYM.match(line.strip())
        if m:
            sym, pend = m.group(1), None
            continue
        text = line.split("//")[0].split(";")[0].strip()
        if not text or text.endswith(":"):
            continue
        if pend is not None:
            lo, hi, sline = pend
            pend = None
            d = VDST.match(text)
            if d:
                a = int(d.group(1) or d.group(3))
                b = int(d.group(2) or d.group(3))
                if a <= hi and b >= lo:
                    out.append((sym, sline, text))
        s = STORE.match(text)
        if s:
            pend = (int(s.group(1)), int(s.group(2)), text)
    return out


def scan_lib(lib):
    """-> (code objects scanned, findings)"""
    found, n = [], 0
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(lib)):
            path = os.path.join(td, "co%d.o" % i)
            open(path, "wb").write(co)
            proc = subprocess.Popen([OBJDUMP, "-d", "--no-show-raw-insn", "--mcpu=gfx950", path],
                                    stdout=subprocess.PIPE, text=True)
            found += scan_text(proc.stdout)
            proc.wait()
            n += 1
    return n, found


def main():
    libs = sys.argv[1:] or [os.path.join(ROOT, "dune-hdd_amd", "lib", "libhdd_amd.so")]
    bad = 0
    for lib in libs:
        n, found = scan_lib(lib)
        print("%s: %d gfx950 code objects, %d store-data hazards" % (lib, n, len(found)))
        for sym, s, t in found[:20]:
            print("  %s\n    %s\n    %s" % (sym[:120], s, t))
        bad += len(found)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
