"""Static check of the built library's gfx950 machine code (no GPU): no store of more than 8 bytes is followed
directly by a VALU instruction that overwrites one of its data registers (scripts/check_store_hazard.py; hipcc
leaves that hazard unpadded when the store's soffset is a register, and gfx950 then stores a stale first dword --
found in round 5 on the Q1 half-image kernel's sharded SKIP tiles)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
LIB = os.path.join(ROOT, "dune-hdd_amd", "lib", "libhdd_amd.so")


def _scan():
    import check_store_hazard as C
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    # a built library with no disassembler must not pass silently: the guard would check nothing
    assert os.path.exists(C.OBJDUMP), "library present but %s absent: the hazard scan cannot run" % C.OBJDUMP
    n, found = C.scan_lib(LIB)
    assert n > 0, "no gfx950 code object found in %s" % LIB
    assert not found, "store-data hazards: %s" % found[:5]


@pytest.mark.timeout(300)
def test_no_store_data_hazard_in_library():
    _scan()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_no_store_data_hazard_in_library_gpu_suite():
    """the same scan in the GPU suite, on the box that loads the library (same image: llvm-objdump present)"""
    _scan()


def test_scanner_flags_the_round5_pattern():
    import check_store_hazard as C
    bad = ["buffer_store_dwordx4 v[2:5], v127, s[28:31], s58 offen nt", "v_and_b32_e32 v2, s0, v47"]
    ok = ["buffer_store_dwordx4 v[2:5], v127, s[28:31], s58 offen nt", "s_nop 0", "v_and_b32_e32 v2, s0, v47"]
    addr = ["global_store_dwordx4 v[2:3], v[22:25], off offset:-8 nt", "v_lshl_add_u64 v[2:3], v[2:3], 0, 64"]
    data = ["global_store_dwordx4 v2, v[4:7], s[0:1]", "v_mov_b32_e32 v5, 0"]
    assert len(C.scan_text(bad)) == 1
    assert C.scan_text(ok) == []
    assert C.scan_text(addr) == []      # the address pair, not the data
    assert len(C.scan_text(data)) == 1
