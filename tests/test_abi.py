"""The C-ABI library loads, exports every symbol include/hdd.h declares, and fails loudly (status + message,
no exception across the ABI) on bad input.  No device calls: runs without a GPU."""
import ctypes as C

import numpy as np
import pytest

import hdd_amd as H


def test_exports_every_declared_symbol():
    L = H.lib()
    names = H.declared_symbols()
    assert len(names) >= 24
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.hdd_abi_version() == 8


def test_errors_are_status_codes_with_messages():
    L = H.lib()
    h = C.c_void_p()
    d = H.StructuredDesc(H.SIMPLEX, 0, 4, 1, 1, 0, 0, (C.c_double * 2)(0, 0), (C.c_double * 2)(1, 1))
    rc = L.hdd_grid_create_structured(C.byref(d), C.byref(h))
    assert rc == 1 and b"px" in L.hdd_last_error(None)
    d = H.StructuredDesc(7, 4, 4, 1, 1, 0, 0, (C.c_double * 2)(0, 0), (C.c_double * 2)(1, 1))
    assert L.hdd_grid_create_structured(C.byref(d), C.byref(h)) == 3
    g = H.Grid.structured(H.SIMPLEX, 4, 4, px=2, py=2)
    with pytest.raises(H.HddError, match="out|s_begin"):
        g.local(3, 5)
    with pytest.raises(H.HddError):
        g.subdomain_range(2, 2)
    nnz = C.c_int64()
    nb = np.zeros((3, 4), np.int32)
    assert L.hdd_pattern_count(9, 4, 0, 4, nb.ctypes.data, C.byref(nnz)) == 3
    assert L.hdd_pattern_count(H.SIMPLEX, 4, 0, 5, nb.ctypes.data, C.byref(nnz)) == 1


def test_device_entry_points_reject_null_arguments():
    L = H.lib()
    assert L.hdd_swipdg_assemble(None, None, None, 1, None, None, None, None, None) == 1
    assert L.hdd_affine_lincomb(None, 0, None, 1, None, 0, None, 0, None) == 1
    assert L.hdd_soa_gather(None, None, None, 1, 0, None, 0, None, None) == 1
