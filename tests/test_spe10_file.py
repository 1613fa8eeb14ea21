"""SPE10 Model1 built from its permeability data file (problems/spe10.hh:111-125, 151-156), host only.

The reference's Spe10Model1 ctor takes the data file (dune-stuff's Spe10::Model1 function reads
perm_case1.dat).  Neither the file nor dune-stuff is in /root/reference, so the reader is restated
(hdd_spe10_model1_read: whitespace-separated numbers, the first 100 x 20 of the 6000 are the checkerboard cells,
x fastest, mapped affinely from [model1_min, model1_max] onto [min, max]) and checked here on synthetic files
written in that layout -- parity unpinned.  The C++ ctor with the file equals the vector ctor with the expected
cells (examples/problems_main, host code only)."""
import os
import subprocess

import numpy as np
import pytest

import hdd_amd as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HDD_EXAMPLES_BIN: another build of the examples, e.g. examples/bin_asan (make -C dune-hdd_amd asan)
EXE = os.path.join(os.environ.get("HDD_EXAMPLES_BIN") or os.path.join(ROOT, "examples", "bin"), "problems_main")


def _write_model1(path, values, per_line=6):
    """the Model1 layout: 6000 numbers (three 100 x 20 blocks), several per line, mixed notation"""
    with open(path, "w") as f:
        for i in range(0, len(values), per_line):
            row = values[i:i + per_line]
            f.write("  ".join(("%.17g" if (i // per_line) % 2 else "%.17e") % v for v in row) + "\n")


def _synthetic(seed=3):
    rng = np.random.default_rng(seed)
    return 10.0 ** rng.uniform(-3.0, np.log10(998.915), size=6000)


def test_reader_takes_the_first_2000_cells(tmp_path):
    vals = _synthetic()
    p = str(tmp_path / "perm_case1.dat")
    _write_model1(p, vals)
    got = H.spe10_model1_read(p)
    assert got.shape == (2000,)
    assert np.array_equal(got, vals[:2000])   # identity map for the reference's min / max (scale 1, shift 0)


def test_reader_rescales_and_rejects(tmp_path):
    vals = _synthetic(5)
    p = str(tmp_path / "perm.dat")
    _write_model1(p, vals, per_line=1)
    lo, hi = H.SPE10_MODEL1_MIN, H.SPE10_MODEL1_MAX
    got = H.spe10_model1_read(p, 1.0, 2.0)
    scale = (2.0 - 1.0) / (hi - lo)
    assert np.allclose(got, vals[:2000] * scale + (1.0 - scale * lo), rtol=0, atol=1e-15)
    with pytest.raises(H.HddError, match="larger than min"):
        H.spe10_model1_read(p, 2.0, 2.0)
    with pytest.raises(H.HddError, match="could not open"):
        H.spe10_model1_read(str(tmp_path / "missing.dat"))
    short = str(tmp_path / "short.dat")
    _write_model1(short, vals[:1999])
    with pytest.raises(H.HddError, match="1999 values"):
        H.spe10_model1_read(short)


def test_cpp_spe10_from_file_equals_vector_ctor(tmp_path):
    """Problems::Spe10Model1(filename, lower_left, upper_right, channel, forces, layer, parametric) == the vector
    ctor with the expected cells (plain and parametric channel, default and shifted domain, FlatTop default)."""
    assert os.access(EXE, os.X_OK), "examples/bin/problems_main missing: run make -C dune-hdd_amd"
    vals = _synthetic(7)
    data, cells = str(tmp_path / "perm_case1.dat"), str(tmp_path / "cells.bin")
    _write_model1(data, vals)
    vals[:2000].astype(np.float64).tofile(cells)
    r = subprocess.run([EXE, "spe10", data, cells], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "spe10 file == vector: 1" in r.stdout and "missing file rejected" in r.stdout, r.stdout
