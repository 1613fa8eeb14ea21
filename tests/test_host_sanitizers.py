"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; GPU sanitizers are not available on this
pool).  Two drivers, built here from the sources with -fsanitize=address,undefined -fno-sanitize-recover=all:

- tests/host_asan/asan_host.cpp: the product's host code (csrc/host/grid.cpp, errors.cpp) through the C ABI --
  structured 2d / 3d grids, grids from connectivity (and their rejections), rank-local views, vertex-indexed
  geometry, halo plans and send lists, checkerboard / indicator lookups, both CSR pattern builders, block-operator
  maps (the blocks must partition the monolithic pattern);
- tests/host_asan/asan_oracle.c: the CPU oracle (test infrastructure) -- every entry point the parity tests use, every
  coefficient / tensor kind, both boundary kinds, the owner-computes OpenMP variant, BlockSWIPDG, RHS, products,
  the Q_p restatement in 2d and 3d.

A sanitizer report or a failed check ends the driver with a non-zero status."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


def _run(cmd, **kw):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, **kw)


def _build_and_run(compiler, srcs, flags, out):
    if shutil.which(compiler) is None:
        pytest.fail("%s not found: the host sanitizer runs need it" % compiler)
    b = _run([compiler] + flags + SAN + srcs + ["-o", out] + (["-lm"] if compiler == "gcc" else []))
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = _run([out], env=env)
    report = r.stdout + r.stderr
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in report and "runtime error" not in report, \
        report[-6000:]
    assert "all checks passed" in r.stdout


def test_product_host_code_under_asan_ubsan(tmp_path):
    srcs = [os.path.join(ROOT, "tests", "host_asan", "asan_host.cpp"),
            os.path.join(ROOT, "dune-hdd_amd", "csrc", "host", "grid.cpp"),
            os.path.join(ROOT, "dune-hdd_amd", "csrc", "host", "errors.cpp")]
    flags = ["-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "dune-hdd_amd", "csrc", "host")]
    _build_and_run("g++", srcs, flags, str(tmp_path / "asan_host"))


def test_oracle_under_asan_ubsan(tmp_path):
    srcs = [os.path.join(ROOT, "tests", "host_asan", "asan_oracle.c"),
            os.path.join(ROOT, "oracle", "swipdg_oracle.c"),
            os.path.join(ROOT, "oracle", "swipdg_oracle_qp.c")]
    flags = ["-std=c99", "-D_DEFAULT_SOURCE", "-fopenmp", "-I" + os.path.join(ROOT, "oracle")]
    _build_and_run("gcc", srcs, flags, str(tmp_path / "asan_oracle"))
