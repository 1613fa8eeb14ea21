#!/bin/bash
# The C++ examples and the library with AddressSanitizer + UBSan on their HOST code (make -C dune-hdd_amd asan:
# lib_asan/libhdd_asan.so, examples/bin_asan/), driven by the GPU tests that run the examples -- the sharded step on
# thread ranks (mailbox and device transports), the RCCL communicator from C++, the surface / problems drivers --
# with the tests' own checks.  The executables carry the sanitizer runtime (no preloading); device code is compiled
# as in the release build (GPU sanitizers are not available on this pool).
#   usage (on the GPU box): bash scripts/host_asan_gpu.sh RUN
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
[ -x examples/bin_asan/sharded_main ] || { echo "examples/bin_asan missing: make -C dune-hdd_amd asan"; exit 2; }
exec bash scripts/gpu.sh "${1:-asan}" "env ASAN_OPTIONS=detect_leaks=0" "env HDD_EXAMPLES_BIN=examples/bin_asan" \
  "tests -k 'surface or sharded'"
