#!/bin/bash
# C4 store-pattern study (round 3): wstream6 (store patterns of 40 KB tile images) and the production Q1 kernel
# under ablation / schedule bits (HDD_ABLATION build in lib_ab/); first the surface / sharded tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-c4study}; mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 120 ./scripts/microbench/wstream6 > $OUT/wstream6.log 2>&1
rc=$?; echo "wstream6 rc=$rc"; cat $OUT/wstream6.log; [ $rc -eq 0 ] || exit $rc
HDD_AMD_LIB=$PWD/dune-hdd_amd/lib_ab/libhdd_abl.so timeout -k 10 300 python scripts/ablate.py ${ABL_GROUPS:-c4:0,1,2,4,5,32,64,128,256,33 c2:0,32} > $OUT/ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; cat $OUT/ablate.log; exit $rc
