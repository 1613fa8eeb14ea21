#!/bin/bash
# Round-3 GPU pass: GPU tests (optional), production-library A/B of kernel variants (scripts/ablate.py, one
# process, interleaved), extra configs.  usage: [NOTEST=1] [ABL="c4:0,2048"] [CFG="ops"] gpu_r03.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03}; mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:-} > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ABL:-}" ]; then
  timeout -k 10 300 python scripts/ablate.py $ABL > $OUT/ablate.log 2>&1
  rc=$?; echo "ablate rc=$rc"; cat $OUT/ablate.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ABLAB:-}" ]; then
  HDD_AMD_LIB=$PWD/dune-hdd_amd/lib_ab/libhdd_abl.so timeout -k 10 300 python scripts/ablate.py $ABLAB > $OUT/ablate_ab.log 2>&1
  rc=$?; echo "ablate_ab rc=$rc"; cat $OUT/ablate_ab.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${CFG:-}" ]; then
  timeout -k 10 300 python scripts/bench_configs.py $CFG > $OUT/cfg.log 2>&1
  rc=$?; echo "cfg rc=$rc"; grep config $OUT/cfg.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
