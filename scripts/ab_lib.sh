#!/bin/bash
# Same-box A/B of two builds of libhdd_amd.so (HDD_AMD_LIB) on the C3 / C4 configurations, alternating,
# after the GPU parity suite on the in-tree build.  usage: [CONFIGS="c3 c4 f"] [BENCH=1] ab_lib.sh LIB_A LIB_B [tag]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
A=$1; B=$2; TAG=${3:-ab_lib}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for L in $A $B; do
    n=$(basename $(dirname $L))_$(basename $L .so)
    HDD_AMD_LIB=$PWD/$L timeout -k 10 200 python scripts/bench_configs.py ${CONFIGS:-c3} --samples 16 > $OUT/${n}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; exit $rc; }
    echo "$n $(grep -oE '"(assembly_ms|rhs_ms|pattern_ms)": [0-9.]*' $OUT/${n}_$rep.log | tr '\n' ' ')"
    if [ -n "${BENCH:-}" ]; then   # also the bench line (C2)
      HDD_AMD_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${n}_bench_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$n bench rc=$rc"; exit $rc; }
      echo "$n c2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/${n}_bench_$rep.log)"
    fi
  done
done
