#!/bin/bash
# Round-4 measurement pass on the current build: GPU suite + smoke, PMC traffic (scripts/traffic.sh), the bench lines
# (C2; --workload c4 with its cube-strip CPU baseline), the config table, rocprofv3 kernel stats of both bench
# workloads, the C4 / C2 wave-cycle accounting (scripts/pmc_acct.sh).  Each GPU step time-limited; stops at the first
# failure.  usage: [NOTEST=1] [NOTRAFFIC=1] [NOPMC=1] [CFG="c3 c4 c5 f ops"] gpu_r04_pass.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); TAG=${1:-r04}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NOTRAFFIC:-}" ]; then
  bash scripts/traffic.sh "$TAG" > "$OUT/traffic.log" 2>&1
  rc=$?; echo "traffic rc=$rc"; tail -3 "$OUT/traffic.log"; [ $rc -eq 0 ] || exit $rc
fi
TJ=${TRAFFIC_JSON:-profiles/$TAG/traffic.json}
[ -f "$TJ" ] || TJ=gpurun_out/traffic_$TAG/traffic.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --traffic-json $TJ > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 20 --warmup 5 --traffic-json $TJ > "$OUT/bench_c4.log" 2>&1
rc=$?; echo "bench c4 rc=$rc"; tail -1 "$OUT/bench_c4.log" | cut -c1-700; [ $rc -eq 0 ] || exit $rc
if [ -n "${CFG:-}" ]; then
  timeout -k 10 500 python -u scripts/bench_configs.py $CFG > "$OUT/configs.log" 2>&1
  rc=$?; echo "configs rc=$rc"; grep config "$OUT/configs.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_c4.log" 2>&1
rc=$?; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT"
if [ -z "${NOPMC:-}" ]; then
  bash scripts/pmc_acct.sh ${TAG}_c4 --workload c4 > "$OUT/pmc_c4.log" 2>&1
  rc=$?; echo "pmc c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_c4 swipdg_persistent > "$OUT/pmc_c4_summary.md" 2>&1
  bash scripts/pmc_acct.sh ${TAG}_c2 > "$OUT/pmc_c2.log" 2>&1
  rc=$?; echo "pmc c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_c2 swipdg_persistent > "$OUT/pmc_c2_summary.md" 2>&1
  grep -A12 "wave-cycle accounting" "$OUT/pmc_c4_summary.md" "$OUT/pmc_c2_summary.md"
fi
