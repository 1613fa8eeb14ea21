#!/bin/bash
# Round-3 measurement pass: GPU parity suite, smoke, the bench line (C2 and --workload c4), the config
# table, rocprofv3 kernel stats of both bench workloads, PMC traffic passes (scripts/traffic.sh).
# Each GPU step time-limited; stops at the first failure.  usage: [NOTEST=1] [NOTRAFFIC=1] gpu_r03_pass.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); TAG=${1:-r03}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NOTRAFFIC:-}" ]; then
  bash scripts/traffic.sh "$TAG" > "$OUT/traffic.log" 2>&1
  rc=$?; echo "traffic rc=$rc"; tail -3 "$OUT/traffic.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --traffic-json ${TRAFFIC_JSON:-profiles/$TAG/traffic.json} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline --traffic-json ${TRAFFIC_JSON:-profiles/$TAG/traffic.json} > "$OUT/bench_c4.log" 2>&1
rc=$?; echo "bench c4 rc=$rc"; tail -1 "$OUT/bench_c4.log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc
if [ -n "${CFG:-}" ]; then
  timeout -k 10 400 python -u scripts/bench_configs.py $CFG > "$OUT/configs.log" 2>&1
  rc=$?; echo "configs rc=$rc"; grep config "$OUT/configs.log"; [ $rc -eq 0 ] || exit $rc
fi
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_c4.log" 2>&1
rc=$?; echo "rocprof c4 rc=$rc"; exit $rc
