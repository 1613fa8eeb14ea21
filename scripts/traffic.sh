#!/bin/bash
# HBM bytes per launch of the hot kernel from PMC counters (own rocprofv3 passes, kernel-trace only),
# plus a calibration of FETCH_SIZE / WRITE_SIZE on kernels of known byte counts and the same access widths;
# both bench workloads (C2, --workload c4).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/traffic_${1:-r01}
mkdir -p "$OUT"
MB=$ROOT/scripts/microbench
[ -x "$MB/stream" ] || /opt/rocm/bin/hipcc -O3 -Wno-unused-result -Wno-unused-value --offload-arch=gfx950 "$MB/stream.hip" -o "$MB/stream" || exit 1
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c -d "$OUT/cal_$c" -o run --output-format csv -- "$ROOT/scripts/microbench/stream" > "$OUT/cal_$c.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$OUT/bench_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_$c.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$OUT/c4_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c4_$c.log" 2>&1 || exit $?
done
cd "$ROOT" && python3 scripts/traffic_summary.py "${1:-r01}" > "$OUT/summary.log" 2>&1 || exit $?
echo traffic passes ok
