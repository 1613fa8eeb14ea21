#!/bin/bash
# One parameterised GPU-box runner (replaces the per-session scripts/gpu_r0*.sh).  Every step runs under its own time
# limit; the first failing step ends the run (no GPU step after a fault / abort / timeout).
#
# usage: scripts/gpu.sh RUN STEP [STEP ...]      outputs under gpurun_out/RUN/
#   "tests [pytest args]"        python -m pytest -m gpu (default: the whole GPU suite)
#   "smoke"                      __graft_entry__.smoke()
#   "bench TAG [bench.py args]"  one bench.py line -> bench_TAG.log
#   "ab REPS TAG [bench args]"   alternating bench.py runs, REPS rounds over the trees in $AB_TREES (name=dir ...: dir holds
#                                that revision's bench.py, dune-hdd_amd/python and dune-hdd_amd/lib, e.g. ab/r04; "cur" or
#                                an empty dir = this tree) -> ab_TAG.log, one JSON line per run, prefixed by the name
#   "prof TAG [bench args]"      rocprofv3 --kernel-trace --stats of bench.py -> prof_TAG/
#   "pmc TAG [bench args]"       scripts/pmc_acct.sh (wave-cycle accounting + FETCH/WRITE_SIZE) -> pmc_TAG/ + summary
#   "traffic TAG"                scripts/traffic.sh (build-stamped PMC traffic of the bench workloads)
#   "py TAG LIMIT script.py [args]"  any study script under its own limit -> py_TAG.log
#   "env K=V"                    export K=V for the following steps (empty V: unset)
#   "sh TAG LIMIT cmd [args]"    any command under its own limit -> sh_TAG.log
#   "rocstats TAG script.py [args]"  rocprofv3 --kernel-trace --stats of a script -> rocstats_TAG/
#   "rocpmc TAG C1,C2,.. script.py [args]"  one rocprofv3 --pmc pass (kernel trace only) of a script -> rocpmc_TAG/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
RUN=$1; shift
OUT=$ROOT/gpurun_out/$RUN
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "step '$1' rc=$2 -- stopping"; exit "$2"; }
for step in "$@"; do
  eval "set -- $step"   # (a step may quote an argument: "tests -k 'sharded or watchdog'")
  kind=$1; shift
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread "$@" \
        > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || fail tests $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || fail smoke $rc ;;
    bench)
      tag=$1; shift
      timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$tag.log" 2>&1
      rc=$?; echo "bench $tag rc=$rc"; tail -1 "$OUT/bench_$tag.log" | cut -c1-400; [ $rc -eq 0 ] || fail "bench $tag" $rc ;;
    ab)
      reps=$1; tag=$2; shift 2
      for ((i = 0; i < reps; ++i)); do
        for nl in ${AB_TREES:-cur=}; do
          name=${nl%%=*}; dir=${nl#*=}
          [ "$name" = cur ] || [ -z "$dir" ] && dir=.
          timeout -k 10 300 python "$dir/bench.py" --no-cpu-baseline "$@" > "$OUT/ab_${tag}_last.log" 2>&1
          rc=$?
          [ $rc -eq 0 ] || { tail -5 "$OUT/ab_${tag}_last.log"; fail "ab $tag $name" $rc; }
          echo "$name $(tail -1 "$OUT/ab_${tag}_last.log")" >> "$OUT/ab_$tag.log"
          python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print('%-5s %s ms/step %.4f kernel %.4f frac %.3f' % (sys.argv[1], '$tag', d['ms_per_step'], r.get('step_ms_event', r.get('kernel_ms_avg', 0)), r['frac']))" "$name" "$(tail -1 "$OUT/ab_${tag}_last.log")"
        done
      done ;;
    prof)
      tag=$1; shift
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/prof_$tag.log" 2>&1)
      rc=$?; echo "prof $tag rc=$rc"; [ $rc -eq 0 ] || fail "prof $tag" $rc
      f=$(find "$OUT/prof_$tag" -name "*kernel_stats.csv" | head -1)
      [ -n "$f" ] && head -4 "$f" | cut -c1-220 ;;
    pmc)
      tag=$1; shift
      bash scripts/pmc_acct.sh "${RUN}_$tag" "$@" > "$OUT/pmc_$tag.log" 2>&1
      rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$OUT/pmc_$tag.log"; fail "pmc $tag" $rc; }
      python3 scripts/pmc_summary.py "gpurun_out/pmc_${RUN}_$tag" swipdg_persistent > "$OUT/pmc_${tag}_summary.md" 2>&1
      grep -A14 "wave-cycle accounting" "$OUT/pmc_${tag}_summary.md" | head -16 ;;
    traffic)
      bash scripts/traffic.sh "$1" > "$OUT/traffic.log" 2>&1
      rc=$?; echo "traffic rc=$rc"; tail -3 "$OUT/traffic.log"; [ $rc -eq 0 ] || fail traffic $rc ;;
    rocpmc)   # "rocpmc TAG COUNTER[,COUNTER...] script.py [args]": one --pmc pass (counters comma-separated) of a script
      tag=$1; ctrs=${2//,/ }; shift 2
      (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/rocpmc_$tag" -o run --output-format csv -- \
        python3 "$ROOT/$1" "${@:2}" > "$OUT/rocpmc_$tag.log" 2>&1)
      rc=$?; echo "rocpmc $tag rc=$rc"; tail -2 "$OUT/rocpmc_$tag.log" | cut -c1-300; [ $rc -eq 0 ] || fail "rocpmc $tag" $rc ;;
    rocstats)   # "rocstats TAG script.py [args]": kernel-trace stats of any script
      tag=$1; shift
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocstats_$tag" -o run --output-format csv -- \
        python3 "$ROOT/$1" "${@:2}" > "$OUT/rocstats_$tag.log" 2>&1)
      rc=$?; echo "rocstats $tag rc=$rc"; tail -2 "$OUT/rocstats_$tag.log" | cut -c1-300; [ $rc -eq 0 ] || fail "rocstats $tag" $rc ;;
    env)   # "env K=V": export for the following steps ("env K=" unsets K)
      k=${1%%=*}; v=${1#*=}
      if [ -z "$v" ]; then unset "$k"; else export "$k=$v"; fi
      echo "env $k=${v:-<unset>}" ;;
    sh)    # "sh TAG LIMIT cmd [args]": any command under its own limit -> sh_TAG.log
      tag=$1; lim=$2; shift 2
      timeout -k 10 "$lim" "$@" > "$OUT/sh_$tag.log" 2>&1
      rc=$?; echo "sh $tag rc=$rc"; tail -2 "$OUT/sh_$tag.log" | cut -c1-300; [ $rc -eq 0 ] || fail "sh $tag" $rc ;;
    py)
      tag=$1; lim=$2; shift 2
      timeout -k 10 "$lim" python -u "$@" > "$OUT/py_$tag.log" 2>&1
      rc=$?; echo "py $tag rc=$rc"; tail -4 "$OUT/py_$tag.log" | cut -c1-300; [ $rc -eq 0 ] || fail "py $tag" $rc ;;
    *)
      echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "gpu.sh $RUN done"
