#!/bin/bash
# Same-box A/B of an environment switch (e.g. HDD_DYN=1) on the C2 / C4 bench lines: GPU parity suite with
# the switch on, then alternating runs.  usage: ab_env.sh NAME=VALUE [tag]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SW=$1; TAG=${2:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
env $SW timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest($SW) rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for w in c2 c4; do
    for v in on off; do
      if [ $v = on ]; then E="$SW"; else E="HDD_AB_OFF=1"; fi
      env $E timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${w}_${v}_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $w $v rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.4f ms' % d['ms_per_step'], '%.3g' % d['value'], round(d['roofline']['frac'], 4))" $OUT/${w}_${v}_$rep.log $w $v
    done
  done
done
