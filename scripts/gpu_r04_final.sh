#!/bin/bash
# Final round-4 pass on the current build (scripts/gpu_r04_pass.sh: suite, smoke, traffic, bench lines, configs,
# rocprof stats, wave-cycle accounting), then study A/Bs that need no rebuild.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04}
CFG="c3 c4 c5 f ops" bash scripts/gpu_r04_pass.sh $TAG || exit $?
bash scripts/ab_sets.sh ${TAG}_ab c2 3 - HDD_DEBUG_FLAGS=67108864 || exit 1
bash scripts/ab_sets.sh ${TAG}_ab c4 2 - HDD_DEBUG_FLAGS=67108864 HDD_DEBUG_FLAGS=1048576 || exit 1
