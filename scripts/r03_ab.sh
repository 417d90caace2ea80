#!/bin/bash
# round-3 A/B: smoke + GPU tests + bench, then alternating library A/B (scripts/ab_libs.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-smoke,tests,bench} bash scripts/gpu_check.sh || exit $?
grep -q "rc=0\|rc=1" gpurun_out/summary.log || exit 1
[ -n "$AB" ] && { bash scripts/ab_libs.sh ${REPS:-3} "$AB" ${AB_ARGS:-} || exit $?; }
[ -n "$AB2" ] && { bash scripts/ab_libs.sh ${REPS2:-1} "$AB2" ${AB2_ARGS:-} || exit $?; }
exit 0
