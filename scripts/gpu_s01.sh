#!/bin/bash
# Round-6 session driver: selected GPU tests (K = pytest -k expression; NO_TESTS=1 skips them), then library A/Bs
# AB="vals|cases" pairs separated by '#' (vals: library variants of scripts/build_variant.sh, "default" = the build;
# cases: scripts/ab.sh CASES syntax).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
OUT=gpurun_out/${S_OUT:?set S_OUT}; mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest ${T:-tests/test_gpu_box.py tests/test_gpu_golden.py tests/test_gpu_edges.py tests/test_gpu_parity_full.py} -k "${K:-box or kats or crops or lane_priority or fast_equals_exact or fast_kernel_on_reference or survey_bars}" -v -s --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL|differ|outliers" $OUT/tests.log | tail -60
[ $rc -ne 0 ] && exit $rc
fi
IFS='#' read -ra ABS <<< "$AB"
i=0
for ab in "${ABS[@]}"; do
  i=$((i+1))
  OPT=lib VALS="${ab%%|*}" REPS=${REPS:-2} CASES="${ab#*|}" bash scripts/ab.sh $S_OUT/ab$i || exit 1
done
exit 0
