#!/bin/bash
# A/B of one scene option on bench lines (interleaved runs in one call).
# usage: OPT=name [VALS="0 1"] scripts/ab.sh OUTNAME   (runs each case with --opt $OPT=v for v in VALS, REPS times)
#        OPT=lib VALS="default nocons" ...                  (library A/B: RTAMD_LIB=lib/librtamd_$v.so, "default" = the build)
#        OPT=opts VALS="base wide_order=0 wide_order=0,tlas_sah=1"   (option sets: comma-separated k=v, "base" = none)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
OPT=${OPT:?set OPT=option}
REPS=${REPS:-2}
CASES=${CASES:-"c2_20|--steps 20 --warmup 5;c2_100|--steps 100;share8|--steps 100 --shard 0/8;c3|--config C3 --steps 40;lbvh_rb|--build lbvh --rebuild --steps 60"}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
for rep in $(seq 1 $REPS); do
  IFS=';' read -ra CS <<< "$CASES"
  for c in "${CS[@]}"; do
    name=${c%%|*}; args=${c#*|}
    for v in ${VALS:-0 1}; do
      if [ "$OPT" = lib ]; then
        if [ "$v" = default ]; then lib=""; else lib=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_$v.so; fi
        RTAMD_LIB=$lib timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > $OUT/${name}_${v}_$rep.log 2>&1
      elif [ "$OPT" = opts ]; then
        oa=""; [ "$v" != base ] && for kv in ${v//,/ }; do oa="$oa --opt $kv"; done
        timeout -k 10 300 python3 bench.py $args --no-cpu-baseline $oa > $OUT/${name}_${v}_$rep.log 2>&1
      else
        timeout -k 10 300 python3 bench.py $args --no-cpu-baseline --opt $OPT=$v > $OUT/${name}_${v}_$rep.log 2>&1
      fi
      rc=$?
      if [ $rc -ne 0 ]; then echo "$name $v rc=$rc"; tail -5 $OUT/${name}_${v}_$rep.log; exit $rc; fi
      python3 - "$OUT/${name}_${v}_$rep.log" "$name" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:8s} opt={sys.argv[3]} ms/frame {d['ms_per_step']:.4f}  Mrays/s {d['value']:.0f}  serial {d['kernel_ms']:.4f}  lat {d['frame_latency_ms_median']:.4f}", flush=True)
PY
    done
  done
done
exit 0
