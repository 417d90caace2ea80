#!/bin/bash
# r05 session 36: where C2's WRITE_SIZE goes — the default library against one whose pixel stores are switched
# off at run time (diagnostic build of trace_kernel.hip, same code otherwise); C2 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s36; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
for cfg in C2 C3; do
  for v in default nostore; do
    lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
    RTAMD_LIB=$lib PMC_STEPS=5 timeout -k 10 400 bash scripts/pmc_tagged.sh $O/pmc_${cfg}_$v -- --config $cfg > $O/pmc_${cfg}_$v.log 2>&1 || { echo "pmc fail $cfg $v"; tail -5 $O/pmc_${cfg}_$v.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/pmc_${cfg}_$v/summary.json')); print('$cfg $v write MB', round(d['write_bytes_per_launch']/1e6,2), 'fetch MB', round(d['fetch_bytes_per_launch_corrected']/1e6,2))"
    rm -rf $O/pmc_${cfg}_$v/pass*
  done
done
