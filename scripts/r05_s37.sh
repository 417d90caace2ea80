#!/bin/bash
# r05 session 37: traversal-stack page-outs per frame (diagnostic build counting each page-out as a triangle test:
# page-outs = its triangle tests - the default's), C2 / C3 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s37; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
for cfg in C2 C3; do
  for v in default pgcount; do
    lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
    RTAMD_LIB=$lib timeout -k 10 300 python3 scripts/work_counts.py --config $cfg --tag $v > $O/wc_${cfg}_$v.log 2>&1 || { echo "fail $cfg $v"; tail -5 $O/wc_${cfg}_$v.log; exit 1; }
    cat $O/wc_${cfg}_$v.log
  done
done
