#!/bin/bash
# r05 session 39: are queue claims (device-scope atomics, counted as TCC_EA write requests) part of C2's WRITE_SIZE?
# library without pixel stores, screen walk (reorder 0), 64 / 256 / 1024 pixels per claim
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s39; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
for g in 64 256 1024; do
  d=$O/w$g
  RTAMD_LIB=$L/librtamd_nostore.so timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $d -o run --output-format csv -- \
      python3 bench.py --opt reorder=0 --opt grab=$g --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline > $O/w$g.log 2>&1 || { echo "fail $g"; tail -5 $O/w$g.log; exit 1; }
  echo "=== nostore reorder 0 grab $g"; python3 scripts/pmc_kernels.py $d | grep render_persistent_kernel.false
  rm -rf $d
done
