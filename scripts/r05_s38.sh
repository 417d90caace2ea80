#!/bin/bash
# r05 session 38: C2's write traffic without pixel stores (diagnostic library) — per kernel, with and without the
# claim reorder (schedule kernel + unit-cost atomics)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s38; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
i=0
for args in "" "--opt reorder=0" "--opt reorder=0 --opt lds_scene=0"; do
  d=$O/w$i
  RTAMD_LIB=$L/librtamd_nostore.so timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $d -o run --output-format csv -- \
      python3 bench.py $args --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline > $O/w$i.log 2>&1 || { echo "fail $i"; tail -5 $O/w$i.log; exit 1; }
  echo "=== nostore $args"; python3 scripts/pmc_kernels.py $d
  rm -rf $d; i=$((i+1))
done
d=$O/wdef
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $d -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline > $O/wdef.log 2>&1 || { echo "fail def"; exit 1; }
echo "=== default"; python3 scripts/pmc_kernels.py $d; rm -rf $d
