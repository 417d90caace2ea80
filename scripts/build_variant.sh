#!/bin/bash
# Build an A/B variant of librtamd.so whose FAST trace kernel gets extra defines:
#   scripts/build_variant.sh NAME "-DFOO=1 -DBAR=2"   ->  real-time-gpu-ray-tracer_amd/lib/librtamd_NAME.so
#   SRC=path/to/trace_kernel.hip (optional): another version of the kernel source (e.g. git show HEAD:...)
# (load it with RTAMD_LIB=...; everything else is the default build's objects)
set -e
cd "$(dirname "$0")/../real-time-gpu-ray-tracer_amd/csrc"
make -s
NAME=$1; FLAGS=$2
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-use-amdgpu-trackers -DRT_EXACT=0 -DRT_FAST_IEEE=1 -ffp-contract=off $FLAGS \
  -I. -I$PWD -c ${SRC:-trace_kernel.hip} -o ../build/trace_fast_$NAME.o
objs=""
for o in rt_api trace_exact trace_fastmath assemble schedule lbvh vtk_reader comm instances interactive; do objs="$objs ../build/$o.o"; done
$HIPCC -shared -fPIC --offload-arch=gfx950 -o ../lib/librtamd_$NAME.so $objs ../build/trace_fast_$NAME.o -ldl
echo "built ../lib/librtamd_$NAME.so"
