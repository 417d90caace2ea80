#!/bin/bash
# Build an A/B variant of librtamd.so whose GPU BVH builder (lbvh.hip) gets extra defines:
#   scripts/build_lbvh_variant.sh NAME "-DFOO=1"   ->  real-time-gpu-ray-tracer_amd/lib/librtamd_NAME.so  (RTAMD_LIB=...)
set -e
cd "$(dirname "$0")/../real-time-gpu-ray-tracer_amd/csrc"
make -s
NAME=$1; FLAGS=$2
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -ffp-contract=off $FLAGS -c lbvh.hip -o ../build/lbvh_$NAME.o
objs=""
for o in rt_api trace_exact trace_fast trace_fastmath assemble schedule vtk_reader comm instances interactive; do objs="$objs ../build/$o.o"; done
$HIPCC -shared -fPIC --offload-arch=gfx950 -o ../lib/librtamd_$NAME.so $objs ../build/lbvh_$NAME.o -ldl
echo "built ../lib/librtamd_$NAME.so"
