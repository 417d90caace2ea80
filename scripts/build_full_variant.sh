#!/bin/bash
# Full A/B build of librtamd.so (host and kernels) with extra defines, in its own object directory:
#   scripts/build_full_variant.sh NAME "-DFOO=1"   ->  real-time-gpu-ray-tracer_amd/lib/librtamd_NAME.so
#   SRCDIR=/path/to/other/csrc (optional): build another source tree (e.g. a git worktree of HEAD)
set -e
cd "${SRCDIR:-$(dirname "$0")/../real-time-gpu-ray-tracer_amd/csrc}"
NAME=$1; FLAGS=$2
LIBDIR=$(cd "$(dirname "$0")" 2>/dev/null; pwd)
OUTLIB=${OUTLIB:-$(realpath -m ../lib)/librtamd_$NAME.so}
make -s -j8 OBJ=../build_$NAME LIB="$OUTLIB" \
  COMMON="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS" 2>&1 | grep -E "error" || true
ls -la "$OUTLIB"
