#!/bin/bash
# Round 4 step 29: smoke and the full-frame parity file on the final library
set -o pipefail
O=gpurun_out/r04s29; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -q -rf -s --timeout 500 --timeout-method thread tests/test_gpu_parity_full.py > $O/parity_full.log 2>&1
tail -3 $O/parity_full.log
