#!/bin/bash
# r05 session 16: tagged PMC of the current library: C2 deep (occupancy, lane use, L2/L1), C3/C5 FETCH/WRITE
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s16; mkdir -p $O
export TMPDIR=/tmp
PMC_SET=deep bash scripts/pmc_tagged.sh $O/pmc_C2 -- --config C2 || exit 1
bash scripts/pmc_tagged.sh $O/pmc_C3 -- --config C3 || exit 1
PMC_STEPS=3 bash scripts/pmc_tagged.sh $O/pmc_C5 -- --config C5 --build lbvh || exit 1
for c in C2 C3 C5; do python3 -c "
import json; d=json.load(open('$O/pmc_$c/summary.json')); print('$c', json.dumps({k: v for k, v in d.items() if k not in ('cmd','tag')})[:1500])"; done
