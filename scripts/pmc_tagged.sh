#!/bin/bash
# PMC passes of one bench workload, summarised with the workload's tag (bench.py --print-pmc-tag: config,
# builder, kernel, options, library hash) so bench.py prices `traffic` only with counters of that workload.
# usage: pmc_tagged.sh OUTDIR -- <bench.py args>      (runs: python3 bench.py <args> --steps 5 --warmup 2 --overlap 1)
# One counter group per rocprofv3 run (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2: never together).
OUT=$1; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p "$OUT"
python3 bench.py "$@" --print-pmc-tag > "$OUT/tag.json" || exit 1
PASSES=("FETCH_SIZE" "WRITE_SIZE" ${PMC_EXTRA:+"$PMC_EXTRA"})
if [ "${PMC_SET:-}" = "deep" ]; then   # occupancy, lane utilisation, L2 / L1 behaviour of the same workload (verdict r4 3)
  PASSES+=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM"
           "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum")
fi
dirs=()
i=0
for p in "${PASSES[@]}"; do
  d="$OUT/pass$i"
  echo "=== pmc pass $i: $p"
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $p -d "$d" -o run --output-format csv -- \
      python3 bench.py "$@" --steps ${PMC_STEPS:-5} --warmup 2 --overlap 1 --no-cpu-baseline > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
  dirs+=("$d")
  i=$((i+1))
done
python3 scripts/pmc_summary.py "$OUT/summary.json" "render_persistent_kernel<false" "${dirs[@]}" --tag "$OUT/tag.json" \
    --cmd "bench.py $* --steps ${PMC_STEPS:-5} --warmup 2 --overlap 1"
