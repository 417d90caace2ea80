#!/bin/bash
# rocprofv3 PMC passes (one counter group per run; --pmc is never combined with tracing domains).
# usage: pmc_passes.sh OUTDIR KERNEL_SUBSTRING -- command...
# (TA_* counters are left out: a pass collecting them hung the box once in round 1.)
OUT=$1; KSUB=$2; shift 3
export TMPDIR=/tmp
mkdir -p "$OUT"
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
)
if [ "${PMC_SET:-}" = "deep" ]; then   # latency / front-end breakdown of the persistent kernel
PASSES=(
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VSKIPPED"
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_FLAT"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
)
fi
i=0
dirs=()
for p in "${PASSES[@]}"; do
  d="$OUT/pass$i"
  echo "=== pmc pass $i: $p"
  timeout -k 10 300 rocprofv3 --pmc $p -d "$d" -o run --output-format csv -- "$@" > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; if [ $rc -ne 1 ]; then break; fi; fi
  dirs+=("$d")
  i=$((i+1))
done
python3 scripts/pmc_summary.py "$OUT/summary.json" "$KSUB" "${dirs[@]}"
