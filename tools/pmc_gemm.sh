#!/bin/bash
# PMC passes over single GEMM variants of tools/gemm_bench (one counter group per pass).
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_gemm; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
i=0
for spec in "conv0 0" "ff1 12 1" "convtr3 6" "convtr3 0" "ff2 0 1"; do
  j=0
  for P in "$P1" "$P2" "$P3"; do
    (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $P -d "$OUT/c${i}_p$j" -o run --output-format csv \
       -- "$ROOT/tools/bin/gemm_bench" $spec > "$OUT/c${i}_p$j.log" 2>&1) || exit $?
    j=$((j+1))
  done
  echo "$i: $spec" >> "$OUT/index.txt"
  i=$((i+1))
done
