#!/bin/bash
# PMC passes over register-blocked LDS-DMA GEMM variants of tools/gemm_bench (NOELU=1).
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_rb; mkdir -p "$OUT"; export TMPDIR=/tmp
export NOELU=1
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU"
i=0
for spec in "rb.convtr3m 21" "rb.convtr3m 6" "rb.mimi.ff2 21 1" "rb.convtr2m 22"; do
  j=0
  for P in "$P1" "$P3"; do
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/c${i}_p$j" -o run --output-format csv \
       -- "$ROOT/tools/bin/gemm_bench" $spec > "$OUT/c${i}_p$j.log" 2>&1) || exit $?
    j=$((j+1))
  done
  echo "$i: $spec" >> "$OUT/index.txt"
  i=$((i+1))
done
