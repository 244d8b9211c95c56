#!/bin/bash
# Round 4: GEMM-core and bf16-back tests, the bench with its variants, then the L2-prefetch A/B
# (probe build, PTTS_NO_PF=1 turns the row reduces' prefetch side job off), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_r04c.sh || exit 1
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_PF REPS=4 VALUES="- 1" bash tools/sweep_env.sh
