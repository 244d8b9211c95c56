#!/bin/bash
# Round 4: the FlowLM out projection in 4 K slices of 256 (k_gemv<1, 64>: 128 workgroups, 4 slabs
# for the out reduce) instead of 8 of 128 - the step parity tests on the probe build with the knob
# set, then A/B (PTTS_OUT64=1 against the product's 8 slices), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_OUT64 REPS=3 VALUES="- 1" bash tools/sweep_env.sh
