#!/bin/bash
# Round 4 (the front part bounds the frame-pair step again at the closing build): the FlowLM step
# attention's waves x keys re-measured - probe build, PTTS_ATT 416 (4 waves x 64 keys) and 88
# (8 waves x 32) against the product's 4 x 32; the GPU parity tests of the step paths on the probe
# build with each; steady ms/step, interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_ATT REPS=3 VALUES="- 416 88" bash tools/sweep_env.sh
