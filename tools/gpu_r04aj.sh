#!/bin/bash
# Round 4 (the front part bounds the frame-pair step again at the closing build): the issue
# priorities and the back workgroup cap re-measured - probe build of the closing sources, the back
# tile waves at priority 2 (PTTS_BACK_PRIO, product 3) and front waves at priority 3
# (PTTS_FRONT_PRIO, product 0); the probe library must not be gpurun-ignored for this run;
# steady ms/step, interleaved repeats.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_BACK_PRIO REPS=3 VALUES="- 2" bash tools/sweep_env.sh || exit 1
VAR=PTTS_FRONT_PRIO REPS=3 VALUES="- 3" bash tools/sweep_env.sh
