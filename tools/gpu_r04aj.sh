#!/bin/bash
# Round 4 (the front part bounds the frame-pair step again at the closing build): the issue
# priorities and the back workgroup cap re-measured - probe build of the closing sources, the back
# tile waves at priority 2 / 0 (PTTS_BACK_PRIO, product 3), front waves at priority 3
# (PTTS_FRONT_PRIO, product 0) and two back workgroups per CU (PTTS_BACK_WG_CAP, product 1);
# steady ms/step, interleaved repeats.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_BACK_PRIO REPS=3 VALUES="- 2 0" bash tools/sweep_env.sh || exit 1
VAR=PTTS_FRONT_PRIO REPS=3 VALUES="- 3 1" bash tools/sweep_env.sh || exit 1
VAR=PTTS_BACK_WG_CAP REPS=3 VALUES="- 2" bash tools/sweep_env.sh
