#!/bin/bash
# Round 4: the back part bounds the frame-pair step (tools/stamps.py: back stream busy end to end,
# back MFMAs skipped -> 0.554 -> 0.484 ms). Knobs that favour it (probe build): issue priority of
# the back part's tile waves (PTTS_BACK_PRIO, s_setprio), and two back workgroups per CU
# (PTTS_BACK_WG_CAP=2); interleaved repeats (tools/sweep_env.sh).
set -u
cd "$(dirname "$0")/.."
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_BACK_PRIO REPS=2 VALUES="- 1 3" bash tools/sweep_env.sh || exit 1
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_BACK_WG_CAP REPS=2 VALUES="- 2" bash tools/sweep_env.sh
