#!/bin/bash
# Round 4: back-part tiles / split-K under frame pairs (M doubled): steady-step sweep of PTTS_OVR
# on the probe build, interleaved repeats (tools/sweep_env.sh).
set -u
cd "$(dirname "$0")/.."
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_OVR REPS=${REPS:-3} VALUES="${VALUES:-- seanet.up0.convtr=32:1 seanet.conv0=32:1 seanet.conv0=32:2 mimi.ff2=32:2 mimi.out=32:2 mimi.out=32:1 mimi.qkv=35 mimi.ff1=35 seanet.up1.convtr=35 seanet.up2.convtr=35 seanet.up0.convtr=32:1,seanet.conv0=32:2,mimi.ff2=32:2}" \
  bash tools/sweep_env.sh
