# Is the frame-pair step bound by the back part? (probe build, same box): back MFMAs skipped
# (PTTS_BACK_PROBE=1, results wrong: a bound only), persistent back tiles (layout 41), per-op
# caps of 2 for the heaviest SEANet convs
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
VAR=PTTS_BACK_PROBE VALUES="- 1" REPS=2 BF=2 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/bf2_bp.log 2>&1
grep MEDIAN gpurun_out/bf2_bp.log
O41="mimi.qkv=41,mimi.out=41:4,mimi.ff1=41,mimi.ff2=41:4,seanet.conv0=41:4,seanet.up0.convtr=41:4,seanet.up1.convtr=41,seanet.up2.convtr=41"
VAR=PTTS_OVR VALUES="- $O41" REPS=3 BF=2 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/bf2_ovr.log 2>&1
grep MEDIAN gpurun_out/bf2_ovr.log
VAR=PTTS_OP_CAP VALUES="- seanet.up2.convtr=2 seanet.up1.convtr=2" REPS=2 BF=2 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/bf2_opcap.log 2>&1
grep MEDIAN gpurun_out/bf2_opcap.log
