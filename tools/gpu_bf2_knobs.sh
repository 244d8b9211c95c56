# Frame-pair stepping (the bench default) under the probe build's front-priority and back-cap
# knobs, same box, three alternating rounds each
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
VAR=PTTS_FRONT_PRIO VALUES="- 1 2 3" REPS=3 BF=2 timeout -k 10 400 python -u tools/env_ab.py > gpurun_out/bf2_prio.log 2>&1
grep MEDIAN gpurun_out/bf2_prio.log
VAR=PTTS_BACK_WG_CAP VALUES="- 2" REPS=3 BF=2 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/bf2_cap.log 2>&1
grep MEDIAN gpurun_out/bf2_cap.log
