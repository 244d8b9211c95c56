# Frame-pair back passes (BF=2) bound by the front part: register-resident qkv / linear1
# (PTTS_GEMV_MASK 31 = every FlowLM matrix, 27 = + qkv, 30 = + linear1; product 26) against the
# single-frame product configuration, probe build, same box.
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
VAR=PTTS_GEMV_MASK VALUES="- 31" REPS=3 BF=1 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/gemv_bf1.log 2>&1
grep MEDIAN gpurun_out/gemv_bf1.log
VAR=PTTS_GEMV_MASK VALUES="- 31 27 30" REPS=3 BF=2 timeout -k 10 400 python -u tools/env_ab.py > gpurun_out/gemv_bf2.log 2>&1
grep MEDIAN gpurun_out/gemv_bf2.log
