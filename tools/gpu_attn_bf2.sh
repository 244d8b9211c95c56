# FlowLM step attention splits (probe build, PTTS_ATTN_VAR: 1 = 4 waves x 64 keys, 2 = 8 x 32,
# (the PTTS_ATTN_VAR knob was a temporary probe-build patch, removed after this measurement)
# 3 = 4 x 48, 4 = 8 x 16; default 4 x 32) under frame-pair stepping, where the front part bounds
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
VAR=PTTS_ATTN_VAR VALUES="- 1 2 3 4" REPS=3 BF=2 timeout -k 10 500 python -u tools/env_ab.py > gpurun_out/attn_bf2.log 2>&1
grep MEDIAN gpurun_out/attn_bf2.log
