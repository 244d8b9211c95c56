# Frame pairs: which FlowLM matrices should be register-resident (PTTS_GEMV_MASK bits: 1 qkv,
# 2 out, 4 linear1, 8 linear2, 16 adaLN; pair default 31), probe build, same box
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
VAR=PTTS_GEMV_MASK VALUES="- 23 29 30 15" REPS=3 BF=2 timeout -k 10 500 python -u tools/env_ab.py > gpurun_out/bf2_mask.log 2>&1
grep MEDIAN gpurun_out/bf2_mask.log
