# What bounds the frame-pair step: back-part kernels with their operand loads (2) or loads and
# MFMAs (3) skipped (probe build, results wrong: bounds only)
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
VAR=PTTS_BACK_PROBE VALUES="- 2 3" REPS=2 BF=2 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/bf2_bp23.log 2>&1
grep MEDIAN gpurun_out/bf2_bp23.log
VAR=PTTS_FRONT_PROBE VALUES="- 1 3" REPS=2 BF=2 timeout -k 10 300 python -u tools/env_ab.py > gpurun_out/bf2_fp.log 2>&1
grep MEDIAN gpurun_out/bf2_fp.log
