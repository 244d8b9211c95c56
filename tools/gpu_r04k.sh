#!/bin/bash
# Round 4: linear2 on gemv_fk in 4 K slices (A = linear1 output in fragment order) - parity tests,
# then A/B on the probe build (PTTS_NO_FK2=1 restores the k_gemv linear2), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_fk2.log 2>&1 || { tail -n 40 $OUT/pytest_fk2.log; exit 1; }
tail -n 1 $OUT/pytest_fk2.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_FK2 REPS=4 VALUES="- 1" bash tools/sweep_env.sh
