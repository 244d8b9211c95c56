#!/bin/bash
# Round 4: whole-K linear1 (gemv_fk, GELU in its epilogue, no ff1 reduce launch) - parity tests,
# then A/B on the probe build (PTTS_NO_FK=1 restores split-K linear1 + its reduce), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_fk.log 2>&1 || { tail -n 40 $OUT/pytest_fk.log; exit 1; }
tail -n 1 $OUT/pytest_fk.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_FK REPS=4 VALUES="- 1" bash tools/sweep_env.sh
