#!/bin/bash
# Round 4: whole-K out projection (residual + norm2 statistics in its epilogue, linear1 LayerNorms
# its A in registers: no out reduce launch) - parity tests, then A/B on the probe build
# (PTTS_NO_FK_OUT=1 restores the out split-K GEMM + reduce), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_streaming.py tests/test_gpu_refdata.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_fko.log 2>&1 \
  || { tail -n 40 $OUT/pytest_fko.log; exit 1; }
tail -n 1 $OUT/pytest_fko.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_FK_OUT REPS=4 VALUES="- 1" bash tools/sweep_env.sh
