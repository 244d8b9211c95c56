#!/bin/bash
# Round 4: the fused feed-forward in 8 groups of 32 (linear2 K slices of 512: 8 slabs for the ff2
# reduce instead of 16) - parity tests, then A/B on the probe build (PTTS_FFN16=1: 16 groups of
# 16), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest_ffn8.log 2>&1 || { tail -n 40 $OUT/pytest_ffn8.log; exit 1; }
tail -n 1 $OUT/pytest_ffn8.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_FFN16 REPS=3 VALUES="- 1" bash tools/sweep_env.sh
