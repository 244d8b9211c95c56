#!/bin/bash
# Round 4: the out projection's row reduce + norm2 folded into the fused feed-forward launch
# (FfnArgs::Pin: workgroups 0..7 reduce 128 columns each and publish them with their row
# statistics; every wave LayerNorms its own A fragment) - parity tests over the step paths, then
# A/B on the probe build (PTTS_NO_FFN_RED=1: the reduce as its own launch), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest_ffnred.log 2>&1 || { tail -n 40 $OUT/pytest_ffnred.log; exit 1; }
tail -n 1 $OUT/pytest_ffnred.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_FFN_RED REPS=3 VALUES="- 1" bash tools/sweep_env.sh
