#!/bin/bash
# Round 4: the FlowLM step attention fused with the out projection (attention_step_out: the 32
# workgroups of a head hand their outputs to each other, then each multiplies them by 32 columns of
# the out projection into a per-head slab) - parity tests over the step paths, then A/B on the probe
# build (PTTS_NO_AO=1 restores the out GEMM launch), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest_ao.log 2>&1 || { tail -n 40 $OUT/pytest_ao.log; exit 1; }
tail -n 1 $OUT/pytest_ao.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_AO REPS=3 VALUES="- 1" bash tools/sweep_env.sh
