#!/bin/bash
# Round 4: frame-pair Mimi attention with RoPE + ring append fused in (the second frame's
# workgroups append the first frame's keys themselves; no separate qkv_rope launch) - parity tests,
# then A/B on the probe build (PTTS_PAIR_ROPE=1: the separate launch), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py tests/test_gpu_bf16.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $OUT/pytest_pairrope.log 2>&1 || { tail -n 40 $OUT/pytest_pairrope.log; exit 1; }
tail -n 1 $OUT/pytest_pairrope.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_PAIR_ROPE REPS=3 VALUES="- 1" bash tools/sweep_env.sh
