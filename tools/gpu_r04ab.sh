#!/bin/bash
# Round 4: the back part's commit one workgroup per row (every history as float4 copies; one capped
# round instead of two) - parity tests, then the product bench against the previous library
# (lib-base), alternating, both back-pass modes (tools/bf_ab.sh).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT; rm -f $OUT/ab_summary.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py tests/test_voice_frontend.py tests/test_gpu_refdata.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $OUT/pytest_commit.log 2>&1 || { tail -n 40 $OUT/pytest_commit.log; exit 1; }
tail -n 1 $OUT/pytest_commit.log
bash tools/bf_ab.sh
