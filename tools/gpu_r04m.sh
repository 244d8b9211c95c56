#!/bin/bash
# Round 4: shared voice prefixes (slots read positions < F from the voice's own KV cache, no
# copy-on-admit): GPU parity over the paths that read the FlowLM cache (steps, batched admission,
# long prompts, the bench shape, configs), then the product bench against lib-base (tools/bf_ab.sh).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT; rm -f $OUT/ab_summary.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py \
  tests/test_voice_frontend.py tests/test_gpu_configs.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $OUT/pytest_shared.log 2>&1 || { tail -n 40 $OUT/pytest_shared.log; exit 1; }
tail -n 1 $OUT/pytest_shared.log
bash tools/bf_ab.sh
