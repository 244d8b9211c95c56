#!/bin/bash
# Round 4: frame pairs - the front waits for the back only at even calls (the pass it waits for
# also read the odd call's buffer), and a pass delivers both frames' PCM + meta with ONE copy node
# (pair blocks laid out contiguously) - parity tests, then the product bench against the previous
# library (lib-base), alternating, both back-pass modes (tools/bf_ab.sh).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT; rm -f $OUT/ab_summary.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py tests/test_gpu_serve.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $OUT/pytest_pair_io.log 2>&1 || { tail -n 40 $OUT/pytest_pair_io.log; exit 1; }
tail -n 1 $OUT/pytest_pair_io.log
bash tools/bf_ab.sh
