#!/bin/bash
# Round 4: front_commit requests the next step's input-projection / norm1 operands at its start
# (in flight with the slot-state loads) - parity tests, then the product bench against the
# previous library (lib-base), alternating, both back-pass modes (tools/bf_ab.sh).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT; rm -f $OUT/ab_summary.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest_fc.log 2>&1 || { tail -n 40 $OUT/pytest_fc.log; exit 1; }
tail -n 1 $OUT/pytest_fc.log
bash tools/bf_ab.sh
