#!/bin/bash
# Round 4: the hand-off timeout word in host-mapped memory (no copy node at the end of every front
# graph): GPU parity subset, then the product bench against the previous library (lib-base),
# alternating, both back-pass modes (tools/bf_ab.sh).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 300 \
  --timeout-method thread > $OUT/pytest_err.log 2>&1 || { tail -n 30 $OUT/pytest_err.log; exit 1; }
tail -n 1 $OUT/pytest_err.log
bash tools/bf_ab.sh
