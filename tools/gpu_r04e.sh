#!/bin/bash
# Round-4 evidence session at the product build: the GPU test suite, the default bench line
# (CPU baseline, first-chunk latency, variants, per-op times), then tools/gpu_r03b.sh's kernel
# trace / PMC passes of the measured configuration (frame pairs) and the HTTP serving load
# (serve.py's default, back_frames 2). First failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -n 40 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 900 python bench.py > $OUT/bench_default.log 2>&1 || { tail -n 20 $OUT/bench_default.log; exit 1; }
tail -n 1 $OUT/bench_default.log | cut -c1-400
bash tools/gpu_r03b.sh
