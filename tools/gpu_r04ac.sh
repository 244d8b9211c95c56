#!/bin/bash
# Round-4 closing evidence session at the product build: the full GPU test suite, a same-box A/B of
# the event records trimmed to the ones waited for (frame pairs) against the previous library
# (lib-base, tools/bf_ab.sh), then tools/gpu_r04e.sh's default bench line and the profiles of the
# measured configuration (kernel trace, PMC passes, serving load). First failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT; rm -f $OUT/ab_summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -n 40 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
bash tools/bf_ab.sh || exit 1
timeout -k 10 900 python bench.py > $OUT/bench_default.log 2>&1 || { tail -n 20 $OUT/bench_default.log; exit 1; }
tail -n 1 $OUT/bench_default.log | cut -c1-400
bash tools/gpu_r03b.sh
