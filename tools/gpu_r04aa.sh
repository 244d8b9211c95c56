#!/bin/bash
# Round 4: the back part's row reduces four rows per 512-thread workgroup (one capped round; now also
# round instead of four) - parity tests, then A/B on the probe build (PTTS_NO_RR4=1: one row per
# workgroup), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py tests/test_voice_frontend.py tests/test_gpu_refdata.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $OUT/pytest_rr4.log 2>&1 || { tail -n 40 $OUT/pytest_rr4.log; exit 1; }
tail -n 1 $OUT/pytest_rr4.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_RR4 REPS=3 VALUES="- 1" bash tools/sweep_env.sh
