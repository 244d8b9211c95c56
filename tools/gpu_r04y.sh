#!/bin/bash
# Round 4: stream waits only for events still pending (Engine::wait_event: hipEventQuery first) -
# the pipelining / admission / streaming parity tests, then A/B on the probe build
# (PTTS_ALWAYS_WAIT=1: the unconditional GPU waits), interleaved, both back-pass modes.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py tests/test_gpu_serve.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $OUT/pytest_wait.log 2>&1 || { tail -n 40 $OUT/pytest_wait.log; exit 1; }
tail -n 1 $OUT/pytest_wait.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_ALWAYS_WAIT REPS=3 VALUES="- 1" bash tools/sweep_env.sh || exit 1
rm -f gpurun_out/sweep_all.txt
BENCH_ARGS="--back-frames 1" VAR=PTTS_ALWAYS_WAIT REPS=2 VALUES="- 1" bash tools/sweep_env.sh
