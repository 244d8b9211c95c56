#!/bin/bash
# Round 4: whole-K qkv (gemv_fk; the step attention sums one slab) - parity tests,
# then A/B on the probe build (PTTS_NO_FK_QKV=1 restores the split-K qkv), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_fk.log 2>&1 || { tail -n 40 $OUT/pytest_fk.log; exit 1; }
tail -n 1 $OUT/pytest_fk.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_FK_QKV REPS=4 VALUES="- 1" bash tools/sweep_env.sh
