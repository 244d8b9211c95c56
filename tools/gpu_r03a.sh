#!/bin/bash
# Round-3 GPU session: parity tests, the default bench, the GEMM-core microbenchmark, and a sweep of
# the back part's tile choices in the pipelined step (probe build, PTTS_OVR). Each GPU step has its
# own time limit; a failure stops the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfP --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -n 40 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline --ops-out $OUT/bench_ops.json > $OUT/bench.log 2>&1 \
    || { echo "bench failed"; tail -n 20 $OUT/bench.log; exit 1; }
tail -n 1 $OUT/bench.log | cut -c1-700
if [ "${MMB:-1}" = "1" ]; then
  timeout -k 10 300 ./gpubin/mm_bench > $OUT/mm_bench.log 2>&1 || { echo "mm_bench failed"; tail -n 20 $OUT/mm_bench.log; exit 1; }
  grep -c BAD $OUT/mm_bench.log || true
fi
if [ -n "${SWEEP:-}" ]; then
  PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so VAR=${SWEEP_VAR:-PTTS_OVR} VALUES="$SWEEP" REPS=${REPS:-2} \
      bash tools/sweep_env.sh > $OUT/sweep.log 2>&1 || { echo "sweep failed"; tail -n 20 $OUT/sweep.log; exit 1; }
  grep median $OUT/sweep.log
fi
if [ -f gpubin/devlib/libprobes.so ] && [ "${DEVX:-1}" = "1" ]; then  # experiments on a working-copy probe build
  MMB_CAP=1 timeout -k 10 300 ./gpubin/mm_bench mimi > $OUT/mm_bench_cap1_mimi.log 2>&1 || { echo "mm_bench cap failed"; exit 1; }
  MMB_CAP=1 timeout -k 10 300 ./gpubin/mm_bench conv > $OUT/mm_bench_cap1_conv.log 2>&1 || { echo "mm_bench cap failed"; exit 1; }
  L40="mimi.qkv=40,mimi.out=40:4,mimi.ff1=40,mimi.ff2=40:4,seanet.conv0=40:4,seanet.up0.convtr=40:4,seanet.up1.convtr=40,seanet.up2.convtr=40"
  PTTS_LIB=gpubin/devlib/libprobes.so VAR=PTTS_OVR VALUES="- $L40" REPS=2 bash tools/sweep_env.sh > $OUT/sweep40.log 2>&1 \
      || { echo "sweep40 failed"; tail -n 5 $OUT/sweep40.log; exit 1; }
  grep median $OUT/sweep40.log
fi
exit 0
