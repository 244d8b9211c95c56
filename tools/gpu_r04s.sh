#!/bin/bash
# Round 4: FlowLM feed-forward as ONE launch per layer (ffn_fused: linear1 + GELU, a group-local
# hand-off, linear2 slice) - parity tests over the step paths, then A/B on the probe build
# (PTTS_NO_FFN=1 restores the linear1 / linear2 launches), interleaved; back-part issue priority 3
# beside it; then per-op stamps of both FFN forms.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest_ffn.log 2>&1 || { tail -n 40 $OUT/pytest_ffn.log; exit 1; }
tail -n 1 $OUT/pytest_ffn.log
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_NO_FFN REPS=3 VALUES="- 1" bash tools/sweep_env.sh || exit 1
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_BACK_PRIO REPS=3 VALUES="- 3" bash tools/sweep_env.sh || exit 1
for v in 0 1; do
  if [ $v = 1 ]; then export PTTS_NO_FFN=1; else unset PTTS_NO_FFN; fi
  PTTS_STAMP_OPS=1 PTTS_STAMPS=$OUT/opst_ffn$v.txt timeout -k 10 200 python bench.py --no-cpu-baseline \
    --no-quant-variant --no-latency --no-op-times > $OUT/opst_ffn$v.log 2>&1 || { tail -5 $OUT/opst_ffn$v.log; exit 1; }
  python tools/op_stamps.py $OUT/opst_ffn$v.txt $OUT/opst_ffn$v.json > $OUT/opst_ffn$v.summary
  head -2 $OUT/opst_ffn$v.summary
done
