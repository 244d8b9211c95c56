#!/bin/bash
# Round-4 closing stamps (probe build of the closing sources): graph stamps (tools/stamps.py) and
# per-op stamps (tools/op_stamps.py) of the frame-pair bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
PTTS_STAMPS=$OUT/close_graph.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-latency \
  --no-op-times > $OUT/close_graph.log 2>&1 || { tail -5 $OUT/close_graph.log; exit 1; }
python tools/stamps.py $OUT/close_graph.txt $OUT/close_graph.json
PTTS_STAMP_OPS=1 PTTS_STAMPS=$OUT/close_ops.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant \
  --no-latency --no-op-times > $OUT/close_ops.log 2>&1 || { tail -5 $OUT/close_ops.log; exit 1; }
python tools/op_stamps.py $OUT/close_ops.txt $OUT/close_ops.json > $OUT/close_ops.summary
head -2 $OUT/close_ops.summary
