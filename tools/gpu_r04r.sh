#!/bin/bash
# Round 4: per-op intervals of the frame-pair bench's front and back graphs (probe build, a stamp
# kernel ahead of every op: tools/op_stamps.py), product tiles; then the same with the front's GEMM
# weights / MFMAs / cached K-V skipped (PTTS_FRONT_SKIP=7, results wrong).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
for v in 0 7; do
  PTTS_FRONT_SKIP=$v PTTS_STAMP_OPS=1 PTTS_STAMPS=$OUT/opst_fs$v.txt timeout -k 10 200 python bench.py --no-cpu-baseline \
    --no-quant-variant --no-latency --no-op-times > $OUT/opst_fs$v.log 2>&1 || { tail -5 $OUT/opst_fs$v.log; exit 1; }
  tail -1 $OUT/opst_fs$v.log | cut -c1-250
  python tools/op_stamps.py $OUT/opst_fs$v.txt $OUT/opst_fs$v.json > $OUT/opst_fs$v.summary
  head -3 $OUT/opst_fs$v.summary
done
