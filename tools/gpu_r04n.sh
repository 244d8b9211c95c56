#!/bin/bash
# Round 4: what bounds the frame-pair step at the shared-voice build. (1) graph stamps (probe build,
# PTTS_STAMPS: s_memrealtime at the start / end of every front and back graph) of the bench in both
# back-pass modes -> tools/stamps.py timelines; (2) the bench with the back part's GEMM / conv
# tiles skipping their MFMAs (PTTS_BACK_PROBE=1) or MFMAs and operand loads (3), results wrong.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
for bf in 2 1; do
  PTTS_STAMPS=$OUT/stamps_bf$bf.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-latency \
    --no-op-times --back-frames $bf > $OUT/stamps_bf$bf.log 2>&1 || { tail -5 $OUT/stamps_bf$bf.log; exit 1; }
  tail -1 $OUT/stamps_bf$bf.log | cut -c1-330
  python tools/stamps.py $OUT/stamps_bf$bf.txt $OUT/stamps_bf$bf.json
done
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_BACK_PROBE REPS=2 VALUES="- 1 3" bash tools/sweep_env.sh
