#!/bin/bash
# Evidence session for the MEASURED configuration (pipelined frame-pair stepping, bench.py's
# default): the bench line with per-op timings at the job midpoint (--ops-out), a rocprofv3
# kernel trace + stats of the bench attributed per op and per part (tools/prof_ops.py piped), the
# PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy; one counter group per run, each under its own
# kill timer) attributed per op, and optionally the HTTP serving load test (SERVE=1). Outputs under
# gpurun_out/; copy the summaries to profiles/rNN/. The first failure ends the script (no retries).
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
FR=${FRAMES:-30}
NOVAR="--no-cpu-baseline --no-quant-variant --no-latency --no-distinct-voices --no-voice-bench --no-text-bench"
timeout -k 10 300 python bench.py $NOVAR --ops-out "$OUT/bench_ops.json" > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
tail -n 1 "$OUT/bench.json" | cut -c1-300
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python "$ROOT/bench.py" --warmup 5 --profile-frames $FR $NOVAR --no-op-times > "$OUT/prof.log" 2>&1) \
  || { echo "rocprof trace failed"; tail -n 20 "$OUT/prof.log"; exit 1; }
python tools/prof_ops.py piped "$OUT/prof/run_kernel_trace.csv" "$OUT/bench_ops.json" "$OUT/op_stats.csv" \
    "$OUT/piped_steps.json" || exit 1
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  T=$(echo "$C" | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$T" -o run --output-format csv \
      -- python "$ROOT/bench.py" --profile-frames ${PMC_FRAMES:-12} --warmup 2 $NOVAR --no-op-times > "$OUT/pmc_$T.log" 2>&1) \
    || { echo "pmc $C failed"; tail -n 5 "$OUT/pmc_$T.log"; exit 1; }
  for c in $C; do
    python tools/prof_ops.py counters "$OUT/pmc_$T/run_counter_collection.csv" "$OUT/bench_ops.json" $c \
        "$OUT/pmc_$c.json" || exit 1
  done
done
python tools/prof_ops.py traffic "$OUT/pmc_FETCH_SIZE.json" "$OUT/pmc_WRITE_SIZE.json" "$OUT/traffic.json" || exit 1
python tools/prof_ops.py mfma "$OUT/pmc_SQ_VALU_MFMA_BUSY_CYCLES.json" "$OUT/pmc_GRBM_GUI_ACTIVE.json" \
    "$OUT/op_stats.csv" "$OUT/mfma.json" || exit 1
if [ "${SERVE:-0}" = "1" ]; then
  timeout -k 10 420 python tools/serve_load.py --rounds ${ROUNDS:-5} --seconds ${SECONDS_PER_ROUND:-6} \
      --out "$OUT/serve_load.json" > "$OUT/serve_load.log" 2>&1 || { echo "serve_load failed"; tail -n 20 "$OUT/serve_load.log"; exit 1; }
  tail -n 4 "$OUT/serve_load.log"
fi
exit 0
