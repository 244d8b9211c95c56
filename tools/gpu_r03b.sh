#!/bin/bash
# Round-3 evidence session for the MEASURED configuration (pipelined stepping): rocprofv3
# kernel-trace of the bench attributed per op and per part (tools/prof_ops.py piped), the PMC
# passes of the pipelined bench (FETCH_SIZE, WRITE_SIZE, MFMA busy; one counter group per run,
# attributed per op), then the HTTP serving load test. Every GPU step has its own time limit;
# the first failure ends the script (no retries).
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
FR=${FRAMES:-30}
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quant-variant --no-latency --ops-out "$OUT/bench_ops.json" \
    > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -n 1 "$OUT/bench.log" | cut -c1-300
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python "$ROOT/bench.py" --warmup 5 --profile-frames $FR --no-cpu-baseline --no-latency --no-quant-variant \
    --no-op-times > "$OUT/prof.log" 2>&1) || { echo "rocprof trace failed"; tail -n 20 "$OUT/prof.log"; exit 1; }
python tools/prof_ops.py piped "$OUT/prof/run_kernel_trace.csv" "$OUT/bench_ops.json" "$OUT/op_stats.csv" \
    "$OUT/piped_steps.json"
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  T=$(echo "$C" | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$T" -o run --output-format csv \
      -- python "$ROOT/bench.py" --profile-frames 6 --warmup 2 --no-cpu-baseline --no-latency --no-op-times \
      --no-quant-variant > "$OUT/pmc_$T.log" 2>&1) || { echo "pmc $C failed"; tail -n 5 "$OUT/pmc_$T.log"; exit 1; }
  for c in $C; do
    python tools/prof_ops.py counters "$OUT/pmc_$T/run_counter_collection.csv" "$OUT/bench_ops.json" $c "$OUT/pmc_$c.json"
  done
done
python tools/prof_ops.py traffic "$OUT/pmc_FETCH_SIZE.json" "$OUT/pmc_WRITE_SIZE.json" "$OUT/traffic.json"
python tools/prof_ops.py mfma "$OUT/pmc_SQ_VALU_MFMA_BUSY_CYCLES.json" "$OUT/pmc_GRBM_GUI_ACTIVE.json" \
    "$OUT/op_stats.csv" "$OUT/mfma.json"
if [ "${SERVE:-1}" = "1" ]; then
  timeout -k 10 420 python tools/serve_load.py --rounds ${ROUNDS:-5} --seconds ${SECONDS_PER_ROUND:-6} \
      --out "$OUT/serve_load.json" > "$OUT/serve_load.log" 2>&1 || { echo "serve_load failed"; tail -n 20 "$OUT/serve_load.log"; exit 1; }
  tail -n 4 "$OUT/serve_load.log"
fi
exit 0
