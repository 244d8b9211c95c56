#!/bin/bash
# Quick GPU iteration: parity tests (-x), bench without the CPU baseline / variants, optional PMC
# traffic pass (PMC=1). Every GPU step has its own time limit; a failure stops the script.
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rfP --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -n 30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -n 2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quant-variant --ops-out "$OUT/bench_ops.json" \
    ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -n 20 "$OUT/bench.log"; exit 1; }
tail -n 1 "$OUT/bench.log" | cut -c1-600
if [ "${PMC:-0}" = "1" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$C" -o run --output-format csv \
        -- python "$ROOT/bench.py" --profile-frames 6 --warmup 2 --no-cpu-baseline --no-latency --no-op-times --no-pipeline \
        --no-quant-variant > "$OUT/pmc_$C.log" 2>&1) || { echo "pmc $C failed"; tail -n 5 "$OUT/pmc_$C.log"; exit 1; }
    python tools/prof_ops.py counters "$OUT/pmc_$C/run_counter_collection.csv" "$OUT/bench_ops.json" $C \
        "$OUT/pmc_$C.json"
  done
  python tools/prof_ops.py traffic "$OUT/pmc_FETCH_SIZE.json" "$OUT/pmc_WRITE_SIZE.json" "$OUT/traffic.json"
fi
exit 0
