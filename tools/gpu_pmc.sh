#!/bin/bash
# PMC traffic passes only (FETCH_SIZE, WRITE_SIZE; separate runs), attributed per op -> gpurun_out/traffic.json
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quant-variant --no-latency --ops-out "$OUT/bench_ops.json" \
    > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$C" -o run --output-format csv \
      -- python "$ROOT/bench.py" --profile-frames 6 --warmup 2 --no-cpu-baseline --no-latency --no-op-times --no-pipeline \
      --no-quant-variant > "$OUT/pmc_$C.log" 2>&1) || { echo "pmc $C failed"; tail -n 5 "$OUT/pmc_$C.log"; exit 1; }
  python tools/prof_ops.py counters "$OUT/pmc_$C/run_counter_collection.csv" "$OUT/bench_ops.json" $C "$OUT/pmc_$C.json"
done
python tools/prof_ops.py traffic "$OUT/pmc_FETCH_SIZE.json" "$OUT/pmc_WRITE_SIZE.json" "$OUT/traffic.json"
python -c "import json; t=json.load(open('$OUT/traffic.json'))['ops']; print('head.chain', t['head.chain'])"
