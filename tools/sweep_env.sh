#!/bin/bash
# Bench sweep over one environment knob: VAR=name VALUES="a b c" bash tools/sweep_env.sh
# (bench without the CPU baseline, variants, per-op timings or latency; one line per value)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in $VALUES; do
  env "$VAR=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-op-times --no-latency \
      ${BENCH_ARGS:-} > gpurun_out/sweep_$v.log 2>&1 || { echo "$VAR=$v failed"; tail -5 gpurun_out/sweep_$v.log; exit 1; }
  python - "$VAR=$v" gpurun_out/sweep_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", d["value"], "steady_ms", d["steady_ms_per_step"], flush=True)
PY
done
