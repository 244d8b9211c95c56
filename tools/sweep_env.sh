#!/bin/bash
# Bench sweep over one environment knob, interleaved repeats (noise is ~1-2% run to run):
#   VAR=name VALUES="a b c" [REPS=3] bash tools/sweep_env.sh
# Value "-" leaves VAR unset. One line per run, then the median steady ms per value.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
REPS=${REPS:-1}
for r in $(seq 1 "$REPS"); do
  for v in $VALUES; do
    t=$(echo "$v" | tr '/' '_' | cut -c1-60)$(echo "$v" | md5sum | cut -c1-6)
    if [ "$v" = "-" ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-op-times --no-latency \
          ${BENCH_ARGS:-} > gpurun_out/sweep_$t.log 2>&1 || { echo "$VAR unset failed"; tail -5 gpurun_out/sweep_$t.log; exit 1; }
    else
      env "$VAR=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-op-times --no-latency \
          ${BENCH_ARGS:-} > gpurun_out/sweep_$t.log 2>&1 || { echo "$VAR=$v failed"; tail -5 gpurun_out/sweep_$t.log; exit 1; }
    fi
    python - "$VAR=$v" gpurun_out/sweep_$t.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
import os
key = os.environ.get("METRIC", "steady_ms_per_step")
print(sys.argv[1][:60], "value", d["value"], "steady_ms", d["steady_ms_per_step"], "admit_ms", d["admit_ms"], flush=True)
with open("gpurun_out/sweep_all.txt", "a") as f:
    f.write(f"{sys.argv[1]} {d[key]}\n")
PY
  done
done
python - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for line in open("gpurun_out/sweep_all.txt"):
    k, v = line.split()
    d[k].append(float(v))
for k, v in d.items():
    print(f"median {k[:70]}: {statistics.median(v):.4f} over {len(v)}")
PY
rm -f gpurun_out/sweep_all.txt
