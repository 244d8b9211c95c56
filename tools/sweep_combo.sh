#!/bin/bash
# Bench sweep over environment combinations, interleaved repeats:
#   COMBOS="A=1+B=0 A=0+B=1 -" [REPS=3] bash tools/sweep_combo.sh   ("-" = nothing set)
# One line per run, then the median steady ms per combination. Also records head.chain (isolated).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/combo_all.txt
for r in $(seq 1 "${REPS:-3}"); do
  for c in $COMBOS; do
    envs=()
    [ "$c" != "-" ] && IFS='+' read -ra envs <<< "$c"
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-latency \
        ${BENCH_ARGS:-} > gpurun_out/combo.log 2>&1 || { echo "$c failed"; tail -2 gpurun_out/combo.log; continue; }
    python - "$c" gpurun_out/combo.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
chain = next((o["avg_us"] for o in d.get("top_ops", []) if o["op"] == "head.chain"), None)
print(sys.argv[1], "steady_ms", d["steady_ms_per_step"], "value", d["value"], "chain_us", chain, flush=True)
with open("gpurun_out/combo_all.txt", "a") as f:
    f.write(f"{sys.argv[1]} {d['steady_ms_per_step']} {chain}\n")
PY
  done
done
python - <<'PY'
import collections, statistics
d = collections.defaultdict(list); ch = collections.defaultdict(list)
for line in open("gpurun_out/combo_all.txt"):
    k, v, c = line.split()
    d[k].append(float(v)); ch[k].append(float(c))
for k in d:
    print(f"median {k}: steady {statistics.median(d[k]):.4f} ms, head.chain {statistics.median(ch[k]):.1f} us over {len(d[k])}")
PY
