#!/bin/bash
# A/B runner: the bench's steady step under several arms, interleaved repeats on ONE box (run-to-run
# noise is 1-2 %, box-to-box more, so only same-box interleaved medians are compared).
#
#   ARMS="label:K=V,K=V label2:- ..." [REPS=3] [BENCH_ARGS="..."] [METRIC=steady_ms_per_step] \
#       [PRE="command run once before the arms, e.g. a pytest subset"] bash tools/ab.sh [summary.txt]
#
# An arm is a label and a comma-separated list of environment settings ("-" = none); the pseudo
# setting BENCH=a+b+c appends the bench.py arguments "a b c" for that arm only. The usual ones:
#   PTTS_LIB=gpubin/libbase.so                               a base library (tools/build_base.sh REV)
#   PTTS_LIB=gpubin/libNAME.so                               a patch variant (tools/build_variant.sh NAME PATCH)
#   PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so  the measurement build (make -C pocket-tts_amd probes)
#   PTTS_BACK_PRIO / PTTS_FRONT_PRIO / PTTS_BACK_WG_CAP / PTTS_OVR=op=layout:splits ...  probe knobs
# Every bench run is under its own time limit; a failing run ends the script (no retries).
# One line per run, then the median of METRIC per arm, appended to the summary file
# (default gpurun_out/ab_summary.txt).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=${1:-gpurun_out/ab_summary.txt}
REPS=${REPS:-3}
METRIC=${METRIC:-steady_ms_per_step}
RAW=$(mktemp /tmp/ab_raw.XXXXXX)
if [ -n "${PRE:-}" ]; then
  bash -c "$PRE" > gpurun_out/ab_pre.log 2>&1 || { echo "PRE failed"; tail -20 gpurun_out/ab_pre.log; exit 1; }
  tail -3 gpurun_out/ab_pre.log
fi
for r in $(seq 1 "$REPS"); do
  for arm in $ARMS; do
    label=${arm%%:*}
    envs=${arm#*:}
    settings=()
    extra=""
    if [ "$envs" != "-" ]; then IFS=',' read -ra all <<< "$envs"; fi
    for kv in "${all[@]:-}"; do
      [ -z "$kv" ] && continue
      if [ "${kv%%=*}" = "BENCH" ]; then extra="${kv#BENCH=}"; extra="${extra//+/ }"; else settings+=("$kv"); fi
    done
    all=()
    log=gpurun_out/ab_${label}_$r.log
    env "${settings[@]}" timeout -k 10 240 python bench.py --no-cpu-baseline --no-quant-variant --no-op-times \
        --no-latency --no-distinct-voices --no-voice-bench --no-text-bench ${BENCH_ARGS:-} $extra > "$log" 2>&1 \
      || { echo "arm $label failed (round $r)"; tail -5 "$log"; exit 1; }
    python - "$label" "$r" "$log" "$METRIC" "$RAW" <<'PY'
import json, sys
label, r, log, key, raw = sys.argv[1:]
d = json.loads(open(log).read().strip().splitlines()[-1])
print(f"{label} round {r}: value {d['value']} steady_ms {d['steady_ms_per_step']} {key} {d[key]}", flush=True)
open(raw, "a").write(f"{label} {d[key]}\n")
PY
  done
done
python - "$RAW" "$OUT" "$METRIC" "$ARMS" <<'PY'
import collections, statistics, sys
raw, out, key, arms = sys.argv[1:]
d = collections.defaultdict(list)
for line in open(raw):
    k, v = line.split()
    d[k].append(float(v))
with open(out, "a") as f:
    f.write(f"# ARMS={arms}\n")
    for k, v in d.items():
        line = f"median {key} {k}: {statistics.median(v):.4f} over {len(v)} ({' '.join(f'{x:.4f}' for x in v)})"
        print(line)
        f.write(line + "\n")
PY
rm -f "$RAW"
