#!/bin/bash
# Round 4: what the boundary between two front graphs costs (17-us gaps in the graph stamps):
# probe build, graph stamps with the front's wait on the back event dropped (PTTS_NO_FRONT_WAIT,
# unsafe in general, A/B only) and / or the timeout-word copy node dropped (PTTS_NO_ERR_COPY).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
for r in 1 2; do
for v in none wait copy both; do
  unset PTTS_NO_FRONT_WAIT PTTS_NO_ERR_COPY
  case $v in wait) export PTTS_NO_FRONT_WAIT=1;; copy) export PTTS_NO_ERR_COPY=1;; both) export PTTS_NO_FRONT_WAIT=1 PTTS_NO_ERR_COPY=1;; esac
  PTTS_STAMPS=$OUT/stb_$v.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant \
    --no-latency --no-op-times > $OUT/stb_$v.log 2>&1 || { tail -5 $OUT/stb_$v.log; exit 1; }
  python - $v $OUT/stb_$v.log $OUT/stb_$v.txt <<'PY'
import json, subprocess, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = json.loads(subprocess.run([sys.executable, "tools/stamps.py", sys.argv[3]], capture_output=True, text=True).stdout)
print(f"{sys.argv[1]:5s} steady_ms {d['steady_ms_per_step']} front_dur {s['front']['dur_us_median']:.1f} "
      f"front_gap {s['front']['gap_us_median']:.1f} back_dur {s['back']['dur_us_median']:.1f} "
      f"back_gap {s['back']['gap_us_median']:.1f}", flush=True)
PY
done
done
