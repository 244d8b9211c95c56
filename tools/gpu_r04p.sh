#!/bin/bash
# Round 4: which of the front part's resources slow the concurrent back part (the bound of the
# frame-pair step)? Probe build, graph stamps (tools/stamps.py) per PTTS_FRONT_SKIP variant
# (results wrong): 1 = the skinny GEMMs' weight loads skipped, 2 = their MFMAs, 4 = the step
# attention's cached K / V loads, 7 = all three.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
for r in 1 2; do
for v in 0 1 2 4 7; do
  PTTS_FRONT_SKIP=$v PTTS_STAMPS=$OUT/st_fs$v.txt timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant \
    --no-latency --no-op-times > $OUT/st_fs$v.log 2>&1 || { tail -5 $OUT/st_fs$v.log; exit 1; }
  python - $v $OUT/st_fs$v.log $OUT/st_fs$v.txt <<'PY'
import json, subprocess, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = json.loads(subprocess.run([sys.executable, "tools/stamps.py", sys.argv[3]], capture_output=True, text=True).stdout)
print(f"FRONT_SKIP={sys.argv[1]} steady_ms {d['steady_ms_per_step']} front_dur {s['front']['dur_us_median']:.1f} "
      f"front_gap {s['front']['gap_us_median']:.1f} back_dur {s['back']['dur_us_median']:.1f} "
      f"back_gap {s['back']['gap_us_median']:.1f}", flush=True)
PY
done
done
