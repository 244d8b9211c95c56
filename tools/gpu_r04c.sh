#!/bin/bash
# Round 4: GEMM-core and bf16-back tests, then the bench with its variants (int8, fp8, bf16 back).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_core.py tests/test_gpu_bf16.py -x -v -s --timeout 200 \
  --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -n 40 $OUT/pytest_new.log; exit 1; }
grep -E "worst|SNR|passed|failed" $OUT/pytest_new.log | tail -20
timeout -k 10 400 python bench.py --no-cpu-baseline --no-latency --no-op-times > $OUT/bench_var.log 2>&1 \
  || { tail -n 20 $OUT/bench_var.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_var.log").read().strip().splitlines()[-1])
print("f32", d["value"], d["steady_ms_per_step"])
for k in ("int8_flowlm_variant", "fp8_flowlm_variant", "bf16_back_variant"):
    v = d[k]; print(k, v["value"], v["steady_ms_per_step"], v.get("pcm_snr_db_vs_f32"))
PY
