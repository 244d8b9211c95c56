# A/B with the product library against a base library (pocket-tts_amd/lib-base, e.g. the previous
# commit): one frame vs frame pairs per back pass, bench.py, alternating rounds
set -e
for r in 1 2; do
  for lib in base new; do
    for bf in 1 2; do
      if [ $lib = base ]; then export PTTS_LIB=pocket-tts_amd/lib-base/libpocket_tts_hip.so; else unset PTTS_LIB; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-latency --no-op-times --back-frames $bf > gpurun_out/ab.log 2>&1
      python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$lib bf=$bf round $r', d['value'], d['steady_ms_per_step'], d['per_job']['median'])" | tee -a gpurun_out/ab_summary.txt
    done
  done
done
