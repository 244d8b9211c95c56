#!/bin/bash
# Round 4: flush calls (ptts_flush_async) - the parity tests that drive them, then the product
# bench with the job drain as flush calls against step calls (--no-flush), interleaved.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "flush or varying or frame_pairs or pipelined" \
  --timeout 200 --timeout-method thread > $OUT/pytest_flush.log 2>&1 || { tail -n 40 $OUT/pytest_flush.log; exit 1; }
tail -n 1 $OUT/pytest_flush.log
for r in 1 2 3; do
  for f in flush step; do
    a=""; [ $f = step ] && a="--no-flush"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-latency --no-op-times $a > $OUT/ab.log 2>&1 \
      || { tail -5 $OUT/ab.log; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/ab.log').read().strip().splitlines()[-1]); print('$f round $r', d['value'], d['ms_per_step'], d['steady_ms_per_step'], d['admit_ms'])"
  done
done
