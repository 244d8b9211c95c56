#!/bin/bash
# Round 4: admission ahead of the back-tail wait - the admission / pipelining parity tests, then the
# bench with the next job's admission overlapping the drain against admission after the fetch.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streaming.py tests/test_gpu_edges.py -x -v \
  --timeout 200 --timeout-method thread > $OUT/pytest_admit.log 2>&1 || { tail -n 40 $OUT/pytest_admit.log; exit 1; }
tail -n 1 $OUT/pytest_admit.log
for r in 1 2 3; do
  for f in overlap serial; do
    a=""; [ $f = serial ] && a="--no-overlap-admission"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-quant-variant --no-latency --no-op-times $a > $OUT/ab.log 2>&1 \
      || { tail -5 $OUT/ab.log; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/ab.log').read().strip().splitlines()[-1]); print('$f round $r', d['value'], d['ms_per_step'], d['steady_ms_per_step'], d['admit_ms'], d['per_job'])"
  done
done
