#!/bin/bash
# GPU session: parity tests (-x), head-chain phase stamps, quick bench. Each step time-limited.
set -u
cd "$(dirname "$0")/.."
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rfP --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -n 30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -n 2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 200 python tools/head_stamps.py > "$OUT/head_stamps.log" 2>&1 || { echo "stamps failed"; tail -20 "$OUT/head_stamps.log"; exit 1; }
grep -v amdgpu.ids "$OUT/head_stamps.log"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quant-variant --ops-out "$OUT/bench_ops.json" \
    ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -n 20 "$OUT/bench.log"; exit 1; }
tail -n 1 "$OUT/bench.log" | cut -c1-700
