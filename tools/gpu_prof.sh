#!/bin/bash
# Profile-only GPU session: the pipelined bench configuration under rocprofv3 --kernel-trace --stats
# (attributed per op by tools/prof_ops.py piped), then optional extra commands (EXTRA). Every GPU step
# has its own time limit; a failure stops the script (no retries).
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
FRAMES=${FRAMES:-0}
PF=""
if [ "$FRAMES" != "0" ]; then PF="--profile-frames $FRAMES"; fi
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rfP --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -n 30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -n 2 "$OUT/pytest_gpu.log"
fi
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python "$ROOT/bench.py" --warmup 5 $PF --no-cpu-baseline --no-latency --no-quant-variant \
    --ops-out "$OUT/prof_ops.json" > "$OUT/prof.log" 2>&1)
rc=$?
echo "rocprof rc=$rc"; tail -n 1 "$OUT/prof.log" | cut -c1-400
if [ $rc -ne 0 ]; then tail -n 30 "$OUT/prof.log"; exit $rc; fi
python tools/prof_ops.py piped "$OUT/prof/run_kernel_trace.csv" "$OUT/prof_ops.json" "$OUT/op_stats.csv" \
    "$OUT/piped_steps.json"
if [ -n "${EXTRA:-}" ]; then
  bash -c "$EXTRA"
fi
exit 0
