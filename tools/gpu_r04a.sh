#!/bin/bash
# Round-4 first session: GPU tests at the shared-LDS k_gemv build, same-box A/B against the HEAD
# library (lib-base) in both back-pass modes, then a kernel trace of the frame-pair bench for the
# per-launch start-delay table (tools/launch_delay.py). First failure ends the script.
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -n 30 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
bash tools/bf_ab.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quant-variant --no-latency --ops-out "$OUT/bench_ops.json" \
    > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python "$ROOT/bench.py" --warmup 5 --profile-frames 30 --no-cpu-baseline --no-latency --no-quant-variant \
    --no-op-times > "$OUT/prof.log" 2>&1) || { echo "rocprof trace failed"; tail -n 20 "$OUT/prof.log"; exit 1; }
exit 0
