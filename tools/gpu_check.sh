#!/bin/bash
# One GPU-box session: parity tests, smoke, default bench, rocprof kernel-trace of a short bench.
# Every GPU step has its own time limit; a crash/timeout/abort stops the script (no retries).
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() { # exit codes that mean the GPU or process died: stop everything
  case $1 in 124|134|137|139) return 0 ;; *) return 1 ;; esac
}

timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rfP --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest-gpu rc=$rc"; tail -n 30 "$OUT/pytest_gpu.log"
if fatal $rc; then exit $rc; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
echo "smoke rc=$rc"; tail -n 5 "$OUT/smoke.log"
if [ $rc -ne 0 ]; then exit $rc; fi

timeout -k 10 600 python bench.py --ops-out "$OUT/bench_ops.json" > "$OUT/bench.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -n 3 "$OUT/bench.log"
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SEQ:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --no-pipeline --no-cpu-baseline --no-latency --no-op-times \
      > "$OUT/bench_seq.log" 2>&1
  rc=$?
  echo "bench sequential rc=$rc"; tail -n 1 "$OUT/bench_seq.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
fi

if [ "${PROFILE:-1}" = "1" ]; then
  # the MEASURED configuration: pipelined engine, full 125-frame jobs (front / back graphs on two
  # streams; tools/prof_ops.py piped attributes each hardware queue to its part of the plan)
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
      -- python "$ROOT/bench.py" --warmup 5 --no-cpu-baseline --no-latency --no-quant-variant \
      --ops-out "$OUT/prof_ops.json" > "$OUT/prof.log" 2>&1)
  rc=$?
  echo "rocprof rc=$rc"; tail -n 2 "$OUT/prof.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  python tools/prof_ops.py piped "$OUT/prof/run_kernel_trace.csv" "$OUT/prof_ops.json" "$OUT/op_stats.csv" \
      "$OUT/piped_steps.json"
fi

if [ "${PMC:-0}" = "1" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$C" -o run --output-format csv \
        -- python "$ROOT/bench.py" --profile-frames 6 --warmup 2 --no-cpu-baseline --no-latency --no-op-times --no-quant-variant \
        > "$OUT/pmc_$C.log" 2>&1)
    rc=$?
    echo "pmc $C rc=$rc"; tail -n 2 "$OUT/pmc_$C.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
    python tools/prof_ops.py counters "$OUT/pmc_$C/run_counter_collection.csv" "$OUT/bench_ops.json" $C \
        "$OUT/pmc_$C.json"
  done
  python tools/prof_ops.py traffic "$OUT/pmc_FETCH_SIZE.json" "$OUT/pmc_WRITE_SIZE.json" "$OUT/traffic.json"
  # MFMA utilisation: one pass with both counters (1 SQ_ + 1 GRBM_ counter: within one pass's limits)
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmc_mfma" \
      -o run --output-format csv \
      -- python "$ROOT/bench.py" --profile-frames 6 --warmup 2 --no-cpu-baseline --no-latency --no-op-times --no-quant-variant \
      > "$OUT/pmc_mfma.log" 2>&1)
  rc=$?
  echo "pmc mfma rc=$rc"; tail -n 2 "$OUT/pmc_mfma.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
  for C in SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; do
    python tools/prof_ops.py counters "$OUT/pmc_mfma/run_counter_collection.csv" "$OUT/bench_ops.json" $C "$OUT/pmc_$C.json"
  done
  python tools/prof_ops.py mfma "$OUT/pmc_SQ_VALU_MFMA_BUSY_CYCLES.json" "$OUT/pmc_GRBM_GUI_ACTIVE.json" \
      "$OUT/op_stats.csv" "$OUT/mfma.json"
fi
exit 0
