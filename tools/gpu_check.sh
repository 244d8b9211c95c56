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

timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest-gpu rc=$rc"; tail -n 30 "$OUT/pytest_gpu.log"
if fatal $rc; then exit $rc; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
echo "smoke rc=$rc"; tail -n 5 "$OUT/smoke.log"
if [ $rc -ne 0 ]; then exit $rc; fi

timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -n 3 "$OUT/bench.log"
if [ $rc -ne 0 ]; then exit $rc; fi

if [ "${PROFILE:-1}" = "1" ]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
      -- python "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu-baseline --no-latency > "$OUT/prof.log" 2>&1)
  rc=$?
  echo "rocprof rc=$rc"; tail -n 3 "$OUT/prof.log"
fi
exit 0
