#!/bin/bash
# GPU session: parity tests (-x; TESTS=0 skips), head-chain stamps, then tools/sweep_combo.sh over $COMBOS.
set -u
cd "$(dirname "$0")/.."
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rfP --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -n 30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -n 2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 200 python tools/head_stamps.py > "$OUT/head_stamps.log" 2>&1 || { echo "stamps failed"; tail -20 "$OUT/head_stamps.log"; exit 1; }
grep -v amdgpu.ids "$OUT/head_stamps.log"
[ -n "${COMBOS:-}" ] && bash tools/sweep_combo.sh
exit 0
