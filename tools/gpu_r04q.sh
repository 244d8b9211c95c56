#!/bin/bash
# Round 4: the front part's skeleton - tools/overlap_probe.py (front graph alone, back graph alone,
# both on two streams; single-frame plan) with and without the front's GEMM weights / MFMAs /
# cached K-V loads (PTTS_FRONT_SKIP=7, probe build, results wrong).
set -u
cd "$(dirname "$0")/.."
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so PTTS_PROBE_MODES=012
for v in 0 7 1 2; do
  echo "FRONT_SKIP=$v"
  PTTS_FRONT_SKIP=$v timeout -k 10 120 python tools/overlap_probe.py 2>&1 | grep -E "^front|wall" || exit 1
done
