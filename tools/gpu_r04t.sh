#!/bin/bash
# Round 4 (combined session): tools/gpu_r04s.sh (fused FFN parity + A/B + back priority + per-op
# stamps), then tools/gpu_r04q.sh (overlap probe with the front skip probes).
set -u
cd "$(dirname "$0")/.."
bash tools/gpu_r04s.sh || exit 1
bash tools/gpu_r04q.sh
