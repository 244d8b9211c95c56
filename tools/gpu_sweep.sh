#!/bin/bash
# A/B only: interleaved bench runs of abl/libbase.so and the in-tree library (REPS, default 5).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
VAR=PTTS_LIB VALUES="$(pwd)/abl/libbase.so -" REPS=${REPS:-5} bash tools/sweep_env.sh
