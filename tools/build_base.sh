#!/bin/bash
# Build the library of a git revision (default HEAD) into gpubin/libbase.so (git-ignored, pushed to GPU boxes), for A/B runs:
#   bash tools/build_base.sh [rev]; then ARMS="base:PTTS_LIB=gpubin/libbase.so new:-" bash tools/ab.sh
set -eu
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
WT=$(mktemp -d /tmp/ptts_base.XXXXXX)
git worktree add -q --detach "$WT" "$REV"
make -C "$WT/pocket-tts_amd" -j8 > /dev/null 2>&1
mkdir -p gpubin
cp "$WT/pocket-tts_amd/lib/libpocket_tts_hip.so" gpubin/libbase.so
git worktree remove --force "$WT"
echo "gpubin/libbase.so <- $(git rev-parse --short "$REV")"
