#!/bin/bash
# Build the library of a git revision (default HEAD) into abl/libbase.so, for A/B sweeps:
#   bash tools/build_base.sh [rev]; then VAR=PTTS_LIB VALUES="/root/repo/abl/libbase.so -" bash tools/sweep_env.sh
set -eu
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
WT=$(mktemp -d /tmp/ptts_base.XXXXXX)
git worktree add -q --detach "$WT" "$REV"
make -C "$WT/pocket-tts_amd" -j8 > /dev/null 2>&1
mkdir -p abl
cp "$WT/pocket-tts_amd/lib/libpocket_tts_hip.so" abl/libbase.so
git worktree remove --force "$WT"
echo "abl/libbase.so <- $(git rev-parse --short "$REV")"
