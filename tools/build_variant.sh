#!/bin/bash
# Build an A/B variant library: a git revision (default HEAD) with a patch applied, into
# gpubin/lib<NAME>.so (git-ignored, pushed to GPU boxes). The patch is the variant: product sources
# carry no compile-time A/B switches.
#   bash tools/build_variant.sh NAME PATCH [REV] [EXTRA_FLAGS]
#   ARMS="prod:- v:PTTS_LIB=gpubin/libv.so" bash tools/ab.sh
# A variant's build id differs from the product's, so its bench lines say "NOT A PRODUCT RUN".
set -eu
cd "$(dirname "$0")/.."
NAME=$1
PATCH=$(realpath "$2")
REV=${3:-HEAD}
WT=$(mktemp -d /tmp/ptts_var.XXXXXX)
git worktree add -q --detach "$WT" "$REV"
trap 'git worktree remove --force "$WT"' EXIT
git -C "$WT" apply "$PATCH"
make -C "$WT/pocket-tts_amd" -j8 ${4:+EXTRA_FLAGS="$4"} > "/tmp/variant_$NAME.log" 2>&1 \
  || { tail -20 "/tmp/variant_$NAME.log"; exit 1; }
mkdir -p gpubin
cp "$WT/pocket-tts_amd/lib/libpocket_tts_hip.so" "gpubin/lib$NAME.so"
echo "gpubin/lib$NAME.so <- $(git rev-parse --short "$REV") + $(basename "$PATCH")"
