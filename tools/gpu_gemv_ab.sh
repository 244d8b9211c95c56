# Product bench, same box: the previous library (pocket-tts_amd/lib-base) against the current one,
# single-frame and frame-pair back passes, two alternating rounds (tools/bf_ab.sh)
set -e
bash tools/bf_ab.sh
