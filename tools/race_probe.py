#!/usr/bin/env python3
"""Stress probe of the bench's job loop (bench.py timed_job, same call sequence and timing): JOBS
jobs of B rows x 125 frames, the next job's admission issued before the drain's fetch, and the
last frame of every job checked (valid and last flags, finite PCM). Prints one JSON line: jobs
run, and per failing job the rows without a valid / last flag.

  [PTTS_LIB=...] python tools/race_probe.py [--jobs 40] [--back-frames 4]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pocket-tts_amd"))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=40)
    ap.add_argument("--back-frames", type=int, default=4)
    args = ap.parse_args()
    import pocket_tts_amd as pt

    B, K = bench.BATCH, bench.UTT_FRAMES
    eng = pt.Engine(device=0, max_slots=B, max_ctx=bench.PROMPT_FRAMES + bench.TEXT_TOKENS + K + 8,
                    lsd_decode_steps=1, seed=0x5EED, pipeline=True, back_frames=args.back_frames)
    v = eng.voice_from_prompt(bench.synth_prompt())

    def admit(j):
        eng.open_many(list(range(B)), [v] * B, [bench.text_ids(b) for b in range(B)],
                      [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), frames_after_eos=3, max_frames=K,
                                           seed=bench.slot_seed(j, 0, b)) for b in range(B)])

    fails = []
    admit(0)
    lag, delay = eng.frame_lag()
    j = 0
    for j in range(args.jobs):  # exactly bench.py's run_calls + overlapped admission + one fetch
        for _ in range(K + delay):
            eng.step_async(B)
        for _ in range(lag):
            eng.flush_async(B)
        if j + 1 < args.jobs:
            admit(j + 1)
        r = eng.fetch(B)
        if not (r.valid.all() and r.last.all() and np.isfinite(r.pcm).all()):
            fails.append({"job": j, "invalid_rows": np.nonzero(~r.valid)[0].tolist()[:8],
                          "not_last_rows": np.nonzero(~r.last)[0].tolist()[:8],
                          "finite": bool(np.isfinite(r.pcm).all())})
            if len(fails) > 4:
                break
    eng.close()
    print(json.dumps({"lib": os.environ.get("PTTS_LIB", "product"), "jobs": j + 1, "fails": fails}), flush=True)


if __name__ == "__main__":
    main()
