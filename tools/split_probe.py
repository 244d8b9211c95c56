#!/usr/bin/env python3
"""Probe: the bench's 32 rows per GPU as ONE engine of 32 slots, or as E engines of 32 / E slots
each stepping on their own streams (their FlowLM chains overlap each other's launch gaps).

Same workload as bench.py (shared 125-frame voice, 40 text tokens, 125 frames at temp 0.7, flush
calls, one admission per job overlapping the previous job's drain); prints one JSON line per
configuration: audio-s/wall-s over `--jobs` timed jobs and the per-step time.

  python tools/split_probe.py [--engines 1 2] [--jobs 8] [--back-frames 4]"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pocket-tts_amd"))

import bench  # noqa: E402  (synth_prompt, text_ids, slot_seed, sizes)


def run(pt, E, jobs, back_frames, B):
    K = bench.UTT_FRAMES
    rows = B // E
    max_ctx = bench.PROMPT_FRAMES + bench.TEXT_TOKENS + K + 8
    engs = [pt.Engine(device=0, max_slots=rows, max_ctx=max_ctx, lsd_decode_steps=1, seed=0x5EED,
                      pipeline=True, back_frames=back_frames) for _ in range(E)]
    voices = [e.voice_from_prompt(bench.synth_prompt()) for e in engs]

    def admit(round_id, n):
        for i, e in enumerate(engs):
            e.open_many(list(range(rows)), [voices[i]] * rows, [bench.text_ids(i * rows + b) for b in range(rows)],
                        [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), frames_after_eos=3, max_frames=n,
                                             seed=bench.slot_seed(round_id, 0, i * rows + b)) for b in range(rows)])

    def calls(n):
        lag, delay = engs[0].frame_lag()
        for _ in range(n + delay):
            for e in engs:
                e.step_async(rows)
        for _ in range(lag):
            for e in engs:
                e.flush_async(rows)

    admit(0, 5)
    calls(5)
    for e in engs:
        e.sync()
    bad = []
    t0 = time.perf_counter()
    admit(1, K)
    for j in range(jobs):
        calls(K)
        if j + 1 < jobs:
            admit(2 + j, K)
        for e in engs:
            r = e.fetch(rows)
            if not (r.valid.all() and r.last.all() and np.isfinite(r.pcm).all()):
                bad.append({"job": j, "valid": int(r.valid.sum()), "last": int(r.last.sum()),
                            "finite": bool(np.isfinite(r.pcm).all())})
    el = time.perf_counter() - t0
    for e in engs:
        e.close()
    return {"engines": E, "rows_per_engine": rows, "back_frames": back_frames, "jobs": jobs,
            "audio_sec_per_wall_sec": round(B * 10.0 * jobs / el, 1), "ms_per_step": round(1e3 * el / (jobs * K), 4),
            "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", ""), "bad": bad[:4]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--back-frames", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=bench.BATCH)
    args = ap.parse_args()
    import pocket_tts_amd as pt

    for _ in range(args.reps):
        for E in args.engines:
            print(json.dumps(run(pt, E, args.jobs, args.back_frames, args.batch)), flush=True)


if __name__ == "__main__":
    main()
