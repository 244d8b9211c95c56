#!/usr/bin/env python3
"""Engine-level first-chunk probe (no HTTP): where a new stream's first frame spends its time under
the serving load of one GPU (BASELINE configs[3] share: 32 rows).

31 rows run long utterances; row 31 is re-admitted with an 8-frame utterance whenever its previous
one ended. The driver loop is the scheduler's (serve.py BatchScheduler._loop: one call in flight,
fetch of the previous call), with the first-frame preview polled while row 31 waits for its first
frame. Per admission: open_many host time, admission -> start call issued, start -> first frame
(preview or regular), and the same on an idle engine (one row). Prints one JSON line.

  python tools/first_chunk_probe.py [--back-frames 2] [--preview-rows 8] [--admissions 60]"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pocket-tts_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--back-frames", type=int, default=2)
    ap.add_argument("--preview-rows", type=int, default=8)
    ap.add_argument("--admissions", type=int, default=60)
    ap.add_argument("--poll-us", type=float, default=0.0, help="sleep between polls (0: spin)")
    ap.add_argument("--idle-only", action="store_true", help="only the one-row engine (for a kernel trace)")
    ap.add_argument("--stamps", default="", help="write every admission's host stamps (monotonic ns) here")
    ap.add_argument("--shallow", type=int, default=1, help="wait for the previous call's FlowLM step before a call")
    args = ap.parse_args()
    import pocket_tts_amd as pt

    B, SHORT = 32, 8
    rng = np.random.default_rng(5)
    prompt = (0.11 * rng.standard_normal((125, 1024))).astype(np.float32)
    ids = [(k * 97 + 13) % 4000 for k in range(40)]
    out = {"back_frames": args.back_frames, "preview_rows": args.preview_rows, "shallow": args.shallow}

    def params(n, seed):
        return pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=n, seed=seed)

    def run(rows_long):
        eng = pt.Engine(device=0, max_slots=B, max_ctx=2048, seed=0x5EED,
                        pipeline=True, back_frames=args.back_frames)
        if args.preview_rows:
            eng.enable_preview(args.preview_rows)
        v = eng.voice_from_prompt(prompt)
        if rows_long:
            eng.open_many(list(range(rows_long)), [v] * rows_long, [ids] * rows_long,
                          [params(1800, i + 1) for i in range(rows_long)])
        rows = rows_long + 1
        issued = []
        rec = []
        state = {"busy": False}
        t = {}

        def poll():
            for slot, _ in eng.fetch_previews() if args.preview_rows else []:
                if slot == rows_long and "first" not in t:
                    t["first"], t["how"] = time.monotonic_ns() * 1e-9, "preview"

        def step():
            if issued and args.shallow:
                eng.front_done(1, wait=True)  # as the scheduler: one FlowLM step queued at most
            eng.step_async(rows)
            issued.append(rows)
            if "start_k" in t and t["start_k"] == 0 and "start" not in t:
                t["start"] = time.monotonic_ns() * 1e-9
            if "start_k" in t:
                t["start_k"] -= 1
            poll()
            if len(issued) == 2:
                if "first" not in t and state["busy"]:
                    while not eng.fetch_ready(1):
                        poll()
                        if args.poll_us:
                            time.sleep(args.poll_us * 1e-6)
                r = eng.fetch(issued[0], calls_back=1)
                issued.pop(0)
                poll()
                if r.valid[rows_long] and "first" not in t:
                    t["first"], t["how"] = time.monotonic_ns() * 1e-9, "regular"
                if r.last[rows_long]:
                    state["busy"] = False

        for _ in range(8):
            step()
        n = 0
        while n < args.admissions:
            if not state["busy"]:
                if t:
                    rec.append(dict(t))
                t.clear()
                t["t0"] = time.monotonic_ns() * 1e-9
                eng.open_many([rows_long], [v], [ids], [params(SHORT, 1000 + n)])
                t["t1"] = time.monotonic_ns() * 1e-9
                t["start_k"] = eng.frame_lag()[1]
                state["busy"] = True
                n += 1
            step()
        for _ in range(20):
            step()
        rec.append(dict(t))
        eng.close()
        if args.stamps:
            with open(args.stamps + (".loaded" if rows_long else ".idle"), "w") as f:
                json.dump(rec, f)
        rec = [r for r in rec[5:] if "first" in r and "start" in r]
        ms = lambda a, b: float(np.median([1e3 * (r[b] - r[a]) for r in rec]))
        return {"admissions": len(rec), "open_many_ms": round(ms("t0", "t1"), 3),
                "admit_to_start_ms": round(ms("t1", "start"), 3), "start_to_first_ms": round(ms("start", "first"), 3),
                "admit_to_first_ms": round(ms("t0", "first"), 3),
                "preview_share": round(float(np.mean([r["how"] == "preview" for r in rec])), 3)}

    if not args.idle_only:
        out["loaded_31_rows"] = run(31)
    out["idle"] = run(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
