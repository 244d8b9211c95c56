"""Steady pipelined step time of the bench job (B = 32, 125 frames, K + lag calls, no fetch in
between) for frame-pair passes (back_frames 2) against one frame per pass, under back-part
per-CU caps (PTTS_BACK_WG_CAP, probe build: PTTS_LIB=pocket-tts_amd/lib-probes/...). Medians of
REPS alternating rounds; CONFIGS="bf:cap,..." (cap '-' = the engine default)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402

B, K = 32, 125
rng = np.random.default_rng(0)
prompt = (0.11 * rng.standard_normal((125, 1024))).astype(np.float32)


def run(bf, cap, jobs=4):
    if cap == "-":
        os.environ.pop("PTTS_BACK_WG_CAP", None)
    else:
        os.environ["PTTS_BACK_WG_CAP"] = cap
    eng = pt.Engine(device=0, max_slots=B, max_ctx=125 + 40 + K + 8, seed=0x5EED, pipeline=True, back_frames=bf)
    v = eng.voice_from_prompt(prompt)
    ts = []
    for j in range(jobs + 1):
        eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                      [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=K, seed=100 * j + b + 1)
                       for b in range(B)])
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(K + sum(eng.frame_lag())):
            eng.step_async(B)
        eng.sync()
        if j:
            ts.append((time.perf_counter() - t0) / K * 1e6)
    eng.close()
    return float(np.median(ts))


configs = [c.split(":") for c in os.environ.get("CONFIGS", "1:-,2:-,2:2,2:0").split(",")]
res = {tuple(c): [] for c in configs}
for _ in range(int(os.environ.get("REPS", "2"))):
    for c in configs:
        res[tuple(c)].append(run(int(c[0]), c[1]))
        print(f"back_frames={c[0]} cap={c[1]}: {res[tuple(c)][-1]:.1f} us/step", flush=True)
for c in configs:
    print(f"MEDIAN back_frames={c[0]} cap={c[1]}: {np.median(res[tuple(c)]):.1f} us/step", flush=True)
