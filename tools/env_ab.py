"""Steady pipelined step time of the bench job (B = 32, 125 frames + lag calls) under probe-build
environment settings: VAR=PTTS_... VALUES="v1 v2 ..." ('-' = unset), medians of REPS alternating
rounds (PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so); BF=2: frame-pair back passes."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402

B, K = 32, 125
prompt = (0.11 * np.random.default_rng(0).standard_normal((125, 1024))).astype(np.float32)


def run(jobs=4):
    eng = pt.Engine(device=0, max_slots=B, max_ctx=125 + 40 + K + 8, seed=0x5EED, pipeline=True,
                    back_frames=int(os.environ.get("BF", "1")))
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


var, values = os.environ["VAR"], os.environ["VALUES"].split()
res = {v: [] for v in values}
for _ in range(int(os.environ.get("REPS", "2"))):
    for v in values:
        if v == "-":
            os.environ.pop(var, None)
        else:
            os.environ[var] = v
        res[v].append(run())
        print(f"{var}={v}: {res[v][-1]:.1f} us/step", flush=True)
for v in values:
    print(f"MEDIAN {var}={v}: {np.median(res[v]):.1f} us/step", flush=True)
