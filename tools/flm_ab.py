"""A/B of the persistent FlowLM launch (k_flow_lm) against the 48-launch form (without PTTS_FLM_ON, probe
build: PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so): steady step time of pipelined and
sequential engines at B = 32 and of a sequential B = 1 engine (the first-chunk path), medians of
REPS alternating rounds."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402


def step_us(B, pipeline, off, n=60):
    if off:
        os.environ.pop("PTTS_FLM_ON", None)
    else:
        os.environ["PTTS_FLM_ON"] = "1"
    eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED, pipeline=pipeline)
    rng = np.random.default_rng(0)
    v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
    eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                  [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=120, seed=b + 1)
                   for b in range(B)])
    for _ in range(10):
        eng.step_async(B)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(n):
        eng.step_async(B)
    eng.sync()
    us = (time.perf_counter() - t0) / n * 1e6
    eng.close()
    return us


reps = int(os.environ.get("REPS", "3"))
for B, pipe in [(32, True), (32, False), (1, False)]:
    res = {False: [], True: []}
    for _ in range(reps):
        for off in (False, True):
            res[off].append(step_us(B, pipe, off))
    print(f"B={B} pipeline={pipe}: persistent {np.median(res[False]):.1f} us, 48 launches {np.median(res[True]):.1f} us",
          flush=True)
