"""Throughput of E engines x (32/E) rows on one GPU, stepped round-robin (each engine pipelined on
its own two streams), against one engine x 32 rows: does a second independent stepping chain fill
what the latency-bound FlowLM part leaves idle? Also prints the overlap probe of one engine."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import pocket_tts_amd as pt  # noqa: E402

K = 125
for E in [int(x) for x in (sys.argv[1:] or ["1", "2"])]:
    B = 32 // E
    engs = [pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED, pipeline=True) for _ in range(E)]
    rng = np.random.default_rng(0)
    prompt = (0.11 * rng.standard_normal((125, 1024))).astype(np.float32)
    vs = [e.voice_from_prompt(prompt) for e in engs]
    res = []
    for rnd in range(2):
        for e, v in zip(engs, vs):
            e.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                        [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=K, seed=b + 1)
                         for b in range(B)])
        for e in engs:
            e.sync()
        t0 = time.perf_counter()
        for _ in range(K + 1):
            for e in engs:
                e.step_async(B)
        for e in engs:
            e.sync()
        res.append(1e3 * (time.perf_counter() - t0) / K)
    us = (C.c_double * 8)()
    pt.lib().ptts_probe_overlap(engs[0].handle, B, 20, us)
    print(json.dumps({"engines": E, "rows_each": B, "ms_per_step": [round(x, 4) for x in res],
                      "rtf": round(32 * 0.08 / (res[-1] / 1e3), 1),
                      "probe_front_us": round(us[0], 1), "probe_back_us": round(us[1], 1),
                      "probe_both_us": round(us[2], 1)}), flush=True)
    for e in engs:
        e.close()
