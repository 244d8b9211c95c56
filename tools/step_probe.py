"""Host issue cost vs GPU time of the stepping loop (B rows, K steps): pipelined and sequential."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import pocket_tts_amd as pt  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
K = 125
q = int(os.environ.get("WQ", "0"))
import ctypes as C  # noqa: E402

# engine environment variants to compare, e.g. VARIANTS = [dict(), dict(PTTS_W8_OFF="1")]
VARIANTS = [dict()]
if os.environ.get("SEQ"):
    VARIANTS = [dict()]
for var in VARIANTS:
    pipeline, prio = not os.environ.get("SEQ"), var
    os.environ.update(var)
    eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED, pipeline=pipeline, weight_quant=q)
    rng = np.random.default_rng(0)
    v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
    for rnd in range(2):
        eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                      [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=K, seed=b + 1)
                       for b in range(B)])
        eng.sync()
        t0 = time.perf_counter()
        issue = []
        for _ in range(K + 1):
            a = time.perf_counter()
            eng.step_async(B)
            issue.append(time.perf_counter() - a)
        t1 = time.perf_counter()
        eng.sync()
        t2 = time.perf_counter()
        print(json.dumps({"pipeline": pipeline, "prio": prio, "round": rnd, "issue_ms_total": round(1e3 * (t1 - t0), 2),
                          "issue_us_median": round(1e6 * float(np.median(issue)), 1),
                          "issue_us_max": round(1e6 * max(issue), 1),
                          "wall_ms": round(1e3 * (t2 - t0), 2), "ms_per_step": round(1e3 * (t2 - t0) / K, 4)}))
    us = (C.c_double * 8)()
    pt.lib().ptts_probe_overlap(eng.handle, B, 20, us)
    print(json.dumps({"probe_front": round(us[0], 1), "probe_back": round(us[1], 1), "probe_both": round(us[2], 1),
                      "probe_both_prio": round(us[3], 1)}))
    eng.close()
