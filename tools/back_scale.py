"""How the back part (Mimi decode) scales with its row count: every back-part op timed alone
(HIP events) at B and 2B utterance rows, and the back graph alone / with the front on two streams
(overlap probe, back capped as in pipelined stepping). Two frames of one utterance in one back
launch have the GEMM / conv shapes of 2B rows, so the 2B sum is the cost of a frame pair."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402
from pocket_tts_amd._lib import check, lib  # noqa: E402

for B in [int(x) for x in os.environ.get("BS", "32,64").split(",")]:
    eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED, pipeline=True)
    rng = np.random.default_rng(0)
    v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
    eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                  [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=120, seed=b + 1)
                   for b in range(B)])
    for _ in range(40):
        eng.step_async(B)
    eng.sync()
    back, front = 0.0, 0.0
    rows = []
    for n in dict.fromkeys(eng.plan_ops(B)):
        us = eng.time_kernel(B, n, 20)
        print(".", end="", flush=True)
        if n.startswith(("mimi.", "seanet.")) or n == "commit":
            back += us * eng.plan_ops(B).count(n)
            rows.append((n, us))
        else:
            front += us * eng.plan_ops(B).count(n)
    print(f"B={B}: back ops sum {back:.1f} us, front ops sum {front:.1f} us", flush=True)
    print("  " + ", ".join(f"{n} {u:.1f}" for n, u in rows), flush=True)
    if os.environ.get("OVERLAP"):
        us = (C.c_double * 8)()
        check(lib().ptts_probe_overlap(eng.handle, B, 20, us))
        print(f"  overlap probe: front {us[0]:.1f} us, back (capped) {us[1]:.1f} us, both {us[2]:.1f} us", flush=True)
    eng.close()
