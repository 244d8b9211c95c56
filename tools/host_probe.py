"""Host side of pipelined stepping at the bench shape (B = 32, 125 frames): wall time of the
step_async calls alone (host issue) against the same calls followed by sync (GPU), per back-pass
mode. A host issue time close to the total means the host bounds the step."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402

B, K = 32, 125
prompt = (0.11 * np.random.default_rng(0).standard_normal((125, 1024))).astype(np.float32)
for bf in (1, 2):
    eng = pt.Engine(device=0, max_slots=B, max_ctx=125 + 40 + K + 8, seed=0x5EED, pipeline=True, back_frames=bf)
    v = eng.voice_from_prompt(prompt)
    for j in range(4):
        eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                      [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=K, seed=100 * j + b + 1)
                       for b in range(B)])
        eng.sync()
        n = K + sum(eng.frame_lag())
        per = []
        t0 = time.perf_counter()
        for _ in range(n):
            a = time.perf_counter()
            eng.step_async(B)
            per.append(time.perf_counter() - a)
        t1 = time.perf_counter()
        eng.sync()
        t2 = time.perf_counter()
        per = np.array(per) * 1e6
        print(f"bf={bf} job {j}: issue {1e6 * (t1 - t0) / K:.1f} us/step (call p50 {np.median(per):.1f}, "
              f"p90 {np.percentile(per, 90):.1f}, max {per.max():.1f}), total {1e6 * (t2 - t0) / K:.1f} us/step",
              flush=True)
    eng.close()
