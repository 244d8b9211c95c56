"""Flow-head chain probe: head.chain time (HIP events, B=32, steady-state KV) per PTTS_HEAD_POLL
mode, each in a fresh process."""
import json
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
    import numpy as np

    import pocket_tts_amd as pt

    B = 32
    eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED)
    rng = np.random.default_rng(0)
    v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
    eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                  [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1)
                   for b in range(B)])
    for _ in range(20):
        eng.step_async(B)
    eng.sync()
    print(json.dumps({"poll": os.environ.get("PTTS_HEAD_POLL", "1"),
                      "chain_us": round(eng.time_kernel(B, "head.chain", 200), 2)}), flush=True)
    eng.close()
else:
    for mode in sys.argv[1:] or ["0", "1", "2", "3"]:
        env = dict(os.environ, PTTS_HEAD_POLL=mode)
        subprocess.run([sys.executable, __file__, "child"], env=env, check=True)
