"""Decode-attention phase probe: time flow.l0.attention under PTTS_ATTN_DBG modes in fresh
processes (0 full, 1 no QKV slab sum, 3 no score/PV loop: KV loads of the first block only)."""
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
    for _ in range(60):
        eng.step_async(B)
    eng.sync()
    print(json.dumps({"dbg": os.environ.get("PTTS_ATTN_DBG", "0"),
                      "attn_us": round(eng.time_kernel(B, "flow.l0.attention", 50), 2),
                      "qkv_us": round(eng.time_kernel(B, "flow.l0.qkv_gemm", 50), 2)}))
    eng.close()
else:
    for mode in ("0", "1", "3"):
        env = dict(os.environ, PTTS_ATTN_DBG=mode)
        subprocess.run([sys.executable, __file__, "child"], env=env, check=True)
