"""configs[1] first-chunk path (B = 1: text prefill + one sequential step, voice precomputed),
repeated, for a rocprofv3 --kernel-trace --stats breakdown and wall times."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import pocket_tts_amd as pt  # noqa: E402

e1 = pt.Engine(device=0, max_slots=1, max_ctx=bench.PROMPT_FRAMES + bench.TEXT_TOKENS + 16, seed=0x5EED)
v1 = e1.voice_from_prompt(bench.synth_prompt())
lat, adm = [], []
for i in range(30):
    t = time.perf_counter()
    e1.open(0, v1, bench.text_ids(0), pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=4,
                                                          seed=i + 1))
    e1.sync()
    t1 = time.perf_counter()
    e1.step(1)
    lat.append(time.perf_counter() - t)
    adm.append(t1 - t)
print(f"p50 first chunk {1000 * np.median(lat[5:]):.3f} ms, of which admission {1000 * np.median(adm[5:]):.3f} ms")
e1.close()
