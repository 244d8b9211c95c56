"""Admission only (the bench's batched open_many of 32 utterances, 40 text tokens each), repeated,
for a rocprofv3 --kernel-trace --stats breakdown of the admission path."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import pocket_tts_amd as pt  # noqa: E402

B = 32
eng = pt.Engine(device=0, max_slots=B, max_ctx=320, lsd_decode_steps=1, seed=0x5EED, pipeline=True)
voice = eng.voice_from_prompt(bench.synth_prompt())
params = [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=125, seed=b + 1) for b in range(B)]
ids = [bench.text_ids(b) for b in range(B)]
for i in range(6):
    t0 = time.perf_counter()
    eng.open_many(list(range(B)), [voice] * B, ids, params)
    eng.sync()
    print(f"admission {i}: {1000 * (time.perf_counter() - t0):.3f} ms", flush=True)
