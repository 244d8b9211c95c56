"""Time the FlowLM+flow-head part and the Mimi part of a B=32 step alone and concurrently."""
import ctypes as C
import faulthandler
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import pocket_tts_amd as pt  # noqa: E402
from pocket_tts_amd._lib import check, lib  # noqa: E402

faulthandler.dump_traceback_later(60, repeat=True)  # a stall shows where it sits
B = int(os.environ.get("ROWS", "32"))  # rows of the step
print("engine", flush=True)
eng = pt.Engine(device=0, max_slots=B, max_ctx=400, lsd_decode_steps=1, seed=0x5EED)
voice = eng.voice_from_prompt(bench.synth_prompt())
eng.open_many(list(range(B)), [voice] * B, [bench.text_ids(b) for b in range(B)],
              [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1)
               for b in range(B)])
for _ in range(5):
    eng.step(B)
print("stepped", flush=True)
import os
import time
us = (C.c_double * 8)()
t0 = time.perf_counter()
check(lib().ptts_probe_overlap(eng.handle, B, int(os.environ.get("REPS", "50")), us))
print(f"probe wall {time.perf_counter() - t0:.2f} s", flush=True)
eng.step(B)  # surfaces a flow-head hand-off timeout of the probe's launches as an engine error
print(f"front {us[0]:.1f} us, back {us[1]:.1f} us, both concurrently {us[2]:.1f} us "
      f"(sum {us[0] + us[1]:.1f}); front high-priority {us[3]:.1f} us")
print(f"front graph || back op by op on a CU-masked stream: 8/8 {us[4]:.1f} us, 6/8 {us[5]:.1f} us, "
      f"4/8 {us[6]:.1f} us")
print(f"front || Mimi transformer || SEANet on three streams: {us[7]:.1f} us")
