"""Tile / split-K tuning of the back part's conv launches under the pipelined per-CU cap.

Caution (measured): the capped op time alone is the wrong objective. Every choice this tool
found faster alone made the pipelined step SLOWER (heavier workgroups crowd the concurrent front
part); the arbiter is the steady step time, e.g.
  VAR=PTTS_OVR VALUES="- seanet.up0.res_conv3=6" REPS=2 bash tools/sweep_env.sh

For each op, every candidate `layout[:splits]` is set through PTTS_OVR (read at each plan
build) and the op (plus its split-K reduce when it has one) is timed alone with HIP events, with
the cap of pipelined stepping (PTTS_TIME_CAP). Candidates the engine rejects are skipped.
Prints one line per candidate and the best per op. Usage: python tools/back_tune.py [op ...]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT))
os.environ["PTTS_TIME_CAP"] = "1"
import bench  # noqa: E402
import pocket_tts_amd as pt  # noqa: E402

LAYOUTS = [6, 11, 12, 13, 14, 15, 16, 8, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27]
OPS = {  # op -> (its reduce op or None, split counts to try)
    "seanet.conv0": ("seanet.conv0_reduce", [1, 2, 4, 8]),
    "seanet.up0.convtr": ("seanet.up0.convtr_reduce", [1, 2, 4, 8]),
    "seanet.up1.convtr": (None, [1]),
    "seanet.up2.convtr": (None, [1]),
    "seanet.up0.res_conv3": (None, [1]),
    "seanet.up1.res_conv3": (None, [1]),
    "seanet.up2.res_conv3": (None, [1]),
    "seanet.up0.res_conv1": (None, [1]),
    "seanet.up1.res_conv1": (None, [1]),
    "seanet.up2.res_conv1": (None, [1]),
}

B = 32
eng = pt.Engine(device=0, max_slots=B, max_ctx=400, lsd_decode_steps=1, seed=0x5EED, pipeline=True)
voice = eng.voice_from_prompt(bench.synth_prompt())
eng.open_many(list(range(B)), [voice] * B, [bench.text_ids(b) for b in range(B)],
              [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1)
               for b in range(B)])
for _ in range(4):
    eng.step(B)
ops = sys.argv[1:] or list(OPS)
for op in ops:
    red, splits = OPS[op]
    os.environ.pop("PTTS_OVR", None)
    base = eng.time_kernel(B, op, reps=20) + (eng.time_kernel(B, red, reps=20) if red else 0.0)
    print(f"{op} default {base:.1f} us", flush=True)
    best = (base, "default")
    for s in splits:
        for lay in LAYOUTS:
            cand = f"{lay}:{s}" if red else f"{lay}"
            os.environ["PTTS_OVR"] = f"{op}={cand}"
            try:
                us = eng.time_kernel(B, op, reps=20)
                if red and s > 1:
                    us += eng.time_kernel(B, red, reps=20)
            except pt.PocketTTSError:
                continue
            print(f"  {op} {cand} {us:.1f} us", flush=True)
            if us < best[0]:
                best = (us, cand)
    os.environ.pop("PTTS_OVR", None)
    print(f"BEST {op} {best[1]} {best[0]:.1f} us (default {base:.1f})", flush=True)
