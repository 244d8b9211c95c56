"""Per-op tile choice for the back part in f32 and bf16x6 (back_mfma): every big back-part GEMM /
conv of a frame-pair pass timed alone with HIP events (plus its split-K reduce) on candidate
layouts set through PTTS_OVR (probe builds: PTTS_LIB=<probe library>), uncapped and with the
pipelined step's per-CU cap (PTTS_TIME_CAP). The step is the arbiter (tools/ab.sh); this ranks
candidates. Usage: PTTS_LIB=... python tools/x6_tune.py [op ...]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import pocket_tts_amd as pt  # noqa: E402

OPS = {  # PTTS_OVR key -> (timed op, its reduce or None, splits)
    "mimi.qkv": ("mimi.l0.qkv_gemm", None, 1),
    "mimi.ff1": ("mimi.l0.ff1_gemm", None, 1),
    "mimi.ff2": ("mimi.l0.ff2_gemm", "mimi.l0.ff2_reduce", 4),
    "mimi.out": ("mimi.l0.out_gemm", "mimi.l0.out_reduce_ln2", 4),
    "seanet.conv0": ("seanet.conv0", "seanet.conv0_reduce", 4),
    "seanet.up0.convtr": ("seanet.up0.convtr", "seanet.up0.convtr_reduce", 4),
    "seanet.up1.convtr": ("seanet.up1.convtr", None, 1),
    "seanet.up2.convtr": ("seanet.up2.convtr", None, 1),
    "seanet.up0.res_conv3": ("seanet.up0.res_conv3", None, 1),
    "seanet.up1.res_conv3": ("seanet.up1.res_conv3", None, 1),
    "seanet.up2.res_conv3": ("seanet.up2.res_conv3", None, 1),
    "seanet.up0.res_conv1": ("seanet.up0.res_conv1", None, 1),
    "seanet.up1.res_conv1": ("seanet.up1.res_conv1", None, 1),
    "seanet.up2.res_conv1": ("seanet.up2.res_conv1", None, 1),
}
LAYOUTS = {0: [32, 39, 36, 31, 30, 35], 2: [232, 239, 236, 231, 230, 235]}
B = 32


def run(mfma, ops):
    os.environ["PTTS_RESBLOCK_STAGES"] = "0"  # stage 2 as its two convs (comparable in both modes)
    eng = pt.Engine(device=0, max_slots=B, max_ctx=400, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=2, back_mfma=mfma)
    voice = eng.voice_from_prompt(bench.synth_prompt())
    eng.open_many(list(range(B)), [voice] * B, [bench.text_ids(b) for b in range(B)],
                  [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1)
                   for b in range(B)])
    for _ in range(8):
        eng.step(B)
    for key in ops:
        op, red, s = OPS[key]
        for lay in LAYOUTS[mfma]:
            os.environ["PTTS_OVR"] = f"{key}={lay}:{s}" if red else f"{key}={lay}"
            res = []
            for cap in (False, True):
                if cap:
                    os.environ["PTTS_TIME_CAP"] = "1"
                else:
                    os.environ.pop("PTTS_TIME_CAP", None)
                try:
                    us = eng.time_kernel(B, op, reps=20) + (eng.time_kernel(B, red, reps=20) if red else 0.0)
                except pt.PocketTTSError as e:
                    us = float("nan")
                res.append(us)
            print(f"mfma {mfma} {key:22s} {lay:4d} alone {res[0]:7.2f} capped {res[1]:7.2f} us", flush=True)
        os.environ.pop("PTTS_OVR", None)
    eng.close()


ops = sys.argv[1:] or list(OPS)
for mfma in (0, 2):
    run(mfma, ops)
