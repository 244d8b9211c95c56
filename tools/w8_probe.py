"""FlowLM step GEMMs with int8 codes vs f32 weights (B rows): per-op HIP-event timings of every
front op, and the front/back/overlap probe (ptts_probe_overlap) for each engine."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import pocket_tts_amd as pt  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
modes = [("f32", 0, False), ("int8", 1, False), ("quant_f32kern", 1, True)]
tab = {}
for tag, q, off in modes:
    if off:
        os.environ["PTTS_W8_OFF"] = "1"
    else:
        os.environ.pop("PTTS_W8_OFF", None)
    eng = pt.Engine(device=0, max_slots=B, max_ctx=256, seed=0x5EED, weight_quant=q)
    plan = eng.plan(B)
    front = [n for n, _, _ in plan if n.startswith(("flow.", "head.", "front"))]
    tab[tag] = {n: eng.time_kernel(B, n, reps=30) for n in dict.fromkeys(front)}
    us = (C.c_double * 8)()
    pt.lib().ptts_probe_overlap(eng.handle, B, 30, us)
    print(json.dumps({"engine": tag, "front_ops_sum_us": round(sum(tab[tag].values()), 1),
                      "front_us": round(us[0], 1), "back_us": round(us[1], 1), "both_us": round(us[2], 1)}))
    eng.close()
for n in tab["f32"]:
    print(f"{n:32s} " + " ".join(f"{tab[t][n]:7.2f}" for t, _, _ in modes))
