"""Engine-variant probe (FP8=1 / WQ=<mode> select the fp8 / int8 engines): for each environment variant (JSON list of dicts on argv[1]), run in a fresh
process the bench workload (B = 32 rows, 125 pipelined steps after batched admission), report the
steady ms/step and the HIP-event time of selected ops, and the max |diff| of the first 8 frames'
latents / PCM against the first variant (so a variant that changes numerics shows it)."""
import json
import os
import subprocess
import sys

import numpy as np

B, K = 32, 125

if len(sys.argv) > 2 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
    import time

    import pocket_tts_amd as pt

    ops = sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] else []
    eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED, pipeline=True,
                    fp8_gemm=bool(int(os.environ.get("FP8", "0"))), weight_quant=int(os.environ.get("WQ", "0")))
    rng = np.random.default_rng(0)
    v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
    res = {}
    for rnd in range(2):
        eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
                      [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=K, seed=b + 1)
                       for b in range(B)])
        eng.sync()
        if rnd == 0:  # numerics: first frames
            lat, pcm = [], []
            for _ in range(9):
                r = eng.step(B)
                if r.valid.any():
                    lat.append(np.array(r.latents))
                    pcm.append(np.array(r.pcm))
            np.savez(sys.argv[2], lat=np.stack(lat), pcm=np.stack(pcm))
            for _ in range(K - 8):
                eng.step_async(B)
            eng.sync()
            continue
        t0 = time.perf_counter()
        for _ in range(K + 1):
            eng.step_async(B)
        eng.sync()
        res["ms_per_step"] = round(1e3 * (time.perf_counter() - t0) / K, 4)
    for o in ops:
        res[o] = round(eng.time_kernel(B, o, 30), 2)
    print("RESULT " + json.dumps(res), flush=True)
    eng.close()
else:
    variants = json.loads(sys.argv[1])
    ops = sys.argv[2] if len(sys.argv) > 2 else ""
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    ref = None
    for i, var in enumerate(variants):
        env = dict(os.environ, **var)
        f = os.path.join(out, f"variant{i}.npz")
        p = subprocess.run([sys.executable, __file__, "child", f, ops], env=env, capture_output=True, text=True,
                           timeout=300)
        if p.returncode != 0:
            print(json.dumps({"variant": var, "rc": p.returncode, "err": p.stderr[-2000:]}), flush=True)
            sys.exit(p.returncode)
        line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
        r = json.loads(line[7:])
        d = np.load(f)
        if ref is None:
            ref = d
        r["lat_maxdiff"] = float(np.abs(d["lat"] - ref["lat"]).max())
        r["pcm_maxdiff"] = float(np.abs(d["pcm"] - ref["pcm"]).max())
        print(json.dumps({"variant": var, **r}), flush=True)
