"""Persistent FlowLM launch (k_flow_lm) phase breakdown: s_memrealtime stamps (100 MHz) of
workgroups 0 (a row reducer), 37 and 255 of the last flow.layers launch (PTTS_FLM_DBG buffer; probe
build: PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so), B = 32 rows at a mid-job context.
Per layer the stamps close: qkv staged (h ready), qkv GEMM, attention, out staged, out GEMM,
reduce2 (or the idle workgroups' region fill), ff1 staged, ff1 GEMM, ff2 staged, ff2 GEMM, reduce1."""
import os
import sys

import torch

buf = torch.zeros(3 * 128, dtype=torch.int64, device="cuda:0")
os.environ["PTTS_FLM_DBG"] = str(buf.data_ptr())
os.environ["PTTS_FLM_ON"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402

B = int(os.environ.get("B", "32"))
eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED)
rng = np.random.default_rng(0)
v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
              [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1) for b in range(B)])
for _ in range(60):
    eng.step_async(B)
eng.sync()
print("flow.layers us (isolated, HIP events)", round(eng.time_kernel(B, "flow.layers", 20), 2))
eng.sync()
torch.cuda.synchronize()
names = ["qkv_staged", "qkv_gemm", "attention", "out_staged", "out_gemm", "red2|fill", "ff1_staged", "ff1_gemm",
         "ff2_staged", "ff2_gemm", "red1"]
s = buf.cpu().numpy().reshape(3, 128)
for k, wg in enumerate([0, 37, 255]):
    t = s[k]
    n = int(np.count_nonzero(t))
    t = t[:n].astype(np.int64)
    d = np.diff(t) * 10 / 1000.0  # us
    print(f"wg{wg}: {n} stamps, total {(t[-1] - t[0]) * 10 / 1000:.2f} us")
    per = {x: [] for x in names}
    for i, x in enumerate(d):
        per[names[i % len(names)]].append(x)
    print("  " + "  ".join(f"{x} {np.mean(val):.2f}" for x, val in per.items() if val))
eng.close()
