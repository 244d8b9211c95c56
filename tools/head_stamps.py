"""Flow-head chain phase breakdown: s_memrealtime stamps (100 MHz) of workgroups 0..3 of the last
head.chain launch (PTTS_HEAD_DBG buffer), B = 32, steady-state KV; per ResBlock the stamps are
[mlp1 sweep start, sweep done, LN done, GEMM done, u stored, mlp2 sweep done, GEMM done, x stored]."""
import os
import sys

import torch

buf = torch.zeros(4 * 128, dtype=torch.int64, device="cuda:0")
os.environ["PTTS_HEAD_DBG"] = str(buf.data_ptr())
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pocket-tts_amd"))
import numpy as np  # noqa: E402

import pocket_tts_amd as pt  # noqa: E402

B = int(os.environ.get("B", "32"))
eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED)
rng = np.random.default_rng(0)
v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
              [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1) for b in range(B)])
for _ in range(10):
    eng.step_async(B)
eng.sync()
print("chain_us (isolated, HIP events)", round(eng.time_kernel(B, "head.chain", 50), 2))
eng.sync()
torch.cuda.synchronize()
names = ["sweep1", "ln", "gemm1", "store_u", "sweep2", "gemm2", "store_x", "next"]
# stamps: [entry, x0 published] + 6 x 8 ResBlock stamps + (final layer WGs 0-3: [swept, done])
s = buf.cpu().numpy().reshape(4, 128)
for wg in range(4):
    t = s[wg]
    n = int(np.count_nonzero(t))
    t = t[:n].astype(np.int64)
    d = np.diff(t) * 10 / 1000.0  # us
    print(f"wg{wg}: {n} stamps, total {(t[-1] - t[0]) * 10 / 1000:.2f} us; prologue {d[0]:.2f} us (entry -> x0 "
          f"published), x0 -> block 0 {d[1]:.2f}" + (f"; final layer: sweep {d[-2]:.2f}, rest {d[-1]:.2f}" if n > 51 else ""))
    per = {k: [] for k in names}
    for i, x in enumerate(d[2:2 + 47]):
        per[names[i % len(names)]].append(x)
    print("  " + "  ".join(f"{k} {np.mean(val):.2f}" for k, val in per.items() if val))
eng.close()
