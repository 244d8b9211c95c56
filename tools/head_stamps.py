import os, sys, json
import torch
buf = torch.zeros(4 * 128, dtype=torch.int64, device="cuda:0")
os.environ["PTTS_HEAD_DBG"] = str(buf.data_ptr())
sys.path.insert(0, "pocket-tts_amd")
import numpy as np
import pocket_tts_amd as pt
B = 32
eng = pt.Engine(device=0, max_slots=B, max_ctx=320, seed=0x5EED)
rng = np.random.default_rng(0)
v = eng.voice_from_prompt((0.11 * rng.standard_normal((125, 1024))).astype(np.float32))
eng.open_many(list(range(B)), [v] * B, [np.arange(40, dtype=np.int32) + b for b in range(B)],
              [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=100, seed=b + 1) for b in range(B)])
for _ in range(10):
    eng.step_async(B)
eng.sync()
print("chain_us", eng.time_kernel(B, "head.chain", 50))
eng.sync(); torch.cuda.synchronize()
d = buf.cpu().numpy().reshape(4, 128)
for wg in range(4):
    t = d[wg][:30].astype(np.int64)
    t = (t - t[0]) * 10 / 1000.0  # us (100 MHz)
    print(wg, " ".join(f"{x:.2f}" for x in t))
