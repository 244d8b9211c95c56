"""Output difference of two builds of the library on the bench's job (f32 engine, 32 rows, one voice,
temperature 0, pipelined frame pairs): each library runs in its own child process (PTTS_LIB), the
PCM and latents of every row and frame go to an .npz, and the max abs differences are printed. For a
tile or reduction-order change that has no GPU test of its own build (e.g. a -D variant library).

    python tools/lib_diff.py A.so B.so [frames] [back_frames]
"""

import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out, frames, back_frames=2):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "pocket-tts_amd"))
    import bench
    import pocket_tts_amd as pt

    B = 32
    eng = pt.Engine(device=0, max_slots=B, max_ctx=bench.PROMPT_FRAMES + bench.TEXT_TOKENS + frames + 8,
                    lsd_decode_steps=1, seed=0x5EED, pipeline=True, back_frames=back_frames)
    try:
        voice = eng.voice_from_prompt(bench.synth_prompt())
        eng.open_many(list(range(B)), [voice] * B, [bench.text_ids(b) for b in range(B)],
                      [pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), frames_after_eos=3,
                                           max_frames=frames, seed=1)] * B)
        lag, delay = eng.frame_lag()
        pcm, lat = [], []
        for i in range(frames + lag + delay):
            r = eng.step(B)
            if r.valid.all():
                pcm.append(r.pcm.copy())
                lat.append(r.latents.copy())
        np.savez(out, pcm=np.stack(pcm), lat=np.stack(lat), build=np.array(pt.build_id()))
    finally:
        eng.close()


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
        return
    a, b = sys.argv[1], sys.argv[2]
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    bf = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    res = []
    with tempfile.TemporaryDirectory() as d:
        for i, lib in enumerate((a, b)):
            out = os.path.join(d, f"{i}.npz")
            env = dict(os.environ, PTTS_LIB=os.path.abspath(lib))
            subprocess.run([sys.executable, __file__, "--child", out, str(frames), str(bf)], env=env, check=True,
                           timeout=300)
            res.append(np.load(out))
    dp = np.abs(res[0]["pcm"] - res[1]["pcm"]).max(axis=(1, 2))
    dl = np.abs(res[0]["lat"] - res[1]["lat"]).max(axis=(1, 2))
    print(f"{res[0]['build']} vs {res[1]['build']}: frames {len(dp)}, max |d pcm| {dp.max():.3g} "
          f"(first frame {dp[0]:.3g}), max |d latent| {dl.max():.3g} (first frame {dl[0]:.3g})")


if __name__ == "__main__":
    main()
