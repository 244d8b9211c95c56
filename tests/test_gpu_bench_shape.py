"""GPU parity at the benchmark's own shape (BASELINE configs[2]): f32 engine, 32 rows, 125-frame
voice prompts, 40 text tokens, 132 free-running frames at temperature 0, pipelined stepping (the
bench's mode). The FlowLM context of every row grows 165 -> 297 positions, so the step attention
(k_attn_decode_qkv) takes its second 256-key round for the last 40 frames, and the Mimi decoder's
250-key window slides over 2,112 ring positions (four wraps of the 512-slot ring).

Checked every frame:
  row 0  (the golden `e2e_long` prompt and text) against the reference's own outputs for its
         first 100 frames (tests/golden/gen_golden.py long), and against the C oracle for all 132;
  rows 15, 16, 31 (their own prompts and texts; rows 15/16 straddle a 16-row group boundary of
         the flow-head launch and the attention tiles) against their own oracle runs.
The oracle is pinned to the reference at this shape by tests/test_oracle.py
(test_oracle_long_context_matches_reference).

Gates (all fp32; differences are reduction order only): EOS logit and latent <= 5e-5 max abs,
PCM <= 2e-6 max abs per frame (the golden PCM RMS is 0.035, so 6e-5 of the signal). The worst
errors seen are printed."""

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
from conftest import load_golden

pytestmark = pytest.mark.gpu

FRAMES, PROBE = 132, (0, 15, 16, 31)
LAT_TOL, PCM_TOL = 5e-5, 2e-6


def _row_inputs(d, b):
    if b == 0:
        return d["prompt"], d["text_ids"]
    prompt = np.roll(d["prompt"], 3 * b, axis=0) * np.float32(1.0 + 0.01 * b)
    ids = (d["text_ids"].astype(np.int64) * (b + 1) + 7 * b) % 4000
    return np.ascontiguousarray(prompt, np.float32), ids.astype(np.int32)


def _oracle_run(oracle, prompt, ids, n):
    s = oracle.new_state(320)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    lat, out = None, []
    for _ in range(n):
        o = s.step(lat)
        lat = o["latent"]
        out.append((o["eos_logit"], o["latent"], o["pcm"]))
    return out


def test_bench_shape_b32_long_context_matches_reference_and_oracle(oracle):
    import pocket_tts_amd as pt

    d = load_golden("e2e_long.safetensors")
    B = 32
    inputs = [_row_inputs(d, b) for b in range(B)]
    with ThreadPoolExecutor(len(PROBE)) as ex:  # the oracle runs free (temp 0): precompute them
        futs = {b: ex.submit(_oracle_run, oracle, *inputs[b], FRAMES) for b in PROBE}
        eng = pt.Engine(device=0, max_slots=B, max_ctx=320, lsd_decode_steps=1, seed=0x5EED, pipeline=True)
        try:
            voices = [eng.voice_from_prompt(p) for p, _ in inputs]
            params = pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), frames_after_eos=3,
                                         max_frames=FRAMES, seed=1)
            eng.open_many(list(range(B)), voices, [i for _, i in inputs], [params] * B)
            frames = []
            r = eng.step(B)
            assert not r.valid.any()  # pipelined: the first call returns no frame
            for i in range(FRAMES):
                r = eng.step(B)
                assert r.valid.all(), i
                assert bool(r.last.all()) == (i == FRAMES - 1) and not (r.last.any() and i < FRAMES - 1), i
                frames.append({b: (float(r.eos_logits[b]), r.latents[b].copy(), r.pcm[b].copy()) for b in PROBE})
            assert not eng.step(B).valid.any()
        finally:
            eng.close()
        ref = {b: f.result() for b, f in futs.items()}

    worst = {"golden": [0.0, 0.0, 0.0], "oracle": [0.0, 0.0, 0.0]}

    def cmp(kind, got, exp, where):
        e = [abs(got[0] - exp[0]), float(np.abs(got[1] - exp[1]).max()), float(np.abs(got[2] - exp[2]).max())]
        worst[kind] = [max(a, b) for a, b in zip(worst[kind], e)]
        assert e[0] <= LAT_TOL and e[1] <= LAT_TOL and e[2] <= PCM_TOL, (kind, where, e)

    for i in range(FRAMES):
        for b in PROBE:
            cmp("oracle", frames[i][b], ref[b][i], (i, b))
        if i < d["latent"].shape[0]:
            cmp("golden", frames[i][0], (d["eos_logit"][i], d["latent"][i], d["pcm"][i]), (i, 0))
    print(f"worst |d| eos/latent/pcm: vs golden {worst['golden']}, vs oracle {worst['oracle']}")
