"""GPU parity at the benchmark's own shape (BASELINE configs[2]): f32 engine, 32 rows, 125-frame
voice prompts, 40 text tokens, 132 free-running frames at temperature 0, pipelined stepping with
four frames per Mimi decode pass (the bench's mode since round 6), frame pairs and one frame per pass, and
with frame pairs on the bf16x6 back part (back_mfma = BACK_F32X6: f32 GEMMs as exact bf16 piece
products) at the same gates. The FlowLM context of every row grows 165 -> 297 positions, so the step attention
(k_attn_decode_qkv) takes its second 256-key round for the last 40 frames, and the Mimi decoder's
250-key window slides over 2,112 ring positions (four wraps of the 512-slot ring).

Checked every frame of EVERY row (an indexing fault confined to one row group, tile or XCD
block cannot pass):
  row 0     (the golden `e2e_long` prompt and text) against the reference's own outputs for its
            first 100 frames (tests/golden/gen_golden.py long);
  rows 0-31 (each its own prompt and text) against their own C-oracle runs for all 132 frames.
The 32 oracle runs are single-threaded each (OpenMP team size 1 per worker thread) on a pool of
min(16, cpus) threads (the GPU box's CPU share), started before the engine so that they overlap it.
The oracle is pinned to the reference at this shape by tests/test_oracle.py
(test_oracle_long_context_matches_reference).

Gates (all fp32; differences are reduction order only): EOS logit and latent <= 5e-5 max abs,
PCM <= 2e-6 max abs per frame (the golden PCM RMS is 0.035, so 6e-5 of the signal). The worst
errors seen are printed."""

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
from conftest import load_golden

pytestmark = pytest.mark.gpu

FRAMES, B = 132, 32
LAT_TOL, PCM_TOL = 5e-5, 2e-6


def _row_inputs(d, b):
    if b == 0:
        return d["prompt"], d["text_ids"]
    prompt = np.roll(d["prompt"], 3 * b, axis=0) * np.float32(1.0 + 0.01 * b)
    ids = (d["text_ids"].astype(np.int64) * (b + 1) + 7 * b) % 4000
    return np.ascontiguousarray(prompt, np.float32), ids.astype(np.int32)


def _oracle_run(oracle, prompt, ids, n):
    from _oracle import lib as oracle_lib

    oracle_lib().omp_set_num_threads(1)  # this worker thread's OpenMP team: one thread
    s = oracle.new_state(320)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    lat, out = None, []
    for _ in range(n):
        o = s.step(lat)
        lat = o["latent"]
        out.append((o["eos_logit"], o["latent"], o["pcm"]))
    return out


def _engine_frames(pt, inputs, back_frames, back_mfma=0):
    eng = pt.Engine(device=0, max_slots=B, max_ctx=320, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames, back_mfma=back_mfma)
    try:
        voices = [eng.voice_from_prompt(p) for p, _ in inputs]
        params = pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), frames_after_eos=3,
                                     max_frames=FRAMES, seed=1)
        eng.open_many(list(range(B)), voices, [i for _, i in inputs], [params] * B)
        lag, delay = eng.frame_lag()
        assert (lag, delay) == (2 * back_frames - 1, 0)
        frames = []
        for _ in range(lag + delay):  # pipelined: the first calls return no frame
            assert not eng.step(B).valid.any()
        for i in range(FRAMES):
            r = eng.step(B)
            assert r.valid.all(), i
            assert bool(r.last.all()) == (i == FRAMES - 1) and not (r.last.any() and i < FRAMES - 1), i
            frames.append([(float(r.eos_logits[b]), r.latents[b].copy(), r.pcm[b].copy()) for b in range(B)])
        assert not eng.step(B).valid.any()
        return frames
    finally:
        eng.close()


def test_bench_shape_b32_long_context_matches_reference_and_oracle(oracle):
    import pocket_tts_amd as pt

    d = load_golden("e2e_long.safetensors")
    inputs = [_row_inputs(d, b) for b in range(B)]
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with ThreadPoolExecutor(workers) as ex:  # the oracle runs free (temp 0): precompute them
        futs = {b: ex.submit(_oracle_run, oracle, *inputs[b], FRAMES) for b in range(B)}
        runs = {(bf, mf): _engine_frames(pt, inputs, bf, mf)
                for bf, mf in ((2, pt.BACK_F32), (1, pt.BACK_F32), (4, pt.BACK_F32), (2, pt.BACK_F32X6))}
        ref = {b: f.result() for b, f in futs.items()}

    worst = {"golden": [0.0, 0.0, 0.0], "oracle": [0.0, 0.0, 0.0]}

    def cmp(kind, got, exp, where):
        e = [abs(got[0] - exp[0]), float(np.abs(got[1] - exp[1]).max()), float(np.abs(got[2] - exp[2]).max())]
        worst[kind] = [max(a, b) for a, b in zip(worst[kind], e)]
        assert e[0] <= LAT_TOL and e[1] <= LAT_TOL and e[2] <= PCM_TOL, (kind, where, e)

    for bf, frames in runs.items():
        for i in range(FRAMES):
            for b in range(B):
                cmp("oracle", frames[i][b], ref[b][i], (bf, i, b))
            if i < d["latent"].shape[0]:
                cmp("golden", frames[i][0], (d["eos_logit"][i], d["latent"][i], d["pcm"][i]), (bf, i, 0))
        print(f"back_frames, back_mfma={bf}: worst |d| eos/latent/pcm: vs golden {worst['golden']}, "
              f"vs oracle {worst['oracle']}")


def _oracle_run_noisy(oracle, prompt, ids, n, seed, temp):
    from _oracle import lib as oracle_lib
    from test_gpu_parity import _noise

    oracle_lib().omp_set_num_threads(1)
    s = oracle.new_state(320)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    lat, out = None, []
    for i in range(n):
        o = s.step(lat, noise=_noise(seed, i, temp, None))
        lat = o["latent"]
        out.append((o["eos_logit"], o["latent"], o["pcm"]))
    return out


@pytest.mark.parametrize("back_frames", [2, 4])
def test_bench_exact_input_shared_voice_matches_oracle(oracle, back_frames):
    """bench.py's own job, input for input: ONE voice (bench.synth_prompt, 125 frames) admitted
    into all 32 rows in one batched admission, so every row reads the voice's shared KV prefix
    (KvStore::pre) rather than a copy; bench.text_ids(b); temperature 0.7 with bench.slot_seed's
    noise streams; EOS off; 125 frames; pipelined frame pairs drained by flush calls, exactly as
    bench.run_calls issues them. Every row and frame against its own oracle run (the same noise,
    replayed on the host by test_gpu_parity._noise), at the f32 gates."""
    import bench
    import pocket_tts_amd as pt

    n, temp = bench.UTT_FRAMES, 0.7
    prompt = bench.synth_prompt()
    ids = [bench.text_ids(b) for b in range(B)]
    seeds = [bench.slot_seed(1, 0, b) for b in range(B)]
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with ThreadPoolExecutor(workers) as ex:
        futs = [ex.submit(_oracle_run_noisy, oracle, prompt, ids[b], n, seeds[b], temp) for b in range(B)]
        eng = pt.Engine(device=0, max_slots=B, max_ctx=bench.PROMPT_FRAMES + bench.TEXT_TOKENS + n + 8,
                        lsd_decode_steps=1, seed=0x5EED, pipeline=True, back_frames=back_frames)
        try:
            voice = eng.voice_from_prompt(prompt)
            eng.open_many(list(range(B)), [voice] * B, ids,
                          [pt.GenerationParams(temp=temp, eos_threshold=float("inf"), frames_after_eos=3,
                                               max_frames=n, seed=seeds[b]) for b in range(B)])
            lag, delay = eng.frame_lag()
            got = [[] for _ in range(B)]

            def collect():
                eng.sync()
                r = eng.fetch(B)
                for b in range(B):
                    if r.valid[b]:
                        got[b].append((float(r.eos_logits[b]), r.latents[b].copy(), r.pcm[b].copy()))

            for _ in range(n + delay):
                eng.step_async(B)
                collect()
            for _ in range(lag):
                eng.flush_async(B)
                collect()
        finally:
            eng.close()
        ref = [f.result() for f in futs]
    worst = [0.0, 0.0, 0.0]
    for b in range(B):
        assert len(got[b]) == n, (b, len(got[b]))
        for i in range(n):
            g, e = got[b][i], ref[b][i]
            err = [abs(g[0] - e[0]), float(np.abs(g[1] - e[1]).max()), float(np.abs(g[2] - e[2]).max())]
            worst = [max(x, y) for x, y in zip(worst, err)]
            assert err[0] <= LAT_TOL and err[1] <= LAT_TOL and err[2] <= PCM_TOL, (b, i, err)
    print(f"bench input (shared voice, temp {temp}, back_frames {back_frames}): worst |d| eos/latent/pcm vs oracle "
          f"{worst}")


@pytest.mark.parametrize("back_frames", [2, 4])
def test_overlapped_admission_job_loop_completes_every_job(back_frames):
    """bench.py's job loop: the next job's batched admission is issued before the previous job's
    last frame is fetched (its prefill runs beside that job's last back passes). Every job's last
    frame must come back valid and last for all 32 rows. Regression for the drained-slot race
    (DESIGN.md 14.8): the fetch of job j's last frame marked the slots of job j + 1 drained, so
    job j + 2's admission could reset their state ahead of job j + 1's queued back passes.
    (tools/race_probe.py runs the same loop for many more jobs.)"""
    import sys

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    import bench
    import pocket_tts_amd as pt

    K = 24
    eng = pt.Engine(device=0, max_slots=B, max_ctx=bench.PROMPT_FRAMES + bench.TEXT_TOKENS + K + 8,
                    lsd_decode_steps=1, seed=0x5EED, pipeline=True, back_frames=back_frames)
    try:
        v = eng.voice_from_prompt(bench.synth_prompt())

        def admit(j):
            eng.open_many(list(range(B)), [v] * B, [bench.text_ids(b) for b in range(B)],
                          [pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=K,
                                               seed=bench.slot_seed(j, 0, b)) for b in range(B)])

        admit(0)
        for j in range(24):
            lag, delay = eng.frame_lag()
            for _ in range(K + delay):
                eng.step_async(B)
            for _ in range(lag):
                eng.flush_async(B)
            if j + 1 < 24:
                admit(j + 1)
            r = eng.fetch(B)
            assert r.valid.all() and r.last.all(), (j, np.nonzero(~r.valid)[0][:8])
            assert np.isfinite(r.pcm).all()
    finally:
        eng.close()
