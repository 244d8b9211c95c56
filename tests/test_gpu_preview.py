"""First-frame previews (ptts_preview_enable / ptts_preview_fetch) on the pipelined engine.

A preview decodes a new row's first frame right after its first FlowLM step, alone, from the fresh
Mimi state every utterance starts from (tts_model.rs:941 init_states), so the serving path's first
chunk does not wait the pipeline's frame lag. Checked here against the C oracle (PCM_TOL) and
against the row's own regular frame 0, with rows admitted at and inside a pass, more rows starting
in one call than previews allowed, a re-admitted slot, and the regular stream left unchanged."""

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err

pytestmark = pytest.mark.gpu

INF = float("inf")


def params(**kw):
    from pocket_tts_amd import GenerationParams

    base = dict(temp=0.0, eos_threshold=INF, noise_clamp=None, frames_after_eos=3, max_frames=64, seed=1)
    base.update(kw)
    return GenerationParams(**base)


@pytest.mark.parametrize("back_frames", [1, 2, 4])
def test_previews_equal_first_frames(oracle, back_frames):
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(29)
    S = 6
    eng = pt.Engine(device=0, max_slots=S, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames)
    try:
        eng.enable_preview(3)  # fewer than the 4 rows of the first admission
        orc, lat, frames, first = {}, {}, {}, {}
        previews = []

        def admit(slots, n_frames, scale):
            ids_l, vs = [], []
            for b in slots:
                F = 5 + 2 * b
                prompt = (d["prompt"][:F] * scale * (1.0 + 0.04 * b)).astype(np.float32)
                ids = rng.integers(0, 4000, size=3 + 2 * b).astype(np.int32)
                vs.append(eng.voice_from_prompt(prompt))
                ids_l.append(ids)
                s = oracle.new_state(256)
                s.prefill(prompt)
                s.prefill_tokens(ids)
                orc[b], lat[b], frames[b] = s, None, []
                first[b] = s.step(None)  # the oracle's frame 0 of the utterance
                lat[b] = first[b]["latent"]
            eng.open_many(slots, vs, ids_l, [params(max_frames=n_frames)] * len(slots))

        calls = [0]

        def step():
            calls[0] += 1
            eng.step_async(S)
            r = eng.fetch(S)
            previews.extend(eng.fetch_previews())
            for b in list(orc):
                if not r.valid[b]:
                    continue
                if not frames[b]:
                    o = first[b]
                else:
                    o = orc[b].step(lat[b])
                    lat[b] = o["latent"]
                frames[b].append(r.pcm[b].copy())
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL, (b, len(frames[b]))

        def check_previews(expect):
            previews.extend(eng.fetch_previews(wait=True))
            got = {}
            for slot, pcm in previews:
                assert slot not in got, slot
                got[slot] = pcm
            previews.clear()
            assert sorted(got) == sorted(expect), (sorted(got), expect)
            for b, pcm in got.items():
                assert pcm_err(pcm - first[b]["pcm"]) <= PCM_TOL, b
            return got

        admit([0, 1, 2, 3], 5, 1.0)  # call 0: a pass boundary; 4 rows start, 3 previews
        for _ in range(3):
            step()
        pv = check_previews([0, 1, 2])
        lag, _ = eng.frame_lag()
        for _ in range(2 * lag + 4):
            step()
        for b in range(4):
            assert len(frames[b]) == 5, (b, len(frames[b]))
        for b, pcm in pv.items():  # the preview is the row's regular frame 0 up to float rounding
            assert pcm_err(pcm - frames[b][0]) <= PCM_TOL, b
        # inside a pass (back_frames > 1): rows start at the next boundary, their previews with them;
        # slot 1 is re-admitted (its earlier utterance finished): a new preview for the new utterance
        while back_frames > 1 and calls[0] % back_frames == 0:
            step()
        admit([4, 5, 1], 4, 0.9)
        for _ in range(4):
            step()
        pv = check_previews([4, 5, 1])
        for _ in range(2 * lag + 4):
            step()
        for b in (4, 5, 1):
            assert len(frames[b]) == 4, (b, len(frames[b]))
            assert pcm_err(pv[b] - frames[b][0]) <= PCM_TOL, b
        assert eng.fetch_previews(wait=True) == []
    finally:
        eng.close()


def test_preview_needs_pipelined_engine():
    import pocket_tts_amd as pt

    eng = pt.Engine(device=0, max_slots=2, max_ctx=64, lsd_decode_steps=1, seed=0x5EED, pipeline=False)
    try:
        with pytest.raises(pt.PocketTTSError):
            eng.enable_preview(2)
    finally:
        eng.close()


def test_closed_slot_drops_its_preview(oracle):
    """A slot closed (or re-admitted) before its preview is fetched never returns that preview."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    eng = pt.Engine(device=0, max_slots=2, max_ctx=128, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=2)
    try:
        eng.enable_preview(2)
        v = eng.voice_from_prompt(d["prompt"][:6])
        ids = np.arange(5, dtype=np.int32)
        eng.open_many([0, 1], [v, v], [ids, ids], [params(max_frames=3)] * 2)
        eng.step_async(2)
        eng.sync()
        eng.close_slot(1)
        got = eng.fetch_previews(wait=True)
        assert [s for s, _ in got] == [0]
    finally:
        eng.close()


@pytest.mark.parametrize("back_frames", [2, 4])
def test_front_done_tracks_calls_from_its_first_use(back_frames):
    """ptts_front_done: calls issued before an engine's first front_done are answered from the front
    stream as a whole, later calls from their own event (a driver that never asks puts no event
    marker on the front stream per call). Both answers are consistent with the call order, and the
    frames of the stepping are unaffected."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    eng = pt.Engine(device=0, max_slots=4, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames)
    try:
        v = eng.voice_from_prompt(d["prompt"][:8])
        eng.open_many([0, 1], [v, v], [np.array([260, 2994, 262], np.int32)] * 2, [params(max_frames=40)] * 2)
        for _ in range(6):  # untracked calls
            eng.step_async(2)
        assert eng.front_done(3, wait=True)  # an untracked call: the stream as a whole
        assert eng.front_done(0, wait=False) in (True, False)
        for _ in range(6):  # tracked from here on
            eng.step_async(2)
            assert eng.front_done(1, wait=True)
        eng.sync()
        assert all(eng.front_done(k, wait=False) for k in range(4))
        eng.fetch(2)
    finally:
        eng.close()
