"""Edge cases of the C-ABI boundary on the GPU: argument errors surface as PocketTTSError (the
reference's anyhow::Error -> PyRuntimeError mapping, pocket-tts-bindings/src/lib.rs:17) and leave
the engine usable; an empty text segment and a context filled to exactly max_ctx run to the end
and match the oracle."""

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err, rms

pytestmark = pytest.mark.gpu


def _params(**kw):
    from pocket_tts_amd import GenerationParams

    base = dict(temp=0.0, eos_threshold=float("inf"), max_frames=4)
    base.update(kw)
    return GenerationParams(**base)


def test_boundary_errors_leave_engine_usable(gpu_engine, oracle):
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    v = gpu_engine.voice_from_prompt(d["prompt"][:6])
    ids = np.array([260, 2994, 262], np.int32)
    n = gpu_engine.max_slots
    bad = [
        lambda: gpu_engine.step(0),
        lambda: gpu_engine.step(n + 1),
        lambda: gpu_engine.open(n, v, ids, _params()),  # slot out of range
        lambda: gpu_engine.open(-1, v, ids, _params()),
        lambda: gpu_engine.open(0, v, np.array([4001], np.int32), _params()),  # token id past the vocab
        lambda: gpu_engine.open(0, v, ids, _params(max_frames=0)),
        lambda: gpu_engine.open(0, v, ids, _params(frames_after_eos=-1)),
        lambda: gpu_engine.open(0, v, ids, _params(max_frames=gpu_engine.max_ctx)),  # context overflow
        lambda: gpu_engine.voice_from_prompt(np.zeros((gpu_engine.max_ctx, 1024), np.float32)),
    ]
    for i, f in enumerate(bad):
        with pytest.raises(pt.PocketTTSError):
            f()
    # still works, and matches the oracle
    gpu_engine.open(0, v, ids, _params(max_frames=3))
    s = oracle.new_state(256)
    s.prefill(d["prompt"][:6])
    s.prefill_tokens(ids)
    lat = None
    for _ in range(3):
        r = gpu_engine.step(1)
        ref = s.step(lat)
        lat = ref["latent"]
        np.testing.assert_allclose(r.latents[0], ref["latent"], atol=LAT_TOL)
        assert pcm_err(r.pcm[0] - ref["pcm"]) <= PCM_TOL


def test_empty_text_segment_matches_oracle(gpu_engine, oracle):
    """0 text tokens: the step runs on the voice prefix alone (ptts_slot_open accepts n_ids = 0)."""
    d = load_golden("e2e_lsd1.safetensors")
    prompt = d["prompt"][:8]
    gpu_engine.open(1, gpu_engine.voice_from_prompt(prompt), np.zeros(0, np.int32), _params(max_frames=3))
    s = oracle.new_state(256)
    s.prefill(prompt)
    lat = None
    for i in range(3):
        r = gpu_engine.step(2)
        ref = s.step(lat)
        lat = ref["latent"]
        assert r.valid[1] and r.last[1] == (i == 2)
        np.testing.assert_allclose(r.latents[1], ref["latent"], atol=LAT_TOL)
        assert pcm_err(r.pcm[1] - ref["pcm"]) <= PCM_TOL


def test_context_filled_to_max_ctx(oracle):
    """voice + text + max_frames == max_ctx exactly: every frame matches the oracle and the row
    ends on its max_frames-th frame (the KV cache's last position is written by the last step)."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    F, ids = 9, d["text_ids"][:5]
    frames = 18
    max_ctx = F + ids.size + frames
    eng = pt.Engine(device=0, max_slots=1, max_ctx=max_ctx, seed=0x5EED)
    try:
        eng.open(0, eng.voice_from_prompt(d["prompt"][:F]), ids, _params(max_frames=frames))
        s = oracle.new_state(256)
        s.prefill(d["prompt"][:F])
        s.prefill_tokens(ids)
        lat = None
        for i in range(frames):
            r = eng.step(1)
            ref = s.step(lat)
            lat = ref["latent"]
            assert r.valid[0] and r.last[0] == (i == frames - 1)
            np.testing.assert_allclose(r.latents[0], ref["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[0] - ref["pcm"]) <= PCM_TOL
        assert not eng.step(1).valid[0]  # finished rows report no frame
    finally:
        eng.close()


def test_http_stream_route_on_real_engine(oracle):
    """The HTTP surface over the real pipelined engine (FastAPI TestClient, in process): two
    /stream requests at temperature 0 with token ids return 16-bit PCM equal to each request's
    oracle run (to 1 LSB), with max_gen_len frames (tts_model.rs:968-969 rule for the stated 2 words: (2 + 2) * 13 = 52)."""
    import pocket_tts_amd as pt
    from fastapi.testclient import TestClient
    from pocket_tts_amd.serve import BatchScheduler, TTSService, create_app

    d = load_golden("e2e_lsd1.safetensors")
    prompt = d["prompt"][:6]
    eng = pt.Engine(device=0, max_slots=2, max_ctx=128, seed=0x5EED, pipeline=True)
    sch = BatchScheduler(eng)
    try:
        svc = TTSService(sch, {"v": eng.voice_from_prompt(prompt)}, default_voice="v", temp=0.0)
        client = TestClient(create_app(svc))
        for ids in ([260, 2994, 262, 578], [17, 4, 3999, 1200]):
            r = client.post("/stream", json={"token_ids": ids, "words": 2, "temperature": 0.0, "eos_threshold": 1e9})
            assert r.status_code == 200
            got = np.frombuffer(r.content, "<i2")
            assert got.size == 52 * 1920
            s = oracle.new_state(128)
            s.prefill(prompt)
            s.prefill_tokens(np.array(ids, np.int32))
            lat, ref = None, []
            for _ in range(52):
                o = s.step(lat)
                lat = o["latent"]
                ref.append(o["pcm"])
            want = np.clip(np.concatenate(ref), -1.0, 1.0) * 32767.0
            assert np.abs(got.astype(np.float64) - want).max() <= 1.01  # truncation to i16 + f32 noise
    finally:
        sch.close()
        eng.close()


def _oracle_frames(oracle, prompt, ids, n, quant_oracle=None):
    s = (quant_oracle or oracle).new_state(256)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    lat, out = None, []
    for _ in range(n):
        o = s.step(lat)
        lat = o["latent"]
        out.append(o)
    return out


def test_pipelined_reopen_with_pending_frame_matches_oracle(oracle):
    """a slot re-admitted while its old utterance still has a frame in flight (front
    done, Mimi decode pending on the back stream). The back part of the next call must see the
    admission (it waits for the admission event): the old frame is dropped (no frame for the row
    that call), the new utterance starts from a fresh decoder state and matches its own oracle run
    frame for frame, and the neighbouring row is untouched."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    eng = pt.Engine(device=0, max_slots=2, max_ctx=128, seed=0x5EED, pipeline=True)
    try:
        pa, ia = d["prompt"][:7], d["text_ids"][:4]
        pb, ib = (d["prompt"][:9] * 1.1).astype(np.float32), d["text_ids"][2:8]
        pn, in_ = (d["prompt"][:5] * 0.9).astype(np.float32), d["text_ids"][5:]
        va, vb, vn = eng.voice_from_prompt(pa), eng.voice_from_prompt(pb), eng.voice_from_prompt(pn)
        eng.open_many([0, 1], [va, vb], [ia, ib], [_params(max_frames=20)] * 2)
        ref_b = _oracle_frames(oracle, pb, ib, 8)
        ref_n = _oracle_frames(oracle, pn, in_, 4)
        assert not eng.step(2).valid.any()
        r = eng.step(2)  # frame 0 of both rows; front has frame 1 in flight
        assert r.valid.all()
        eng.open(0, vn, in_, _params(max_frames=4))  # row 0's frame 1 is still pending
        r = eng.step(2)  # back part: row 0's pending frame is dropped, row 1 frame 1
        assert not r.valid[0] and r.valid[1]
        np.testing.assert_allclose(r.latents[1], ref_b[1]["latent"], atol=LAT_TOL)
        assert pcm_err(r.pcm[1] - ref_b[1]["pcm"]) <= PCM_TOL
        for i in range(4):
            r = eng.step(2)
            assert r.valid[0] and r.last[0] == (i == 3)
            np.testing.assert_allclose(r.latents[0], ref_n[i]["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[0] - ref_n[i]["pcm"]) <= PCM_TOL
            np.testing.assert_allclose(r.latents[1], ref_b[2 + i]["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[1] - ref_b[2 + i]["pcm"]) <= PCM_TOL
    finally:
        eng.close()


def test_quantized_engine_steps_right_after_create(oracle):
    """Regression for the r1 race (2f0ee5c): a null-stream memset of a fresh allocation raced the
    finalize kernels on the engine's non-blocking streams and zeroed a derived weight. Create int8
    engines and step them at once, pipelined, against the quantized oracle."""
    import pocket_tts_amd as pt
    from _oracle import Oracle

    d = load_golden("e2e_lsd1.safetensors")
    o = Oracle(0x5EED, 1)
    prompt, ids = d["prompt"][:6], d["text_ids"][:5]
    ref = _oracle_frames(oracle, prompt, ids, 2, quant_oracle=o)
    for _ in range(3):
        eng = pt.Engine(device=0, max_slots=1, max_ctx=64, seed=0x5EED, weight_quant=1, pipeline=True)
        try:
            eng.open(0, eng.voice_from_prompt(prompt), ids, _params(max_frames=2))
            assert not eng.step(1).valid.any()
            for i in range(2):
                r = eng.step(1)
                assert r.valid[0]
                assert abs(r.eos_logits[0] - ref[i]["eos_logit"]) <= LAT_TOL
                np.testing.assert_allclose(r.latents[0], ref[i]["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[0] - ref[i]["pcm"]) <= PCM_TOL
        finally:
            eng.close()


def test_head_chain_needs_coresident_workgroups(gpu_engine):
    """k_flow_head spins on counters other workgroups bump, so it is planned only when its whole
    grid fits on the device at once (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs); the
    8-slot engine's 32-workgroup grid always fits on an MI355X."""
    assert "head.chain" in gpu_engine.plan_ops(8)


def test_nan_latent_propagates_without_stalling_the_head_chain(gpu_engine, oracle):
    """A NaN backbone input (set_latent) makes that row's frame NaN, as in the reference, and does
    not stall the persistent flow-head launch: its hand-offs use an empty pattern that is itself a
    NaN, and every stored NaN is canonicalised. The other row's frame is unaffected."""
    import time

    d = load_golden("e2e_lsd1.safetensors")
    prompt = d["prompt"][:6]
    v = gpu_engine.voice_from_prompt(prompt)
    ids = np.array([260, 2994, 262], np.int32)
    for slot in (0, 1):
        gpu_engine.open(slot, v, ids, _params(max_frames=2))
    gpu_engine.step(2)  # first frame of both rows
    gpu_engine.set_latent(1, np.full(32, np.nan, np.float32))
    t0 = time.perf_counter()
    r = gpu_engine.step(2)
    assert time.perf_counter() - t0 < 1.0  # a timed-out hand-off wait takes seconds
    assert np.isnan(r.latents[1]).all() and np.isnan(r.pcm[1]).all()
    s = oracle.new_state(256)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    lat = s.step(None)["latent"]
    ref = s.step(lat)
    np.testing.assert_allclose(r.latents[0], ref["latent"], atol=LAT_TOL)
    assert pcm_err(r.pcm[0] - ref["pcm"]) <= PCM_TOL


def test_shared_voice_prefix_outlives_destroyed_voice(oracle):
    """Slots read a voice's prefix from the voice's own cache (one copy per voice):
    two slots share voice A, a third row holds voice B of another length. Destroying A while both
    of its utterances run defers the free to the last slot that lets go of it (re-admission with
    B, then slot_close); every frame matches the oracle, including the re-admitted row's."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    eng = pt.Engine(device=0, max_slots=3, max_ctx=128, seed=0x5EED, pipeline=True)
    try:
        pa, pb = d["prompt"][:7], (d["prompt"][:11] * 0.9).astype(np.float32)
        ia, ia2, ib = d["text_ids"][:4], d["text_ids"][3:9], d["text_ids"][1:6]
        va, vb = eng.voice_from_prompt(pa), eng.voice_from_prompt(pb)
        eng.open_many([0, 1, 2], [va, va, vb], [ia, ia2, ib], [_params(max_frames=10)] * 3)
        va.close()  # both of A's utterances still read its prefix
        refs = [_oracle_frames(oracle, pa, ia, 10), _oracle_frames(oracle, pa, ia2, 10),
                _oracle_frames(oracle, pb, ib, 10)]
        got = [[], [], []]
        for _ in range(eng.frame_lag()[0] + 4):
            r = eng.step(3)
            for b in range(3):
                if r.valid[b]:
                    got[b].append((r.latents[b].copy(), r.pcm[b].copy()))
        eng.open(0, vb, ib, _params(max_frames=3))  # row 0 lets go of A; row 1 still holds it
        ref0 = _oracle_frames(oracle, pb, ib, 3)
        got0 = []
        for _ in range(eng.frame_lag()[0] + 8):
            r = eng.step(3)
            if r.valid[0]:
                got0.append((r.latents[0].copy(), r.pcm[0].copy()))
            for b in (1, 2):
                if r.valid[b]:
                    got[b].append((r.latents[b].copy(), r.pcm[b].copy()))
        eng.close_slot(1)  # the last reference: A is freed here
        for b in range(3):
            assert len(got[b]) >= 4
            for i, (lat, pcm) in enumerate(got[b]):
                np.testing.assert_allclose(lat, refs[b][i]["latent"], atol=LAT_TOL)
                assert pcm_err(pcm - refs[b][i]["pcm"]) <= PCM_TOL
        assert len(got0) == 3
        for i, (lat, pcm) in enumerate(got0):
            np.testing.assert_allclose(lat, ref0[i]["latent"], atol=LAT_TOL)
            assert pcm_err(pcm - ref0[i]["pcm"]) <= PCM_TOL
        r = eng.step(3)  # the engine keeps stepping with the freed voice's rows closed
        assert not r.valid[1]
    finally:
        eng.close()
