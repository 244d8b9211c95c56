"""GPU parity: the HIP engine through the C ABI against the reference's golden vectors
(tests/golden, produced by the reference's own Python modules) and the C oracle.

Tolerances (conftest.py; north_star asks for PCM within 1e-4 RMS, these are far tighter):
  eos logit and latent  <= LAT_TOL = 5e-5 max abs
  PCM                   <= PCM_TOL = 2e-6 max abs per frame
All arithmetic is fp32 on both sides; differences are reduction order only."""

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err, rms

pytestmark = pytest.mark.gpu

INF = float("inf")


def params(**kw):
    from pocket_tts_amd import GenerationParams

    base = dict(temp=0.0, eos_threshold=INF, noise_clamp=None, frames_after_eos=3, max_frames=64, seed=1)
    base.update(kw)
    return GenerationParams(**base)


def check_step(r, row, d, i):
    assert r.valid[row]
    assert abs(r.eos_logits[row] - d["eos_logit"][i]) <= LAT_TOL, (i, r.eos_logits[row], d["eos_logit"][i])
    np.testing.assert_allclose(r.latents[row], d["latent"][i], atol=LAT_TOL)
    diff = r.pcm[row] - d["pcm"][i]
    assert pcm_err(diff) <= PCM_TOL, (i, rms(diff), pcm_err(diff))


def test_e2e_matches_reference_golden(gpu_engine):
    d = load_golden("e2e_lsd1.safetensors")
    v = gpu_engine.voice_from_prompt(d["prompt"])
    assert v.n_frames == d["prompt"].shape[0]
    n = d["latent"].shape[0]
    gpu_engine.open(0, v, d["text_ids"], params(max_frames=n))
    for i in range(n):
        r = gpu_engine.step(1)
        check_step(r, 0, d, i)
        assert bool(r.last[0]) == (i == n - 1)
    r = gpu_engine.step(1)
    assert not r.valid[0]


def test_e2e_lsd2_matches_reference_golden():
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd2.safetensors")
    eng = pt.Engine(device=0, max_slots=1, max_ctx=128, lsd_decode_steps=2, seed=0x5EED)
    try:
        v = eng.voice_from_prompt(d["prompt"])
        eng.open(0, v, d["text_ids"], params(max_frames=8))
        for i in range(d["latent"].shape[0]):
            check_step(eng.step(1), 0, d, i)
    finally:
        eng.close()


def test_voice_cloning_encoder_matches_reference(gpu_engine):
    d = load_golden("encoder_4f.safetensors")
    v = gpu_engine.voice_from_pcm(d["pcm"])
    assert v.n_frames == 4
    np.testing.assert_allclose(v.conditioning(), d["conditioning"], atol=1e-5)


def test_ragged_batch_matches_oracle(gpu_engine, oracle):
    """8 slots with different voice lengths and text lengths (ragged KV positions) stepped
    together; every row must equal its own single-utterance oracle run."""
    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(7)
    B, steps = 8, 4
    orc, voices = [], []
    for b in range(B):
        F = 4 + 3 * b
        prompt = (d["prompt"][:F] * (1.0 + 0.1 * b)).astype(np.float32)
        ids = rng.integers(0, 4000, size=2 + b).astype(np.int32)
        v = gpu_engine.voice_from_prompt(prompt)
        voices.append(v)
        gpu_engine.open(b, v, ids, params(max_frames=steps))
        s = oracle.new_state(128)
        s.prefill(prompt)
        s.prefill_tokens(ids)
        orc.append(s)
    lat = [None] * B
    for i in range(steps):
        r = gpu_engine.step(B)
        for b in range(B):
            o = orc[b].step(lat[b])
            lat[b] = o["latent"]
            assert r.valid[b]
            assert abs(r.eos_logits[b] - o["eos_logit"]) <= LAT_TOL
            np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL


def test_batched_admission_matches_oracle(gpu_engine, oracle):
    """ptts_slots_open: 8 utterances admitted in one call, out of slot order, with ragged text
    (0..37 tokens: padding rows inside 16-row groups, groups of one slot spanning several tiles)
    and different voices; every row must equal its own oracle run."""
    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(11)
    B, steps = 8, 3
    slots = [5, 0, 7, 2, 1, 6, 3, 4]
    n_tok = [0, 1, 15, 16, 17, 37, 5, 32]
    voices, ids_list, orc = [], [], {}
    for i, b in enumerate(slots):
        F = 3 + 2 * i
        prompt = (d["prompt"][:F] * (1.0 - 0.05 * i)).astype(np.float32)
        ids = rng.integers(0, 4000, size=n_tok[i]).astype(np.int32)
        voices.append(gpu_engine.voice_from_prompt(prompt))
        ids_list.append(ids)
        s = oracle.new_state(128)
        s.prefill(prompt)
        if ids.size:
            s.prefill_tokens(ids)
        orc[b] = s
    gpu_engine.open_many(slots, voices, ids_list, [params(max_frames=steps)] * B)
    lat = {b: None for b in slots}
    for _ in range(steps):
        r = gpu_engine.step(B)
        for b in slots:
            o = orc[b].step(lat[b])
            lat[b] = o["latent"]
            assert r.valid[b]
            assert abs(r.eos_logits[b] - o["eos_logit"]) <= LAT_TOL
            np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL


def test_eos_termination_rule(gpu_engine):
    """tts_model.rs:1055-1063: the step reaching eos_step + frames_after_eos is yielded and is
    the last; without EOS the segment ends after max_gen_len frames."""
    d = load_golden("e2e_lsd1.safetensors")
    logits = d["eos_logit"]
    v = gpu_engine.voice_from_prompt(d["prompt"])
    for thr, fae, max_frames in [(-0.5, 2, 12), (-0.36, 1, 12), (10.0, 3, 5), (-0.6, 0, 12)]:
        above = np.nonzero(logits > thr)[0]
        assert np.min(np.abs(logits - thr)) > 1e-3
        expect = min(above[0] + fae + 1, max_frames) if above.size else max_frames
        gpu_engine.open(0, v, d["text_ids"], params(eos_threshold=thr, frames_after_eos=fae, max_frames=max_frames))
        got = 0
        while True:
            r = gpu_engine.step(1)
            if not r.valid[0]:
                break
            got += 1
            if r.last[0]:
                break
            assert got < 50
        assert got == expect, (thr, fae, got, expect)


def _mix64(z):
    z = np.uint64(z)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _normal_at(seed, step, k, att):
    M = 2**64
    base = _mix64((seed * 0x9E3779B97F4A7C15 + step * 0xD1B54A32D192ED03 + (k * 64 + att) * 0x8CB92BA72F3D8DD7) % M)
    f = np.float32
    u1 = (f(int(base) >> 41) + f(0.5)) * f(1.0 / 8388608.0)
    u2 = f(int(_mix64(int(base) ^ 0x5851F42D4C957F2D)) >> 40) * f(1.0 / 16777216.0)
    return np.sqrt(f(-2.0) * np.log(u1)) * np.cos(f(6.283185307179586) * u2)


def _noise(seed, step, temp, clamp):
    sd = np.sqrt(np.float32(temp))
    out = np.zeros(32, np.float32)
    for k in range(32):
        x = sd * _normal_at(seed, step, k, 0)
        if clamp:
            att = 1
            while abs(x) > clamp and att < 64:
                x = sd * _normal_at(seed, step, k, att)
                att += 1
            x = min(max(x, -clamp), clamp)
        out[k] = x
    return out


@pytest.mark.parametrize("clamp", [None, 0.5])
def test_temperature_sampling_matches_oracle(gpu_engine, oracle, clamp):
    """temp > 0: the engine's counter-based N(0, sqrt(temp)) (optionally truncated,
    flow_lm.rs:39-65) replayed on the host and fed to the oracle as x_0."""
    d = load_golden("e2e_lsd1.safetensors")
    seed, temp = 1234, 0.7
    v = gpu_engine.voice_from_prompt(d["prompt"][:10])
    gpu_engine.open(0, v, d["text_ids"][:5], params(temp=temp, noise_clamp=clamp, seed=seed, max_frames=4))
    s = oracle.new_state(64)
    s.prefill(d["prompt"][:10])
    s.prefill_tokens(d["text_ids"][:5])
    lat = None
    for i in range(3):
        r = gpu_engine.step(1)
        o = s.step(lat, noise=_noise(seed, i, temp, clamp))
        lat = o["latent"]
        np.testing.assert_allclose(r.latents[0], o["latent"], atol=LAT_TOL)
        assert pcm_err(r.pcm[0] - o["pcm"]) <= PCM_TOL


def test_steps_are_deterministic_and_slots_reset(gpu_engine):
    d = load_golden("e2e_lsd1.safetensors")
    v = gpu_engine.voice_from_prompt(d["prompt"])
    runs = []
    for _ in range(2):
        gpu_engine.open(3, v, d["text_ids"], params(max_frames=3))
        runs.append(np.stack([gpu_engine.step(4).pcm[3] for _ in range(3)]))
    assert np.array_equal(runs[0], runs[1])
    np.testing.assert_allclose(runs[0], d["pcm"][:3], atol=PCM_TOL)


def test_generate_convenience(gpu_engine):
    d = load_golden("e2e_lsd1.safetensors")
    v = gpu_engine.voice_from_prompt(d["prompt"])
    pcm = gpu_engine.generate(0, v, d["text_ids"], params(eos_threshold=-4.0, frames_after_eos=2, max_frames=12))
    # EOS fires at step 0 (every golden logit > -4), so frames 0..2 are produced
    assert pcm.size == 3 * 1920
    assert pcm_err(pcm - d["pcm"][:3].reshape(-1)) <= PCM_TOL


def test_plan_and_kernel_timer(gpu_engine):
    names = gpu_engine.plan_ops(8)
    assert "flow.l0.qkv_gemm" in names and "seanet.conv0" in names and names[-1] == "commit"
    assert gpu_engine.time_kernel(8, "flow.l0.qkv_gemm", reps=5) > 0


def test_pipelined_stepping_matches_oracle(oracle):
    """pipeline=1: the Mimi decode of frame k overlaps the FlowLM step of frame k+1, and a call
    returns the previous call's frame. Rows admitted at different times (continuous batching)
    and a row re-admitted after it finished must still equal their oracle runs frame for frame."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(5)
    eng = pt.Engine(device=0, max_slots=4, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True)
    try:
        voices, orc, lat, got = {}, {}, {}, {}

        def admit(slots, n_frames):
            ids_l, vs = [], []
            for b in slots:
                F = 5 + 3 * b
                prompt = (d["prompt"][:F] * (1.0 + 0.07 * b)).astype(np.float32)
                ids = rng.integers(0, 4000, size=3 + 4 * b).astype(np.int32)
                voices[b] = eng.voice_from_prompt(prompt)
                vs.append(voices[b])
                ids_l.append(ids)
                s = oracle.new_state(256)
                s.prefill(prompt)
                s.prefill_tokens(ids)
                orc[b], lat[b], got[b] = s, None, 0
            eng.open_many(slots, vs, ids_l, [params(max_frames=n_frames)] * len(slots))

        def check_frames(r):
            for b in list(orc):
                if not r.valid[b]:
                    continue
                o = orc[b].step(lat[b])
                lat[b] = o["latent"]
                got[b] += 1
                assert abs(r.eos_logits[b] - o["eos_logit"]) <= LAT_TOL
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL

        admit([0, 1], 4)
        r = eng.step(4)
        assert not r.valid.any()  # first call: nothing decoded yet
        check_frames(eng.step(4))
        admit([2, 3], 3)  # joins while rows 0/1 have a frame in flight
        for _ in range(3):
            check_frames(eng.step(4))
        assert got[0] == 4 and got[1] == 4
        admit([0], 2)  # re-admission of a finished row
        for _ in range(4):
            check_frames(eng.step(4))
        assert got[0] == 2 and got[2] == 3 and got[3] == 3
        assert not eng.step(4).valid.any()
    finally:
        eng.close()


@pytest.mark.parametrize("back_frames", [2, 4])
def test_frame_pairs_continuous_batching_matches_oracle(oracle, back_frames):
    """back_frames = n (2 or 4): one Mimi decode pass per n frames, a call returns the frame computed
    2 n - 1 calls earlier. Rows admitted at a pass boundary, rows admitted inside a pass (they start
    at the next boundary, so that an utterance's frames group into passes from its first), a row
    whose utterance ends on the first frame of a pass (5 frames: the pass commits its codec state
    through that frame only) and a row re-admitted after it finished must all equal their oracle
    runs frame for frame."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(7)
    n = back_frames
    lag = 2 * n - 1
    eng = pt.Engine(device=0, max_slots=4, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=n)
    try:
        orc, lat, got, want = {}, {}, {}, {}
        calls = [0]

        def admit(slots, n_frames):
            ids_l, vs = [], []
            for b in slots:
                F = 6 + 2 * b
                prompt = (d["prompt"][:F] * (1.0 + 0.05 * b)).astype(np.float32)
                ids = rng.integers(0, 4000, size=4 + 3 * b).astype(np.int32)
                vs.append(eng.voice_from_prompt(prompt))
                ids_l.append(ids)
                s = oracle.new_state(256)
                s.prefill(prompt)
                s.prefill_tokens(ids)
                orc[b], lat[b], got[b], want[b] = s, None, 0, n_frames
            eng.open_many(slots, vs, ids_l, [params(max_frames=n_frames)] * len(slots))
            return eng.frame_lag()

        def step_check():
            r = eng.step(4)
            calls[0] += 1
            for b in list(orc):
                if not r.valid[b]:
                    continue
                o = orc[b].step(lat[b])
                lat[b] = o["latent"]
                got[b] += 1
                assert got[b] <= want[b], b
                assert bool(r.last[b]) == (got[b] == want[b]), (b, got[b])
                assert abs(r.eos_logits[b] - o["eos_logit"]) <= LAT_TOL
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL
            return r

        assert admit([0, 1], 5) == (lag, 0)  # call 0 (a pass boundary); 5 frames end on a pass's first
        for _ in range(lag):
            assert not step_check().valid.any()
        c = calls[0]  # inside a pass: rows 2/3 start at the next boundary
        assert admit([2, 3], 4) == (lag, (n - c % n) % n)
        for _ in range(2 * lag):
            step_check()
        assert got[0] == 5 and got[1] == 5  # frames 0..4 of rows 0/1 arrived
        admit([0], 3)  # re-admission of a finished row
        for _ in range(2 * lag + n + 3):
            step_check()
        assert got[0] == 3 and got[2] == 4 and got[3] == 4
        assert not eng.step(4).valid.any()
    finally:
        eng.close()


@pytest.mark.parametrize("back_frames", [1, 2, 4])
def test_varying_rows_per_call_match_oracle(oracle, back_frames):
    """Pipelined stepping with n_rows changing from call to call, so rows pause (outside n_rows)
    and resume with their codec state intact: the overlap-add history, conv histories and Mimi
    position of a row outside a pass must not move. back_frames=2: a row the even
    call left out must not produce the pair's second frame alone (the pass decodes a row's frames
    of a pair as a prefix), so an odd call covers at most the even call's rows and the row pauses
    for the pair. Every frame a row does get must equal its oracle run, in order."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(13)
    n_frames = 6
    eng = pt.Engine(device=0, max_slots=4, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames)
    try:
        orc, lat, got, ids_l, vs = {}, {}, {}, [], []
        for b in range(4):
            F = 5 + 2 * b
            prompt = (d["prompt"][:F] * (1.0 + 0.03 * b)).astype(np.float32)
            ids = rng.integers(0, 4000, size=3 + 2 * b).astype(np.int32)
            vs.append(eng.voice_from_prompt(prompt))
            ids_l.append(ids)
            s = oracle.new_state(256)
            s.prefill(prompt)
            s.prefill_tokens(ids)
            orc[b], lat[b], got[b] = s, None, 0
        eng.open_many(list(range(4)), vs, ids_l, [params(max_frames=n_frames)] * 4)
        # (even, odd) row counts per pair: odd > even leaves rows [even, odd) paused for the pair
        pattern = [(1, 4), (4, 4), (2, 3), (3, 1), (4, 2), (1, 4)] + [(4, 4)] * 8
        for ne, no in pattern:
            for n in (ne, no):
                eng.step_async(n)
                r = eng.fetch(4)  # the frame of an earlier call may cover more rows than n
                for b in range(4):
                    if not r.valid[b]:
                        continue
                    o = orc[b].step(lat[b])
                    lat[b] = o["latent"]
                    got[b] += 1
                    assert bool(r.last[b]) == (got[b] == n_frames), (b, got[b])
                    assert abs(r.eos_logits[b] - o["eos_logit"]) <= LAT_TOL
                    np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                    assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL, (b, got[b])
        assert all(got[b] == n_frames for b in range(4)), got
    finally:
        eng.close()


@pytest.mark.parametrize("back_frames", [1, 2, 4])
def test_flush_calls_drain_and_pause_rows(oracle, back_frames):
    """ptts_flush_async: a pipelined call that starts no frame. Flushes in the middle of a job
    pause every row for the call (their frames resume in order, equal to the oracle's), flushes at
    the end drain the frames already computed (frame_lag() of them deliver every row's last
    frame), and a flush right after an admission is refused."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(17)
    eng = pt.Engine(device=0, max_slots=3, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames)
    try:
        orc, lat, got, vs, ids_l, want = {}, {}, {}, [], [], {0: 5, 1: 7, 2: 6}
        for b in range(3):
            F = 5 + 3 * b
            prompt = (d["prompt"][:F] * (1.0 + 0.04 * b)).astype(np.float32)
            ids = rng.integers(0, 4000, size=4 + b).astype(np.int32)
            vs.append(eng.voice_from_prompt(prompt))
            ids_l.append(ids)
            s = oracle.new_state(256)
            s.prefill(prompt)
            s.prefill_tokens(ids)
            orc[b], lat[b], got[b] = s, None, 0
        eng.open_many([0, 1, 2], vs, ids_l, [params(max_frames=want[b]) for b in range(3)])
        with pytest.raises(pt.PocketTTSError):
            eng.flush_async(3)  # the admitted rows' first frame must fall on a step call

        def check(r):
            for b in range(3):
                if not r.valid[b]:
                    continue
                o = orc[b].step(lat[b])
                lat[b] = o["latent"]
                got[b] += 1
                assert got[b] <= want[b] and bool(r.last[b]) == (got[b] == want[b]), (b, got[b])
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL, (b, got[b])

        # steps and flushes interleaved (two flushes in a row: with frame pairs an even-call flush
        # makes the odd call one too), then the drain
        for kind in "ssffsssfsss":
            (eng.step_async if kind == "s" else eng.flush_async)(3)
            check(eng.fetch(3))
        lag, _ = eng.frame_lag()
        for _ in range(lag):
            eng.flush_async(3)
            check(eng.fetch(3))
        assert got == want, got
    finally:
        eng.close()


def test_long_utterance_wraps_mimi_ring(gpu_engine, oracle):
    """70 frames: the Mimi decoder ring (512 positions = 32 frames) wraps twice and the 250-key
    window slides across the wrap; the FlowLM cache grows to voice + text + 70 positions. Every
    frame must match the oracle (temp 0; the backbone input is teacher-forced to the oracle's
    latent so that per-step differences do not compound through the autoregression)."""
    d = load_golden("e2e_lsd1.safetensors")
    v = gpu_engine.voice_from_prompt(d["prompt"])
    n = 70
    gpu_engine.open(0, v, d["text_ids"], params(max_frames=n))
    s = oracle.new_state(256)
    s.prefill(d["prompt"])
    s.prefill_tokens(d["text_ids"])
    lat = None
    worst = 0.0
    for i in range(n):
        r = gpu_engine.step(1)
        o = s.step(lat)
        lat = o["latent"]
        assert r.valid[0] and r.last[0] == (i == n - 1)
        np.testing.assert_allclose(r.latents[0], o["latent"], atol=LAT_TOL)
        worst = max(worst, pcm_err(r.pcm[0] - o["pcm"]))
        gpu_engine.set_latent(0, o["latent"])  # teacher forcing: no drift over 70 AR steps
    assert worst <= PCM_TOL, worst


@pytest.mark.parametrize("back_frames", [1, 2, 4])
def test_batch_scheduler_matches_oracle(oracle, back_frames):
    """Serving front end (f1) on the real pipelined engine: 6 requests of different lengths through
    3 slots (continuous admission into recycled slots); every request's audio equals its own
    oracle run."""
    import pocket_tts_amd as pt
    from pocket_tts_amd.serve import BatchScheduler

    d = load_golden("e2e_lsd1.safetensors")
    eng = pt.Engine(device=0, max_slots=3, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames)
    sch = BatchScheduler(eng)
    try:
        rng = np.random.default_rng(3)
        jobs = []
        for u in range(6):
            F = 4 + u
            prompt = (d["prompt"][:F] * (1.0 + 0.03 * u)).astype(np.float32)
            ids = rng.integers(0, 4000, size=2 + 3 * u).astype(np.int32)
            n = 2 + u % 3
            v = eng.voice_from_prompt(prompt)
            jobs.append((prompt, ids, n, v))
        reqs = [sch.submit(ids, v, params(max_frames=n)) for _, ids, n, v in jobs]
        for (prompt, ids, n, _), req in zip(jobs, reqs):
            frames = list(req.stream(timeout=120))
            assert len(frames) == n
            s = oracle.new_state(128)
            s.prefill(prompt)
            s.prefill_tokens(ids)
            lat = None
            for f in frames:
                o = s.step(lat)
                lat = o["latent"]
                assert pcm_err(f - o["pcm"]) <= PCM_TOL
    finally:
        sch.close()
        eng.close()


@pytest.mark.parametrize("B,lsd", [(20, 1), (20, 3), (45, 1), (128, 1)])
def test_flow_head_chain_two_row_groups(oracle, B, lsd):
    """B = 20: the persistent flow-head launch (k_flow_head) runs two 16-row groups, the second
    ragged (4 valid rows); B = 45 three (the XCD-aware block -> (row group, column group) map with
    an odd group count, 13 valid rows in the last), B = 128 its largest grid (8 groups, 256
    workgroups; sampled rows). The launch is first replayed alone in a timing loop, which must
    leave its hand-off counters re-armed; then every checked row of every step equals its oracle
    run."""
    import pocket_tts_amd as pt
    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(11)
    steps = 3
    rows = range(B) if B <= 48 else [0, 15, 16, 63, 64, 100, 127]
    eng = pt.Engine(device=0, max_slots=B, max_ctx=64, lsd_decode_steps=lsd, seed=0x5EED)
    try:
        assert "head.chain" in eng.plan_ops(B)
        orc = {}
        for b in range(B):
            F = 3 + (b % 5)
            prompt = (d["prompt"][:F] * (1.0 + 0.05 * b)).astype(np.float32)
            ids = rng.integers(0, 4000, size=2 + b % 3).astype(np.int32)
            eng.open(b, eng.voice_from_prompt(prompt), ids, params(max_frames=steps))
            if b in rows:
                s = oracle.new_state(64)
                s.prefill(prompt)
                s.prefill_tokens(ids)
                orc[b] = s
        assert eng.time_kernel(B, "head.chain", reps=20) > 0
        lat = [None] * B
        for i in range(steps):
            r = eng.step(B)
            assert r.valid.all()
            for b in rows:
                o = orc[b].step(lat[b], lsd_steps=lsd)
                lat[b] = o["latent"]
                assert r.valid[b]
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL
    finally:
        eng.close()


def test_large_batch_uses_multi_launch_head(oracle):
    """B = 136 exceeds the persistent flow-head launch's 128 rows: the head runs as split-K GEMM
    + row-reduce launches. Sampled rows in the first, middle and last 16-row groups (with their
    own prompts and texts) equal their oracle runs."""
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(5)
    B, steps, probe = 136, 2, (0, 70, 135)
    eng = pt.Engine(device=0, max_slots=B, max_ctx=32, lsd_decode_steps=1, seed=0x5EED)
    try:
        assert "head.chain" not in eng.plan_ops(B) and "head.chain" in eng.plan_ops(128)
        base = eng.voice_from_prompt(d["prompt"][:3])
        orc = {}
        for b in range(B):
            if b in probe:
                prompt = (d["prompt"][:4] * (1.0 + 0.1 * probe.index(b))).astype(np.float32)
                ids = rng.integers(0, 4000, size=3).astype(np.int32)
                eng.open(b, eng.voice_from_prompt(prompt), ids, params(max_frames=steps))
                s = oracle.new_state(32)
                s.prefill(prompt)
                s.prefill_tokens(ids)
                orc[b] = s
            else:
                eng.open(b, base, np.array([260, 261], np.int32), params(max_frames=steps))
        lat = {b: None for b in probe}
        for _ in range(steps):
            r = eng.step(B)
            for b in probe:
                o = orc[b].step(lat[b])
                lat[b] = o["latent"]
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - o["pcm"]) <= PCM_TOL
    finally:
        eng.close()
