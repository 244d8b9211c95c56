"""Voice-cloning front end: WAV I/O, the resampler, the chunked
encoder and the whole WAV -> voice path.

Pinning:
  * resampler: the reference's own real-data pair, assets/ref.wav -> assets/ref_mimi_input
    (test_input_parity, parity_tests.rs:379-433; the head is committed in
    tests/golden/resample.safetensors, and the full pair is checked when /root/reference is
    present), plus synthetic signals through the Python reference's convert_audio at 5 rates;
  * chunked encode: the reference's Python streaming modules driven the way the Rust driver
    chunks (gen_golden.py:run_encoder_chunked).
Tolerances: resampler 1e-6 abs (f64 accumulation here vs scipy's f32 upfirdn); encoder
conditioning 1e-5 abs (fp32, reduction order only).

The Rust driver's own resampler (rubato 0.14.1 FastFixedIn / Septic, audio.rs:197-255) is an
option ("rubato"): its source is not in the reference and no fixture of it exists, so its parity
is UNPINNED. The oracle's restatement is checked against properties of the published algorithm
(the f64 position walk and its output count, exact reproduction of degree-7 polynomials, a band-
limited tone at the walk's positions), and the GPU kernel against the oracle bit for bit."""

import struct
from pathlib import Path

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err

REF_ASSETS = Path("/root/reference/assets")
RATES = (48000, 44100, 16000, 22050, 8000)


# ------------------------------------------------------------------ WAV I/O (audio.rs:12-185)
def test_pcm_i16_interleave_and_clamp():
    """audio.rs test_pcm_i16_le_bytes_clamp_and_interleave (audio.rs:242-259)."""
    from pocket_tts_amd.audio import pcm_i16_le_bytes

    t = np.array([[-1.0, 0.0, 1.0], [0.5, -0.5, 2.0]], np.float32)
    got = np.frombuffer(pcm_i16_le_bytes(t), "<i2").tolist()
    assert got == [-32767, 16383, 0, -16383, 32767, 32767]


def test_normalize_peak():
    """audio.rs test_normalize_peak (audio.rs:230-239)."""
    from pocket_tts_amd.audio import normalize_peak

    assert normalize_peak(np.array([[-0.5, 0.2, 0.5]], np.float32)).tolist() == [[-1.0, np.float32(0.4), 1.0]]
    assert normalize_peak(np.zeros((1, 3), np.float32)).tolist() == [[0.0, 0.0, 0.0]]


def test_wav_roundtrip(tmp_path):
    """audio.rs test_wav_io (audio.rs:289-312): 16-bit write then read within 1e-3."""
    from pocket_tts_amd.audio import read_wav, write_wav

    t = np.array([[0.0, 0.5, -0.5, 0.1]], np.float32)
    write_wav(tmp_path / "io.wav", t, 16000)
    x, sr = read_wav(tmp_path / "io.wav")
    assert sr == 16000 and x.shape == (1, 4)
    assert np.abs(x - t).max() < 1e-3


def _riff(fmt_tag, ch, sr, bits, payload, extensible=False, declared=None):
    align = ch * bits // 8
    if extensible:
        fmt = struct.pack("<HHIIHH", 0xFFFE, ch, sr, sr * align, align, bits)
        fmt += struct.pack("<HHI", 22, bits, 0) + struct.pack("<H", fmt_tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
    else:
        fmt = struct.pack("<HHIIHH", fmt_tag, ch, sr, sr * align, align, bits)
    body = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    body += b"LIST" + struct.pack("<I", 3) + b"abc\x00"  # odd-sized chunk: word-aligned skip
    body += b"data" + struct.pack("<I", declared if declared is not None else len(payload)) + payload
    return b"RIFF" + struct.pack("<I", 4 + len(body)) + b"WAVE" + body


@pytest.mark.parametrize("bits", [8, 16, 24, 32])
def test_read_wav_int_formats(bits):
    """hound semantics: integer samples / 2^(bits-1), 8-bit stored unsigned; channels
    de-interleaved to [C, T]."""
    from pocket_tts_amd.audio import read_wav_from_bytes

    rng = np.random.default_rng(bits)
    full = 1 << (bits - 1)
    v = rng.integers(-full, full, size=(5, 2), dtype=np.int64)
    if bits == 8:
        payload = (v + 128).astype(np.uint8).tobytes()
    else:
        w = bits // 8
        payload = b"".join(int(s).to_bytes(w, "little", signed=True) for s in v.reshape(-1))
    for ext in (False, True):
        x, sr = read_wav_from_bytes(_riff(1, 2, 22050, bits, payload, extensible=ext))
        assert sr == 22050 and x.shape == (2, 5)
        np.testing.assert_array_equal(x, (v.T.astype(np.float32) / np.float32(full)))


def test_read_wav_float_and_truncated():
    from pocket_tts_amd.audio import WavError, read_wav_from_bytes

    f = np.array([0.25, -0.75, 1.5], np.float32)
    x, _ = read_wav_from_bytes(_riff(3, 1, 24000, 32, f.tobytes()))
    np.testing.assert_array_equal(x[0], f)
    # data chunk declared longer than the file: the whole samples present are kept (audio.rs:33-49)
    s16 = np.array([100, -200, 300], "<i2").tobytes() + b"\x01"
    x, _ = read_wav_from_bytes(_riff(1, 1, 24000, 16, s16, declared=1000))
    np.testing.assert_array_equal(x[0], np.array([100, -200, 300], np.float32) / 32768.0)
    with pytest.raises(WavError):
        read_wav_from_bytes(b"RIFX0000WAVE")
    with pytest.raises(WavError):
        read_wav_from_bytes(_riff(2, 1, 24000, 16, s16))  # ADPCM: unsupported


def test_read_reference_wav():
    """The reference's own assets/ref.wav: 48 kHz mono s16, 331,708 samples."""
    if not (REF_ASSETS / "ref.wav").exists():
        pytest.skip("reference assets not present")
    from pocket_tts_amd.audio import read_wav

    x, sr = read_wav(REF_ASSETS / "ref.wav")
    g = load_golden("resample.safetensors")
    assert sr == 48000 and x.shape == (1, int(g["ref_lengths"][0]))
    np.testing.assert_array_equal(x[0, :24064], g["refwav_head_i16"].astype(np.float32) / 32768.0)


# ------------------------------------------------------------------ oracle pinning (CPU)
def test_oracle_resample_matches_reference_convert_audio():
    from _oracle import resample

    g = load_golden("resample.safetensors")
    for sr in RATES:
        y = resample(g[f"x_{sr}"], sr)
        assert y.shape == g[f"y_{sr}"].shape, sr
        assert np.abs(y - g[f"y_{sr}"]).max() <= 1e-6, sr


def test_oracle_resample_matches_reference_ref_wav_pair():
    """assets/ref.wav -> assets/ref_mimi_input (the reference's real-data resampler pair)."""
    from _oracle import resample

    g = load_golden("resample.safetensors")
    x = g["refwav_head_i16"].astype(np.float32) / 32768.0
    y = resample(x, 48000)[:12000]
    assert np.abs(y - g["ref_mimi_input_head"]).max() <= 1e-6
    if (REF_ASSETS / "ref_mimi_input.safetensors").exists():  # the whole file, when present
        import wave

        from safetensors.numpy import load_file

        with wave.open(str(REF_ASSETS / "ref.wav"), "rb") as w:
            xs = np.frombuffer(w.readframes(w.getnframes()), np.int16).astype(np.float32) / 32768.0
        m = load_file(str(REF_ASSETS / "ref_mimi_input.safetensors"))["mimi_input"].reshape(-1)
        y = resample(xs, 48000)
        assert np.abs(y - m[:y.size]).max() <= 1e-6 and not m[y.size:].any()
        assert m.size == (y.size + 1919) // 1920 * 1920


def _septic_positions(n, sr_from, sr_to=24000):
    """rubato FastFixedIn's read positions, restated in numpy: from -4, + sr_from / sr_to per
    output (f64, left to right: np.cumsum adds sequentially), while the position before the step
    is < n - 9."""
    t = 1.0 / (sr_to / sr_from)
    m = int((n - 9 + 4) / t) + 3
    walk = np.cumsum(np.concatenate([[-4.0], np.full(m, t)]))
    cnt = int(np.argmax(walk >= n - 9)) if (walk >= n - 9).any() else m
    return walk[1:cnt + 1]


@pytest.mark.parametrize("sr", RATES + (96000, 24000))
def test_oracle_septic_resampler_walk_and_length(sr):
    from _oracle import resample_septic

    for n in (10, 11, 37, 4000, 48001):
        y = resample_septic(np.zeros(n, np.float32), sr)
        if sr == 24000:
            assert y.size == n  # equal rates: the input unchanged (audio.rs:198-200)
            continue
        assert y.size == _septic_positions(n, sr).size, (sr, n)
        assert abs(y.size - (n - 5) * 24000 / sr) <= 1.0 + 24000 / sr


@pytest.mark.parametrize("sr", RATES)
def test_oracle_septic_resampler_reproduces_polynomials(sr):
    """An 8-point septic reproduces every polynomial of degree <= 7 at the read positions whose
    window lies inside the input (f32 rounding apart)."""
    from _oracle import resample_septic

    n = 3000
    rng = np.random.default_rng(sr)
    c = rng.uniform(-1, 1, 8)
    p = lambda u: sum(c[i] * ((u - n / 2) / n) ** i for i in range(8))  # noqa: E731
    y = resample_septic(p(np.arange(n, dtype=np.float64)).astype(np.float32), sr)
    pos = _septic_positions(n, sr)
    inner = (np.floor(pos) >= 3) & (np.floor(pos) + 4 < n)
    assert inner.sum() > 0.9 * y.size
    assert np.abs(y[inner] - p(pos[inner])).max() <= 2e-5


@pytest.mark.parametrize("sr", RATES)
def test_oracle_septic_resampler_tone_at_walk_positions(sr):
    """A 300-Hz tone comes out as the tone sampled at the walk's positions (rubato's output is not
    delay-compensated: output m is the input at -4 + (m + 1) sr / 24000 samples)."""
    from _oracle import resample_septic

    n = 4000
    x = np.sin(2 * np.pi * 300 * np.arange(n) / sr).astype(np.float32)
    y = resample_septic(x, sr)
    pos = _septic_positions(n, sr)
    inner = (pos > 4) & (pos < n - 5)
    assert np.abs(y[inner] - np.sin(2 * np.pi * 300 * pos[inner] / sr)).max() <= 1e-6


def test_resampler_choice_over_the_boundary():
    """ptts_resample_len_ex (host-only: no GPU call) agrees with the oracle for both rules."""
    from _oracle import lib as olib

    from pocket_tts_amd import engine
    from pocket_tts_amd._lib import lib

    for sr in RATES + (24000,):
        for n in (1, 50, 331708):
            assert lib().ptts_resample_len_ex(n, sr, 24000, 0) == olib().orc_resample_len(n, sr, 24000), (sr, n)
            assert lib().ptts_resample_len_ex(n, sr, 24000, 1) == olib().orc_resample_septic_len(n, sr, 24000), (sr, n)
    assert lib().ptts_resample_len_ex(100, 48000, 24000, 7) == 0
    with pytest.raises(ValueError):
        engine.resampler_code("sinc")


def test_oracle_chunked_encoder_matches_reference():
    from _oracle import Oracle

    d = load_golden("encoder_chunked_5f.safetensors")
    o = Oracle(0x5EED)
    cond, _, _, lat = o.encode(d["pcm"], int(d["meta"][2]))
    assert np.abs(lat - d["latent"].T).max() <= 1e-5
    assert np.abs(cond - d["conditioning"]).max() <= 1e-5
    _, _, _, lat1 = o.encode(d["pcm"], -1)
    assert np.abs(lat1 - d["latent_one_pass"].T).max() <= 1e-5
    # the quirk is real: chunk-start frames 2 and 4 differ from the one-pass encode, others do not
    per_frame = np.abs(d["latent"] - d["latent_one_pass"]).max(axis=0)
    assert per_frame[[2, 4]].min() > 1e-3 and per_frame[[0, 1, 3]].max() < 1e-6


# ------------------------------------------------------------------ GPU (through the C ABI)
@pytest.mark.gpu
def test_gpu_resampler_matches_oracle_and_reference(gpu_engine):
    from _oracle import resample

    g = load_golden("resample.safetensors")
    for sr in RATES:
        y = gpu_engine.resample(g[f"x_{sr}"], sr)
        assert y.shape == g[f"y_{sr}"].shape, sr
        assert np.abs(y - resample(g[f"x_{sr}"], sr)).max() <= 1e-7, sr
        assert np.abs(y - g[f"y_{sr}"]).max() <= 1e-6, sr
    x = g["refwav_head_i16"].astype(np.float32) / 32768.0
    assert np.abs(gpu_engine.resample(x, 48000)[:12000] - g["ref_mimi_input_head"]).max() <= 1e-6
    # 10 s at 44.1 kHz (a long, non-trivial ratio: up 80, down 147, 2941 taps)
    x = (0.3 * np.sin(np.arange(441000) * 0.01)).astype(np.float32)
    y = gpu_engine.resample(x, 44100)
    assert y.size == 240000 and np.abs(y - resample(x, 44100)).max() <= 1e-7


@pytest.mark.gpu
def test_gpu_rubato_resampler_matches_oracle(gpu_engine):
    """The Rust driver's resampler option on the GPU against the oracle's restatement: bit for bit
    (same f32 operations in the same order, same host position walk); parity with rubato itself is
    unpinned (no fixture)."""
    from _oracle import resample_septic

    g = load_golden("resample.safetensors")
    for sr in RATES:
        x = g[f"x_{sr}"]
        r = resample_septic(x, sr)
        if r.size == 0:  # x_8000 is one sample: rubato's walk yields nothing, the engine rejects it
            with pytest.raises(Exception):
                gpu_engine.resample(x, sr, resampler="rubato")
            continue
        y = gpu_engine.resample(x, sr, resampler="rubato")
        assert y.shape == r.shape, sr
        np.testing.assert_array_equal(y, r)
    x = (0.3 * np.sin(np.arange(441000) * 0.01)).astype(np.float32)  # 10 s at 44.1 kHz
    np.testing.assert_array_equal(gpu_engine.resample(x, 44100, resampler="rubato"), resample_septic(x, 44100))
    np.testing.assert_array_equal(gpu_engine.resample(x[:1000], 24000, resampler="rubato"), x[:1000])
    with pytest.raises(Exception):
        gpu_engine.resample(x[:4], 48000, resampler="rubato")  # the walk yields no sample: rejected


@pytest.mark.gpu
def test_gpu_rubato_voice_path_matches_oracle_resample(gpu_engine):
    """voice_from_audio with the rubato rule == the oracle's rubato output encoded at 24 kHz."""
    from _oracle import resample_septic

    x = (0.2 * np.random.default_rng(3).standard_normal(48000 * 2)).astype(np.float32)
    v = gpu_engine.voice_from_audio(x, 48000, -1, resampler="rubato")
    w = gpu_engine.voice_from_audio(resample_septic(x, 48000), 24000, -1)
    assert v.n_frames == w.n_frames
    np.testing.assert_array_equal(v.conditioning(), w.conditioning())
    p = gpu_engine.voice_from_audio(x, 48000, -1)  # the default rule differs (a different resampler)
    assert np.abs(p.conditioning() - v.conditioning()).max() > 1e-4
    for a in (v, w, p):
        a.close()


@pytest.mark.gpu
def test_gpu_chunked_voice_matches_reference(gpu_engine):
    d = load_golden("encoder_chunked_5f.safetensors")
    v = gpu_engine.voice_from_audio(d["pcm"], 24000, int(d["meta"][2]))
    assert v.n_frames == 5
    np.testing.assert_allclose(v.conditioning(), d["conditioning"], atol=1e-5)
    v1 = gpu_engine.voice_from_audio(d["pcm"], 24000, -1)  # one pass = the Python reference
    e = load_golden("encoder_4f.safetensors")
    v4 = gpu_engine.voice_from_audio(e["pcm"], 24000, 0)  # adaptive rule: 4 frames -> one chunk
    np.testing.assert_allclose(v4.conditioning(), e["conditioning"], atol=1e-5)
    for x in (v, v1, v4):
        x.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_frames,chunk", [(125, 120), (750, 180)])
def test_gpu_long_voice_prompt_chunked_matches_oracle(oracle, n_frames, chunk):
    """Voice prompts past one chunk through the adaptive chunked encoder (tts_model.rs:530-577:
    120-frame chunks up to 600 frames, 180 up to 1800): a 10-s prompt (125 frames = 120 + 5, the
    bench's prompt length) and a 60-s one (750 frames = 4 x 180 + 30, the reference's stress test,
    tests/memory_usage.rs:7-39). Every chunk re-applies the downsample's replicate pad (the
    quirk), so the conditioning must equal the oracle's encode with the same
    chunking; then 4 generated frames from that voice against the oracle."""
    import pocket_tts_amd as pt

    pcm = (0.1 * np.random.default_rng(n_frames).standard_normal(n_frames * 1920)).astype(np.float32)
    eng = pt.Engine(device=0, max_slots=1, max_ctx=n_frames + 64, lsd_decode_steps=1, seed=0x5EED)
    try:
        v = eng.voice_from_audio(pcm, 24000, 0)  # adaptive rule
        assert v.n_frames == n_frames
        cond, _, _, _ = oracle.encode(pcm, chunk)
        err = float(np.abs(v.conditioning() - cond).max())
        assert err <= 2e-5, err
        # the quirk is exercised: the one-pass encode differs at the chunk starts
        one, _, _, _ = oracle.encode(pcm, -1)
        assert np.abs(one[chunk] - cond[chunk]).max() > 1e-4
        ids = np.array([260, 2994, 262, 578, 682], np.int32)
        eng.open(0, v, ids, pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=4))
        s = oracle.new_state(n_frames + 64)
        s.prefill(cond)
        s.prefill_tokens(ids)
        lat = None
        for i in range(4):
            r = eng.step(1)
            ref = s.step(lat)
            lat = ref["latent"]
            assert r.valid[0]
            np.testing.assert_allclose(r.latents[0], ref["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[0] - ref["pcm"]) <= PCM_TOL, i
        v.close()
        print(f"{n_frames}-frame prompt ({chunk}-frame chunks): conditioning max |d| {err:.3g}")
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_wav_voice_path_matches_oracle(gpu_engine, oracle, tmp_path):
    """WAV at 48 kHz -> read_wav -> GPU resample + encode, vs oracle resample + chunked encode,
    then a generation step from that voice on both sides."""
    import pocket_tts_amd as pt
    from _oracle import resample
    from pocket_tts_amd.audio import read_wav, write_wav

    rng = np.random.default_rng(3)
    x48 = (0.2 * rng.standard_normal(3 * 3840 + 77)).astype(np.float32)
    write_wav(tmp_path / "v.wav", x48[None], 48000)
    xr, sr = read_wav(tmp_path / "v.wav")
    v = gpu_engine.voice_from_audio(xr[0], sr, 2)
    y = resample(xr[0], sr)
    pad = np.zeros((y.size + 1919) // 1920 * 1920, np.float32)
    pad[:y.size] = y
    cond, _, _, _ = oracle.encode(pad, 2)
    assert v.n_frames == cond.shape[0] == 4
    np.testing.assert_allclose(v.conditioning(), cond, atol=1e-5)
    ids = np.array([260, 2994, 262], np.int32)
    gpu_engine.open(0, v, ids, pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=2))
    s = oracle.new_state(64)
    s.prefill(cond)
    s.prefill_tokens(ids)
    r = gpu_engine.step(1)
    ref = s.step(None)
    np.testing.assert_allclose(r.latents[0], ref["latent"], atol=LAT_TOL)
    gpu_engine.close_slot(0)
    v.close()


@pytest.mark.gpu
def test_gpu_voice_errors(gpu_engine):
    from pocket_tts_amd import PocketTTSError

    with pytest.raises(PocketTTSError):
        gpu_engine.voice_from_audio(np.zeros(100, np.float32), 0)
    with pytest.raises(PocketTTSError):
        gpu_engine.voice_from_audio(np.zeros(1920 * 600, np.float32), 24000)  # > max_ctx frames


def test_oracle_resample_matches_whole_reference_pair():
    """The whole assets/ref.wav -> assets/ref_mimi_input pair (tests/golden/ref_voice.safetensors):
    the oracle's resample_poly restatement equals the reference's convert_audio output, which the
    reference zero-pads to whole frames (87 x 1920)."""
    from _oracle import resample

    g = load_golden("ref_voice.safetensors")
    x = g["refwav_i16"].astype(np.float32) / np.float32(32768.0)
    y = resample(x, 48000)
    mi = g["ref_mimi_input"]
    assert x.size == 331708 and y.size == 165854 and mi.size == 87 * 1920
    assert np.abs(y - mi[:y.size]).max() <= 1e-6 and not mi[y.size:].any()
