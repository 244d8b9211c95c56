"""The reference's own data fixtures on the GPU: configs[4] (voice cloning on assets/ref.wav with
the int8-quantised FlowLM and the fp8 MFMA path) and the kernel-level decode seam.

Pinning:
  * assets/ref.wav -> assets/ref_mimi_input (tests/golden/ref_voice.safetensors, both whole
    files): the reference's own resampler pair (test_input_parity, parity_tests.rs:378-433);
  * the voice conditioning and the generation from it against the C oracle (pinned to the
    reference's Python modules by tests/test_oracle.py), with the same weights: synthetic, the
    gated checkpoint being unavailable offline;
  * with a real checkpoint (env PTTS_WEIGHTS = path of tts_b6369a24.safetensors), the
    reference's real-weight fixtures: test_decoder_parity (parity_tests.rs:520-612, tolerances
    0.05 / 0.05 / 0.1) and test_voice_conditioning_parity (parity_tests.rs:59-142, 2e-2).
    Without it those two tests skip, as the reference's own do (parity_tests.rs:62-65)."""

import os

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err

pytestmark = pytest.mark.gpu
INF = float("inf")


def _params(**kw):
    import pocket_tts_amd as pt

    base = dict(temp=0.0, eos_threshold=INF, max_frames=6, seed=1)
    base.update(kw)
    return pt.GenerationParams(**base)


def _refwav():
    g = load_golden("ref_voice.safetensors")
    return g["refwav_i16"].astype(np.float32) / np.float32(32768.0), g["ref_mimi_input"]


def test_decode_latents_matches_reference_golden(gpu_engine):
    """ptts_decode_latents (MimiModel::decode_from_latent seam) on the golden e2e latents: the
    quantizer output, the upsample, the decoder transformer and the PCM of the reference's own
    Python run (gen_golden.py), frame by frame on one streaming state."""
    d = load_golden("e2e_lsd1.safetensors")
    out = gpu_engine.decode_latents(5, d["latent"])
    for i in range(d["latent"].shape[0]):
        if i < d["quantized"].shape[0]:
            np.testing.assert_allclose(out["quantized"][i], d["quantized"][i], atol=2e-5)
            np.testing.assert_allclose(out["after_upsample"][i].T, d["after_upsample"][i], atol=2e-5)
            np.testing.assert_allclose(out["after_transformer"][i].T, d["after_decoder_transformer"][i], atol=2e-5)
        assert pcm_err(out["pcm"][i] - d["pcm"][i]) <= PCM_TOL, i


def test_refwav_voice_cloning_int8_and_fp8_engines(oracle):
    """configs[4] end to end on the reference's ref.wav (48 kHz, 331,708 samples): GPU resample
    == the reference's ref_mimi_input; GPU encode (87 frames, one chunk by the Rust rule) ==
    the oracle's; then generation from that voice on the int8-FlowLM engine (== the quantized
    oracle, fp32 gates) and on the fp8 W8A8 engine (accuracy gates of tests/test_fp8.py against
    the f32 oracle)."""
    import pocket_tts_amd as pt
    from _oracle import Oracle

    x48, mimi_in = _refwav()
    ids = load_golden("e2e_lsd1.safetensors")["text_ids"]
    pad = np.zeros(87 * 1920, np.float32)
    pad[:mimi_in.size] = mimi_in
    eng = pt.Engine(device=0, max_slots=2, max_ctx=160, seed=0x5EED, weight_quant=pt.QUANT_FLOW_LM, pipeline=True)
    try:
        y = eng.resample(x48, 48000)  # ref_mimi_input is the resampled signal zero-padded to 87 frames
        assert y.size == 165854 and np.abs(y - mimi_in[:y.size]).max() <= 1e-6 and not mimi_in[y.size:].any()
        v = eng.voice_from_audio(x48, 48000)
        assert v.n_frames == 87
        oq = Oracle(0x5EED, 1)
        cond, _, _, _ = oq.encode(pad, 87)
        np.testing.assert_allclose(v.conditioning(), cond, atol=1e-5)
        eng.open(1, v, ids, _params())
        s = oq.new_state(160)
        s.prefill(cond)
        s.prefill_tokens(ids)
        assert not eng.step(2).valid.any()
        lat = None
        for i in range(6):
            r = eng.step(2)
            ref = s.step(lat)
            lat = ref["latent"]
            assert r.valid[1] and not r.valid[0]
            assert abs(r.eos_logits[1] - ref["eos_logit"]) <= LAT_TOL
            np.testing.assert_allclose(r.latents[1], ref["latent"], atol=LAT_TOL)
            assert pcm_err(r.pcm[1] - ref["pcm"]) <= PCM_TOL, i
    finally:
        eng.close()

    def snr(x, ref):
        ref = np.asarray(ref, np.float64)
        return 10 * np.log10(np.sum(ref ** 2) / max(np.sum((np.asarray(x, np.float64) - ref) ** 2), 1e-300))

    ef = pt.Engine(device=0, max_slots=1, max_ctx=160, seed=0x5EED, fp8_gemm=True)
    try:
        v = ef.voice_from_audio(x48, 48000)
        cond32, _, _, _ = oracle.encode(pad, 87)
        np.testing.assert_allclose(v.conditioning(), cond32, atol=1e-5)  # the encoder stays f32
        ef.open(0, v, ids, _params())
        s = oracle.new_state(160)
        s.prefill(cond32)
        s.prefill_tokens(ids)
        lat, got, ref_l, ref_p = None, [], [], []
        for i in range(6):
            r = ef.step(1)
            ref = s.step(lat)
            lat = ref["latent"]  # f32 oracle free-running; the fp8 engine runs on its own latents
            got.append((r.latents[0].copy(), r.pcm[0].copy()))
            ref_l.append(ref["latent"])
            ref_p.append(ref["pcm"])
        assert snr([g[0] for g in got], ref_l) >= 15.0
        assert snr([g[1] for g in got], ref_p) >= 30.0
    finally:
        ef.close()


@pytest.fixture(scope="module")
def real_engine():
    path = os.environ.get("PTTS_WEIGHTS")
    if not path or not os.path.exists(path):
        pytest.skip("real checkpoint not present (set PTTS_WEIGHTS=path/to/tts_b6369a24.safetensors)")
    import pocket_tts_amd as pt

    eng = pt.Engine(device=0, max_slots=1, max_ctx=256, seed=0, weights_path=path)
    yield eng
    eng.close()


def test_decoder_parity_real_weights(real_engine):
    """parity_tests.rs test_decoder_parity on assets/ref_decoder_intermediates.safetensors."""
    r = load_golden("ref_decoder_intermediates.safetensors")
    out = real_engine.decode_latents(0, r["latent_from_flowlm"].reshape(1, 32))
    np.testing.assert_allclose(out["quantized"][0], r["quantized"][0, :, 0], atol=2e-2)
    np.testing.assert_allclose(out["after_upsample"][0].T, r["after_upsample"][0], atol=0.05)
    np.testing.assert_allclose(out["after_transformer"][0].T, r["after_decoder_transformer"][0], atol=0.05)
    np.testing.assert_allclose(out["pcm"][0], r["final_audio"][0, 0], atol=0.1)


def test_voice_conditioning_parity_real_weights(real_engine):
    """parity_tests.rs test_voice_conditioning_parity: ref.wav -> conditioning [87, 1024]."""
    x48, _ = _refwav()
    v = real_engine.voice_from_audio(x48, 48000)
    ref = load_golden("ref_voice_conditioning.safetensors")["voice_conditioning"][0]
    assert v.n_frames == ref.shape[0]
    np.testing.assert_allclose(v.conditioning(), ref, atol=2e-2)
