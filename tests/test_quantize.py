"""Weight quantization (BASELINE configs[4]): the reference's quantize.rs.

Pinning. quantize.rs is Rust-only (the Python reference has no weight quantizer) and cannot be
built here, so the restatements - the engine's C++ (`ptts_quantize_tensor`, used when packing),
the oracle's C (`orc_quantize`) and a numpy statement in this file - are pinned by the
reference's own unit tests (quantize.rs:170-219, restated below with their thresholds) and by
agreeing bit for bit with each other. End to end, a quantized engine (int8 codes streamed by
the FlowLM step GEMMs) must equal the oracle built with the same quantized weights within the
fp32 gates of test_gpu_parity (latent / eos <= LAT_TOL, PCM <= PCM_TOL max abs): the codes rebuild
exactly the f32 values the reference's simulated quantization holds."""

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err, rms

import _oracle


def np_quantize(x, num_levels=256):
    """quantize.rs:66-90 in numpy f32: round half away from zero (Rust f32::round)."""
    x = np.asarray(x, np.float32)
    amax = np.float32(np.abs(x).max()) if x.size else np.float32(0)
    half = np.float32(num_levels // 2)
    scale = amax / (half - np.float32(1)) if amax > 0 else np.float32(1)
    y = x / scale
    t = np.trunc(y)
    q = np.where(np.abs(y - t) >= np.float32(0.5), t + np.sign(y), t).astype(np.float32)
    q = np.clip(q, -(half - 1), half - 1).astype(np.float32)
    return (q * scale).astype(np.float32), float(scale)


# ---------------------------------------------------------------- the reference's own tests
def test_reference_quantize_tensor():
    """quantize.rs:175-186 test_quantize_tensor: SNR > 30 dB on a 5-element tensor."""
    from pocket_tts_amd import QuantizedTensor, calculate_snr

    t = np.array([1.0, 2.0, -3.0, 4.5, -2.1], np.float32)
    q = QuantizedTensor.quantize(t, 256)
    assert calculate_snr(t, q.data) > 30.0
    assert q.zero_point == 0.0 and q.num_levels == 256
    np.testing.assert_allclose(q.scale, 4.5 / 127.0, rtol=1e-7)


def test_reference_quantize_large_tensor():
    """quantize.rs:188-200 test_quantize_large_tensor: sin(i * 0.01) * 10, SNR > 30 dB."""
    from pocket_tts_amd import QuantizedTensor, calculate_snr

    t = (np.sin(np.arange(10000, dtype=np.float32) * np.float32(0.01)) * np.float32(10.0)).astype(np.float32)
    q = QuantizedTensor.quantize(t, 256)
    assert calculate_snr(t, q.data) > 30.0


def test_reference_skip_layers_and_savings():
    """quantize.rs:202-218 test_quantize_config_skip_layers / test_theoretical_savings."""
    from pocket_tts_amd import QuantizeConfig, QuantizedTensor
    from pocket_tts_amd.quantize import should_skip_layer

    cfg = QuantizeConfig()
    assert should_skip_layer("model.embed_tokens", cfg)
    assert should_skip_layer("decoder.out_proj", cfg)
    assert not should_skip_layer("encoder.layers.0.linear", cfg)
    q = QuantizedTensor.quantize(np.array([1.0, 2.0, 3.0], np.float32), 256)
    assert q.theoretical_memory_savings() == 4.0


# ---------------------------------------------------------------- restatements agree bit for bit
@pytest.mark.parametrize("case", ["normal", "ties", "zeros", "levels16", "single"])
def test_quantizer_restatements_bit_exact(case):
    from pocket_tts_amd import QuantizedTensor

    rng = np.random.default_rng(3)
    levels = 256
    if case == "normal":
        x = rng.standard_normal(100_000).astype(np.float32) * np.float32(0.03)
    elif case == "ties":  # exact half-way points of the grid: round half away from zero
        x = (np.arange(-300, 301, dtype=np.float32) * np.float32(0.5)).astype(np.float32)
    elif case == "zeros":
        x = np.zeros(2048, np.float32)
    elif case == "levels16":
        x = rng.uniform(-2, 2, 4096).astype(np.float32)
        levels = 16
    else:
        x = np.array([-0.75], np.float32)
    ref, sc = np_quantize(x, levels)
    q = QuantizedTensor.quantize(x, levels)
    o, osc = _oracle.quantize(x, levels)
    assert q.scale == sc == osc
    assert np.array_equal(q.data.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(o.view(np.uint32), ref.view(np.uint32))
    if case == "zeros":
        assert sc == 1.0
    if case == "ties":  # 0.5 * k / scale lands on .5 exactly for odd k when scale = 150 / 127
        codes = np.round(ref / np.float32(sc)).astype(np.int32)
        assert codes.max() == 127 and codes.min() == -127


NAMES = [
    ("flow_lm.transformer.layers.0.self_attn.in_proj.weight", 3072 * 1024, (0, 1, 1)),
    ("flow_lm.transformer.layers.3.self_attn.out_proj.weight", 1024 * 1024, (0, 0, 0)),  # skip out_proj
    ("flow_lm.transformer.layers.5.norm1.weight", 1024, (0, 1, 1)),  # == min_size: quantized
    ("flow_lm.flow_net.res_blocks.0.in_ln.weight", 512, (0, 0, 0)),  # < min_size
    ("flow_lm.flow_net.cond_embed.weight", 512 * 1024, (0, 0, 0)),  # skip embed
    ("flow_lm.flow_net.time_embed.0.mlp.0.weight", 512 * 256, (0, 0, 0)),
    ("flow_lm.conditioner.embed.weight", 4001 * 1024, (0, 0, 0)),
    ("flow_lm.out_eos.weight", 1024, (0, 1, 1)),  # "eos_head" does not match out_eos
    ("flow_lm.flow_net.res_blocks.2.adaLN_modulation.1.weight", 1536 * 512, (0, 1, 1)),
    ("mimi.decoder_transformer.transformer.layers.0.linear1.weight", 2048 * 512, (0, 0, 1)),
    ("mimi.decoder.model.0.conv.weight", 512 * 512 * 7, (0, 0, 1)),
    ("mimi.decoder_transformer.transformer.layers.1.self_attn.out_proj.weight", 512 * 512, (0, 0, 0)),
]


@pytest.mark.parametrize("name,numel,expect", NAMES)
def test_quant_selection_rule(name, numel, expect):
    """quantize_weights selection (quantize.rs:120-150) per scope: C ABI == oracle == expectation."""
    import pocket_tts_amd as pt
    from pocket_tts_amd import QuantizeConfig
    from pocket_tts_amd.quantize import should_skip_layer

    for mode in (0, 1, 2):
        want = bool(expect[mode])
        assert bool(pt.lib().ptts_quant_applies(name.encode(), numel, mode)) == want, (name, mode)
        assert _oracle.quant_applies(name, numel, mode) == want, (name, mode)
    cfg = QuantizeConfig()
    assert (numel >= cfg.min_size and not should_skip_layer(name, cfg)) == bool(expect[2])


def test_quantize_weights_dict():
    from pocket_tts_amd import quantize_weights

    rng = np.random.default_rng(1)
    w = {"a.linear.weight": rng.standard_normal((64, 64)).astype(np.float32),
         "b.out_proj.weight": rng.standard_normal((64, 64)).astype(np.float32),
         "c.bias": rng.standard_normal(16).astype(np.float32)}
    q = quantize_weights(w)
    assert q["a.linear.weight"].num_levels == 256
    assert np.array_equal(q["a.linear.weight"].data, np_quantize(w["a.linear.weight"])[0])
    for k in ("b.out_proj.weight", "c.bias"):
        assert q[k].num_levels == 0 and q[k].scale == 1.0 and np.array_equal(q[k].data, w[k])


def test_packed_blob_quantization_scopes():
    """Host packing with each scope: QUANT_FLOW_LM changes only FlowLM tensors (the blob's
    FlowLM part precedes Mimi's), QUANT_ALL changes Mimi too; the mode marker differs."""
    from pocket_tts_amd import Engine

    b0 = Engine.pack_weights(0x5EED, None, 0)
    b1 = Engine.pack_weights(0x5EED, None, 1)
    b2 = Engine.pack_weights(0x5EED, None, 2)
    d1 = np.flatnonzero(b0 != b1)
    d2 = np.flatnonzero(b0 != b2)
    assert d1.size > 0.9 * 80e6 and d2.size > d1.size
    # QUANT_ALL extends QUANT_FLOW_LM: same values wherever the FlowLM scope changed something
    assert np.array_equal(b1[d1[d1 < d2.max()]][:100000], b2[d1[d1 < d2.max()]][:100000])
    # every changed FlowLM value stays on its tensor's int8 grid: at most 255 distinct values in
    # a run of one tensor (first 1M changed floats belong to the first few FlowLM tensors)
    assert np.unique(b1[d1[:3000]]).size <= 255


# ---------------------------------------------------------------- GPU: int8 streaming engine
def _run(eng, o, prompt, ids, steps, lsd=1):
    from pocket_tts_amd import GenerationParams

    v = eng.voice_from_prompt(prompt)
    eng.open(0, v, ids, GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=steps))
    s = o.new_state(256)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    lat = None
    out = []
    for i in range(steps):
        r = eng.step(1)
        ref = s.step(lat, lsd_steps=lsd)
        lat = ref["latent"]
        out.append((r, ref))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_gpu_int8_engine_matches_quantized_oracle(mode):
    import pocket_tts_amd as pt
    from _oracle import Oracle

    d = load_golden("e2e_lsd1.safetensors")
    eng = pt.Engine(device=0, max_slots=1, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, weight_quant=mode)
    try:
        assert eng.int8_matrices == 6 * 3 + 2 + 1 + 12 + 1
        o = Oracle(0x5EED, mode)
        for i, (r, ref) in enumerate(_run(eng, o, d["prompt"], d["text_ids"], 8)):
            assert r.valid[0]
            assert abs(r.eos_logits[0] - ref["eos_logit"]) <= LAT_TOL, (i, r.eos_logits[0], ref["eos_logit"])
            np.testing.assert_allclose(r.latents[0], ref["latent"], atol=LAT_TOL)
            diff = r.pcm[0] - ref["pcm"]
            assert pcm_err(diff) <= PCM_TOL, (i, pcm_err(diff))
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_int8_batched_pipelined_matches_quantized_oracle():
    """B = 4 rows, pipelined stepping: the int8 GEMMs at M = 4 under the graph path."""
    import pocket_tts_amd as pt
    from pocket_tts_amd import GenerationParams
    from _oracle import Oracle

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(5)
    B, steps = 4, 5
    eng = pt.Engine(device=0, max_slots=B, max_ctx=256, seed=0x5EED, weight_quant=1, pipeline=True)
    o = Oracle(0x5EED, 1)
    try:
        states = []
        for b in range(B):
            prompt = (d["prompt"][: 6 + 2 * b] * (1 + 0.05 * b)).astype(np.float32)
            ids = rng.integers(0, 4000, size=3 + b).astype(np.int32)
            eng.open(b, eng.voice_from_prompt(prompt), ids,
                     GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=steps))
            s = o.new_state(256)
            s.prefill(prompt)
            s.prefill_tokens(ids)
            states.append(s)
        lats = [None] * B
        got = 0
        for call in range(steps + 1):
            r = eng.step(B)
            if call == 0:
                assert not r.valid.any()
                continue
            for b in range(B):
                ref = states[b].step(lats[b])
                lats[b] = ref["latent"]
                assert r.valid[b]
                np.testing.assert_allclose(r.latents[b], ref["latent"], atol=LAT_TOL)
                assert pcm_err(r.pcm[b] - ref["pcm"]) <= PCM_TOL
                got += 1
        assert got == B * steps
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_quant_mode_mismatch_is_an_error():
    """A deferred blob packed without quantization cannot back a weight_quant engine; one
    packed with the same mode can (the multi-GPU path: rank 0 packs, the others receive)."""
    import pocket_tts_amd as pt

    eng = pt.Engine(device=0, max_slots=1, max_ctx=64, defer_weights=True, weight_quant=1)
    try:
        eng.load_blob(pt.Engine.pack_weights(0x5EED, None, 0))
        with pytest.raises(pt.PocketTTSError, match="weight_quant"):
            eng.finalize()
    finally:
        eng.close()
    eng = pt.Engine(device=0, max_slots=1, max_ctx=64, defer_weights=True, weight_quant=1)
    try:
        with pytest.raises(pt.PocketTTSError):
            eng.load_blob(np.zeros(10, np.float32))
        eng.load_blob(pt.Engine.pack_weights(0x5EED, None, 1))
        eng.finalize()
        assert eng.int8_matrices == 34
    finally:
        eng.close()
    with pytest.raises(pt.PocketTTSError):
        pt.Engine(device=0, max_slots=1, max_ctx=64, weight_quant=7)
