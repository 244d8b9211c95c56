"""CPU: the C oracle against the golden vectors the reference produced (tests/golden/gen_golden.py).

Tolerances: FlowLM quantities 2e-5 abs (the oracle and PyTorch differ only in fp32 reduction
order), PCM 1e-6 abs."""

import numpy as np
import pytest
from conftest import load_golden

SHAPES = {
    "flow_lm.transformer.layers.0.self_attn.in_proj.weight": [3072, 1024],
    "flow_lm.bos_emb": [32],
    "mimi.decoder.model.2.convtr.weight": [512, 256, 12],
    "flow_lm.transformer.layers.3.norm2.bias": [1024],
    "mimi.decoder_transformer.transformer.layers.1.layer_scale_2.scale": [512],
}


def test_synthetic_weights_bit_exact(oracle):
    """The C restatement of the weight PRNG equals the numpy one used to fill the reference."""
    g = load_golden("synth_weights_head.safetensors")
    for name, ref in g.items():
        got = oracle.synth_head(0x5EED, name, SHAPES[name], ref.size)
        assert np.array_equal(got, ref), name


def test_synth_numpy_matches_fixture():
    import synth

    g = load_golden("synth_weights_head.safetensors")
    for name, ref in g.items():
        full = synth.synth_tensor(0x5EED, name, tuple(SHAPES[name])).reshape(-1)[: ref.size]
        assert np.array_equal(full, ref), name


@pytest.mark.parametrize("fixture,lsd", [("e2e_lsd1.safetensors", 1), ("e2e_lsd2.safetensors", 2)])
def test_oracle_e2e_matches_reference(oracle, fixture, lsd):
    d = load_golden(fixture)
    s = oracle.new_state(256)
    s.prefill(d["prompt"])
    s.prefill_tokens(d["text_ids"])
    assert s.pos == d["prompt"].shape[0] + d["text_ids"].size
    lat = None
    for i in range(d["latent"].shape[0]):
        r = s.step(lat, lsd_steps=lsd, intermediates=True)
        lat = r["latent"]
        np.testing.assert_allclose(r["tout"], d["tout"][i], atol=2e-5)
        assert abs(r["eos_logit"] - d["eos_logit"][i]) < 2e-5
        np.testing.assert_allclose(lat, d["latent"][i], atol=2e-5)
        np.testing.assert_allclose(r["pcm"], d["pcm"][i], atol=1e-6)
        if i < d["quantized"].shape[0]:
            np.testing.assert_allclose(r["quantized"], d["quantized"][i], atol=2e-5)
            np.testing.assert_allclose(r["after_upsample"].T, d["after_upsample"][i], atol=2e-5)
            np.testing.assert_allclose(r["after_tr"].T, d["after_decoder_transformer"][i], atol=2e-5)


def test_oracle_encoder_matches_reference(oracle):
    d = load_golden("encoder_4f.safetensors")
    cond, enc, tr, lat = oracle.encode(d["pcm"])
    np.testing.assert_allclose(enc, d["after_encoder"].T, atol=1e-6)
    np.testing.assert_allclose(tr, d["after_encoder_transformer"].T, atol=1e-6)
    np.testing.assert_allclose(lat, d["latent"].T, atol=1e-6)
    np.testing.assert_allclose(cond, d["conditioning"], atol=1e-6)


def test_oracle_streaming_state_is_per_utterance(oracle):
    """Two states stepped in lockstep from the same voice stay identical; a third fed a
    different latent diverges (no state leaks between utterances)."""
    d = load_golden("e2e_lsd1.safetensors")
    a, b = oracle.new_state(128), oracle.new_state(128)
    for s in (a, b):
        s.prefill(d["prompt"][:8])
    ra, rb = a.step(None), b.step(None)
    assert np.array_equal(ra["pcm"], rb["pcm"])
    rb2 = b.step(ra["latent"] + 0.5)
    ra2 = a.step(ra["latent"])
    assert not np.allclose(ra2["pcm"], rb2["pcm"])


def test_oracle_long_context_matches_reference(oracle):
    """The bench shape at B = 1 (BASELINE configs[2]): a 125-frame voice prompt, 40 text tokens and
    100 free-running frames at temperature 0 (golden `e2e_long`, made by the reference's own Python
    modules). The FlowLM context grows 165 -> 265 positions, past 256 keys, and the Mimi decoder's
    250-key window slides over 1,600 positions of its ring (attention.rs:167-264, sdpa.rs:128-171).
    Measured: latents 3.5e-6, EOS logits 2e-6, PCM 5e-8 max abs after 100 frames."""
    d = load_golden("e2e_long.safetensors")
    assert d["prompt"].shape == (125, 1024) and d["text_ids"].size == 40 and d["latent"].shape[0] == 100
    s = oracle.new_state(320)
    s.prefill(d["prompt"])
    s.prefill_tokens(d["text_ids"])
    lat = None
    for i in range(d["latent"].shape[0]):
        r = s.step(lat, intermediates=i < 3)
        lat = r["latent"]
        assert abs(r["eos_logit"] - d["eos_logit"][i]) < 2e-5, i
        np.testing.assert_allclose(lat, d["latent"][i], atol=2e-5)
        np.testing.assert_allclose(r["pcm"], d["pcm"][i], atol=1e-6)
        if i < 3:
            np.testing.assert_allclose(r["after_tr"].T, d["after_decoder_transformer"][i], atol=2e-5)


@pytest.mark.parametrize("fixture", ["hello_world.safetensors", "hello_world_maxlen.safetensors"])
def test_oracle_hello_world_matches_reference(oracle, fixture):
    """BASELINE configs[0] (gen_golden.py hello): "Hello, world!" as the reference tokenizer's ids
    of the prepared prompt, temp 0, the Rust stop rule (tts_model.rs:1055-1063) at eos_threshold
    -4.0 (6 frames: EOS at frame 0, 5 tail frames) and above every logit (max_gen_len 52)."""
    d = load_golden(fixture)
    n, eos_step, fae, max_len = (int(v) for v in d["stop"])
    thr = float(d["eos_threshold"][0])
    s = oracle.new_state(256)
    s.prefill(d["prompt"])
    s.prefill_tokens(d["text_ids"])
    lat, stop_at = None, None
    for i in range(max_len):
        r = s.step(lat)
        lat = r["latent"]
        if r["eos_logit"] > thr and stop_at is None:
            stop_at = i + fae
        assert abs(r["eos_logit"] - d["eos_logit"][i]) < 2e-5, i
        np.testing.assert_allclose(lat, d["latent"][i], atol=2e-5)
        np.testing.assert_allclose(r["pcm"], d["pcm"][i], atol=1e-6)
        if stop_at is not None and i >= stop_at:
            break
    assert i + 1 == n and (eos_step < 0 or stop_at == eos_step + fae)
