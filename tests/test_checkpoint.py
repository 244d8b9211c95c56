"""Real-checkpoint readiness (CPU, host-side packer of the C ABI; no GPU needed).

The reference loads `tts_b6369a24.safetensors` through VarBuilder prefixes `flow_lm.*` / `mimi.*`
as F32 (tts_model.rs:192-227, 279-426). The gated checkpoint is unavailable offline, so these tests
write the synthetic weights into safetensors files under the reference's own tensor names and
shapes (tests/golden/checkpoint_names.json, dumped from the reference's Python modules by
tests/golden/gen_golden.py names) and load them through `weights_path`:
  * the packer reads exactly the reference's state-dict tensors (the two TimestepEmbedder `freqs`
    buffers are recomputed, not read);
  * an F32 file packs to the same blob as the synthetic source, bit for bit;
  * BF16 and F16 files pack to the blob of their values widened to f32, bit for bit;
  * extra checkpoint tensors (the dropped VQ codebooks, learnt paddings) are ignored; a missing
    tensor or a wrong shape is an error."""

import json

import numpy as np
import pytest
from conftest import GOLDEN

SEED = 0x5EED


@pytest.fixture(scope="module")
def manifest():
    import pocket_tts_amd as pt

    return pt.Engine.weight_manifest()


@pytest.fixture(scope="module")
def synth_blob():
    import pocket_tts_amd as pt

    return pt.Engine.pack_weights(SEED)


def _tensors(manifest):
    import synth

    return {name: synth.synth_tensor(SEED, name, shape) for name, shape in manifest}


def test_manifest_is_the_reference_state_dict(manifest):
    ref = json.load(open(GOLDEN / "checkpoint_names.json"))
    got = dict(manifest)
    assert len(got) == len(manifest)  # no tensor read twice
    assert {k: tuple(v) for k, v in ref.items() if k in got} == got
    assert sorted(set(ref) - set(got)) == ["flow_lm.flow_net.time_embed.0.freqs", "flow_lm.flow_net.time_embed.1.freqs"]


def test_f32_checkpoint_packs_bit_identical(manifest, synth_blob, tmp_path):
    import pocket_tts_amd as pt
    from safetensors.numpy import save_file

    t = _tensors(manifest)
    t["mimi.quantizer.vq.layers.0.codebook.embedding"] = np.ones((8, 4), np.float32)  # ignored extras
    t["flow_lm.flow_net.time_embed.0.freqs"] = np.zeros(128, np.float32)
    path = tmp_path / "tts_b6369a24.safetensors"
    save_file(t, str(path))
    del t
    blob = pt.Engine.pack_weights(SEED, str(path))
    assert np.array_equal(blob.view(np.uint32), synth_blob.view(np.uint32))


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_half_checkpoint_packs_its_widened_values(manifest, tmp_path, dtype):
    import pocket_tts_amd as pt
    import torch
    from safetensors.numpy import save_file as save_np
    from safetensors.torch import save_file as save_pt

    tdt = torch.bfloat16 if dtype == "bf16" else torch.float16
    half = {k: torch.from_numpy(v).to(tdt) for k, v in _tensors(manifest).items()}
    save_pt(half, str(tmp_path / "half.safetensors"))
    save_np({k: v.float().numpy() for k, v in half.items()}, str(tmp_path / "widened.safetensors"))
    del half
    a = pt.Engine.pack_weights(SEED, str(tmp_path / "half.safetensors"))
    b = pt.Engine.pack_weights(SEED, str(tmp_path / "widened.safetensors"))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_missing_or_misshapen_tensor_is_an_error(manifest, tmp_path):
    import pocket_tts_amd as pt
    from safetensors.numpy import save_file

    small = {name: np.zeros(shape, np.float32) for name, shape in manifest if np.prod(shape) <= 4096}
    save_file(small, str(tmp_path / "partial.safetensors"))
    with pytest.raises(pt.PocketTTSError, match="missing"):
        pt.Engine.pack_weights(SEED, str(tmp_path / "partial.safetensors"))
    name, shape = manifest[1]  # flow_lm.bos_emb [32]
    t = {n: np.zeros(s, np.float32) for n, s in manifest}
    t[name] = np.zeros(shape[0] + 1, np.float32)
    save_file(t, str(tmp_path / "bad_shape.safetensors"))
    del t
    with pytest.raises(pt.PocketTTSError, match="shape"):
        pt.Engine.pack_weights(SEED, str(tmp_path / "bad_shape.safetensors"))
    with pytest.raises(pt.PocketTTSError):
        pt.Engine.pack_weights(SEED, str(tmp_path / "does_not_exist.safetensors"))


def test_transposed_tensor_is_a_shape_error(manifest, tmp_path):
    """Same element count, other shape (e.g. a [K, N] copy of a [N, K] linear weight): rejected."""
    import pocket_tts_amd as pt
    from safetensors.numpy import save_file

    t = {n: np.zeros(s, np.float32) for n, s in manifest}
    name = "flow_lm.input_linear.weight"
    assert t[name].shape == (1024, 32)
    t[name] = np.zeros((32, 1024), np.float32)
    save_file(t, str(tmp_path / "transposed.safetensors"))
    del t
    with pytest.raises(pt.PocketTTSError, match="shape mismatch for flow_lm.input_linear.weight"):
        pt.Engine.pack_weights(SEED, str(tmp_path / "transposed.safetensors"))


@pytest.mark.gpu
def test_gpu_engine_from_checkpoint_file_matches_synthetic(manifest, tmp_path, gpu_engine):
    """ptts_engine_create with weights_path (the reference's TTSModel::load path): an engine built
    from the F32 checkpoint file produces the synthetic engine's frames bit for bit."""
    import pocket_tts_amd as pt
    from conftest import load_golden
    from safetensors.numpy import save_file

    save_file(_tensors(manifest), str(tmp_path / "ckpt.safetensors"))
    d = load_golden("e2e_lsd1.safetensors")
    p = pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=3)
    eng = pt.Engine(device=0, max_slots=8, max_ctx=512, weights_path=str(tmp_path / "ckpt.safetensors"))
    try:
        outs = []
        for e in (eng, gpu_engine):
            e.open(0, e.voice_from_prompt(d["prompt"]), d["text_ids"], p)
            outs.append([e.step(1) for _ in range(3)])
        for a, b in zip(*outs):
            assert np.array_equal(a.pcm[0], b.pcm[0]) and np.array_equal(a.latents[0], b.latents[0])
    finally:
        eng.close()
