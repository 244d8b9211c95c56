"""BASELINE configs[0] on the GPU: "Hello, world!" through the reference's segment driver.

configs[0] is `generate()` of "Hello, world!" at temperature 0 (the reference runs it on Candle's
CPU path; the CLI's defaults, pocket-tts-cli/src/commands/generate.rs:117-187). The fixture
(tests/golden/gen_golden.py hello) is the reference's own Python modules driven the way
tts_model.rs:935-1071 does:
  * prepare_text_prompt("Hello, world!") = "        Hello, world!" (2 words < 5), whose ids under
    the reference's tokenizer.json are text_ids.json reference.native_ids[1] (tokenizers library);
  * eos_threshold -4.0, max_gen_len (2 + 2) * 13 = 52, frames_after_eos 5 (<= 4 words), and the
    Rust stop rule (tts_model.rs:1055-1063): the frame at eos_step + 5 is the last;
  * a second run at eos_threshold 0.25, above every logit, ends at max_gen_len (52 frames).
Synthetic weights (seed 0x5EED) and a synthetic 125-frame voice prompt stand in for the gated
checkpoint and the "alba" voice, both unavailable offline. The synthetic model's EOS logit is
above -4 from the first frame, so the CLI-default run stops after eos_step 0 + 5: 6 frames.
Gates: conftest LAT_TOL (EOS logit, latent) and PCM_TOL (PCM, max abs per frame)."""

import numpy as np
import pytest
from conftest import LAT_TOL, PCM_TOL, load_golden, pcm_err

pytestmark = pytest.mark.gpu

HELLO_WORDS = 2  # "Hello, world!": prepared_text.split_whitespace().count()


@pytest.mark.parametrize("name", ["hello_world", "hello_world_maxlen"])
def test_hello_world_generate_matches_reference(name):
    import pocket_tts_amd as pt

    d = load_golden(f"{name}.safetensors")
    n_frames, eos_step, fae, max_len = (int(v) for v in d["stop"])
    thr = float(d["eos_threshold"][0])
    assert max_len == (HELLO_WORDS + 2) * 13 and fae == 5
    model = pt.TTSModel.load_with_params(temp=0.0, eos_threshold=thr, max_ctx=256, seed=0x5EED)
    try:
        v = model.get_voice_state_from_prompt_tensor(d["prompt"])
        # TTSModel.generate on the reference tokenizer's ids (words= gives max_gen_len and the tail)
        frames = list(model.generate_stream(d["text_ids"], v, words=HELLO_WORDS))
        assert len(frames) == n_frames, (len(frames), n_frames)
        for i, f in enumerate(frames):
            assert f.shape == (1, 1, 1920)
            assert pcm_err(f[0, 0] - d["pcm"][i]) <= PCM_TOL, i
        audio = model.generate(d["text_ids"], v, words=HELLO_WORDS)
        assert audio.shape == (1, n_frames * 1920)
        np.testing.assert_array_equal(audio[0], np.concatenate([f[0, 0] for f in frames]))
        # the same segment on the engine: every frame's EOS logit and latent, the stop frame
        eng = model.engine
        eng.open(0, v, d["text_ids"], pt.GenerationParams(temp=0.0, eos_threshold=thr, frames_after_eos=fae,
                                                          max_frames=max_len, seed=1))
        for i in range(n_frames):
            r = eng.step(1)
            assert r.valid[0] and bool(r.last[0]) == (i == n_frames - 1), i
            assert abs(r.eos_logits[0] - d["eos_logit"][i]) <= LAT_TOL, (i, r.eos_logits[0], d["eos_logit"][i])
            np.testing.assert_allclose(r.latents[0], d["latent"][i], atol=LAT_TOL)
            assert pcm_err(r.pcm[0] - d["pcm"][i]) <= PCM_TOL, i
        assert not eng.step(1).valid[0]
    finally:
        model.engine.close()
