"""GPU mirror of the reference's streaming-equivalence tests (crates/pocket-tts/tests/
streaming_tests.rs:20-70 test_streaming_matches_batch, :72-116 test_streaming_yields_multiple_chunks),
on multi-sentence text that the Rust splitter (split_into_best_sentences, tts_model.rs:601-684)
cuts into several segments, each generated from a fresh copy of the voice state
(generate_stream, tts_model.rs:894-913).

At temperature 0:
  * the concatenated `generate_stream` items equal `generate` bit for bit (the reference allows
    1e-4; here both run the same kernels on the same inputs, so they must be identical);
  * every item is one [1, 1, 1920] frame, and there is more than one;
  * each segment equals its own oracle run (voice prefill + that chunk's prepared ids, fresh
    state) frame for frame at the conftest gates (PCM <= 2e-6 max abs);
for the sequential engine and for the pipelined one (frames arrive one call late there).

The tokenizer is the synthetic Unigram tokenizer of test_text_frontend, wrapped so that every
sentence counts 40 tokens: two sentences never share a 50-token chunk, so the text below
yields three segments."""

import numpy as np
import pytest
from conftest import PCM_TOL
from test_text_frontend import synthetic_tokenizer

pytestmark = pytest.mark.gpu

TEXT = "Hello world. This is a test. Good day."
FRAMES = 10  # per segment (max_frames; EOS off)


class SentenceTokenizer:
    """The synthetic tokenizer's ids, with count_tokens() = 40 per sentence (one chunk each)."""

    def __init__(self, tok):
        self.tok = tok

    def __call__(self, text):
        return self.tok(text)

    def count_tokens(self, text):
        return 40


@pytest.mark.parametrize("pipeline,back_frames", [(False, 1), (True, 1), (True, 2), (True, 4)])
def test_streaming_matches_batch_over_multiple_chunks(oracle, pipeline, back_frames):
    import pocket_tts_amd as pt
    from pocket_tts_amd.text import prepare_text_prompt

    tok = SentenceTokenizer(synthetic_tokenizer())
    eng = pt.Engine(device=0, max_slots=1, max_ctx=256, lsd_decode_steps=1, seed=0x5EED, pipeline=pipeline,
                    back_frames=back_frames)
    try:
        m = pt.TTSModel(eng, temp=0.0, lsd_decode_steps=1, eos_threshold=float("inf"), noise_clamp=None, tokenizer=tok)
        prompt = (0.11 * np.random.default_rng(11).standard_normal((8, 1024))).astype(np.float32)
        v = m.get_voice_state_from_prompt_tensor(prompt)
        chunks = m.split_into_best_sentences(TEXT)
        assert len(chunks) == 3, chunks

        stream = list(m.generate_stream(TEXT, v, max_frames=FRAMES))
        assert len(stream) == 3 * FRAMES > 1
        assert all(f.shape == (1, 1, 1920) and f.dtype == np.float32 for f in stream)
        batch = m.generate(TEXT, v, max_frames=FRAMES)
        assert batch.shape == (1, 3 * FRAMES * 1920)
        assert np.array_equal(np.concatenate(stream, axis=2)[0], batch)  # bit for bit

        worst = 0.0
        for c, chunk in enumerate(chunks):
            ids = np.asarray(tok(prepare_text_prompt(chunk)), np.int32)
            s = oracle.new_state(256)
            s.prefill(prompt)
            s.prefill_tokens(ids)
            lat = None
            for i in range(FRAMES):
                ref = s.step(lat)
                lat = ref["latent"]
                e = float(np.abs(stream[c * FRAMES + i][0, 0] - ref["pcm"]).max())
                worst = max(worst, e)
                assert e <= PCM_TOL, (c, i, e)
        print(f"pipeline={pipeline} back_frames={back_frames}: worst PCM |d| vs oracle {worst:.3g}")
    finally:
        eng.close()
