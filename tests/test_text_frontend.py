"""Text front end: tokenizer, prompt preparation, sentence chunking,
pause markers, and text-driven generation through the engine.

Pinning: token ids are bit-exact against tests/golden/text_ids.json, produced by the `tokenizers`
library (the binding of the crate the reference links) configured as the reference's native
loader (text.rs:58-79) and as Tokenizer::from_file on the reference's tokenizer.json
(gen_text_golden.py). The string rules restate tts_model.rs / pause.rs and carry the reference's
own unit tests (tts_model.rs:1239-1290, pause.rs:187-249, text.rs:316-390)."""

import json
import struct
from pathlib import Path

import numpy as np
import pytest
from conftest import GOLDEN

REF_JSON = Path("/root/reference/crates/pocket-tts/assets/tokenizer.json")


def golden():
    return json.loads((GOLDEN / "text_ids.json").read_text())


def synthetic_tokenizer():
    from pocket_tts_amd.text import Metaspace, Tokenizer, Unigram

    g = golden()["synthetic"]
    return Tokenizer(Unigram([tuple(v) for v in g["vocab"]], g["unk_id"], True), Metaspace())


def sp_model_bytes(vocab, unk_id):
    """A SentencePiece ModelProto with `vocab` (the encoder of text.rs:320-356)."""

    def varint(v):
        out = bytearray()
        while v >= 0x80:
            out.append((v & 0x7F) | 0x80)
            v >>= 7
        out.append(v)
        return bytes(out)

    out = bytearray()
    for i, (p, s) in enumerate(vocab):
        pb = p.encode()
        msg = b"\x0a" + varint(len(pb)) + pb + b"\x15" + struct.pack("<f", s)
        msg += b"\x18" + varint(2 if i == unk_id else (3 if p.startswith("<") and len(p) <= 6 else 1))
        out += b"\x0a" + varint(len(msg)) + msg
    out += b"\x12\x04\x08\x01\x10\x02"  # an unrelated trainer_spec-like field, skipped
    return bytes(out)


# ------------------------------------------------------------------ tokenizer
def test_unigram_matches_tokenizers_library_synthetic_vocab():
    g = golden()
    tok = synthetic_tokenizer()
    for text, ids in zip(g["texts"], g["synthetic"]["native_ids"]):
        assert tok.encode(text) == ids, text


def test_sentencepiece_model_loader_matches():
    """The .model path (text.rs:58-79): protobuf vocabulary -> same ids as the golden native run."""
    from pocket_tts_amd.text import Tokenizer

    g = golden()
    vocab = [(p, float(np.float32(s))) for p, s in g["synthetic"]["vocab"]]
    tok = Tokenizer.from_sentencepiece(sp_model_bytes(vocab, 0))
    assert tok.vocab_size == len(vocab)
    for text, ids in zip(g["texts"], g["synthetic"]["native_ids"]):
        assert tok.encode(text) == ids, text


def test_reference_tokenizer_json_native_and_wasm_configs():
    if not REF_JSON.exists():
        pytest.skip("reference tokenizer.json not present")
    from pocket_tts_amd.text import load_tokenizer

    g = golden()
    native = load_tokenizer(REF_JSON, native=True)
    wasm = load_tokenizer(REF_JSON)
    assert native.vocab_size == g["reference"]["vocab_size"] == 4000
    for text, a, b in zip(g["texts"], g["reference"]["native_ids"], g["reference"]["json_ids"]):
        assert native.encode(text) == a, text
        assert wasm.encode(text) == b, text
    # "        Hello, world!" -> [260 x 7, 2994, 262, 578, 682]
    assert native.encode("        Hello, world!") == [260] * 7 + [2994, 262, 578, 682]


def test_read_varint_and_vocab_parser_kats():
    """text.rs:358-389."""
    from pocket_tts_amd.text import TokenizerError, parse_sentencepiece_vocab, read_varint

    data = bytes([0xAC, 0x02, 0x01])
    a, pos = read_varint(data, 0)
    b, end = read_varint(data, pos)
    assert (a, b, end) == (300, 1, 3)
    vocab, unk = parse_sentencepiece_vocab(sp_model_bytes([("<unk>", -1.0), ("hello", -2.5)], 0))
    assert unk == 0 and [p for p, _ in vocab] == ["<unk>", "hello"]
    assert abs(vocab[0][1] + 1.0) < 1e-6 and abs(vocab[1][1] + 2.5) < 1e-6
    with pytest.raises(TokenizerError, match="No vocabulary found"):
        parse_sentencepiece_vocab(b"")


# ------------------------------------------------------------------ prompt rules (tts_model.rs)
def test_prepare_text_prompt():
    """tts_model.rs:1243-1282."""
    from pocket_tts_amd.text import prepare_text_prompt

    assert prepare_text_prompt("hello world") == "        Hello world."
    assert prepare_text_prompt("Hello world.") == "        Hello world."
    assert prepare_text_prompt("  hello  ") == "        Hello."
    assert prepare_text_prompt("one two three four five") == "One two three four five."
    r = prepare_text_prompt("Hello [pause:500ms] world")
    assert "[pause:" not in r and "Hello" in r and "world" in r
    r = prepare_text_prompt("One [pause:100ms] two [pause:1s] three")
    assert "[pause:" not in r and all(w in r for w in ("One", "two", "three"))
    assert prepare_text_prompt("   ") == "."
    assert prepare_text_prompt("line one\nline two\r") == "        Line one line two."


def test_estimate_frames_after_eos_and_max_gen_len():
    from pocket_tts_amd.text import estimate_frames_after_eos, max_gen_len

    assert estimate_frames_after_eos("Hello world") == 5
    assert estimate_frames_after_eos("One two three four five") == 3
    assert max_gen_len("        Hello world.") == 52


def test_split_into_best_sentences():
    """tts_model.rs:601-684 with a whitespace-count tokenizer: punctuation split, packing up to
    50 tokens, 35-word batches for an over-long sentence."""
    from pocket_tts_amd.text import split_into_best_sentences

    count = lambda s: len(s.split())  # noqa: E731
    assert split_into_best_sentences("hello world", count) == ["Hello world."]
    assert split_into_best_sentences("Hello... world", count) == ["Hello. . . world."]
    a = " ".join(["w"] * 30) + "."
    b = " ".join(["x"] * 30) + "!"
    assert split_into_best_sentences(f"{a} {b}", count) == ["W" + a[1:], b]
    long = " ".join(f"w{i}" for i in range(80))
    out = split_into_best_sentences(f"Short one. {long}", count)
    assert out[0] == "Short one." and len(out[1].split()) == 35 and len(out[2].split()) == 35
    assert len(out[3].split()) == 10 and out[3].endswith(".")
    # a batch still over the limit is halved (tokenizer counting 2 per word)
    out = split_into_best_sentences(" ".join(["z"] * 40), lambda s: 2 * len(s.split()))
    assert [len(c.split()) for c in out] == [17, 18, 5]


# ------------------------------------------------------------------ pause markers (pause.rs)
def test_pause_rules():
    """pause.rs:191-248."""
    from pocket_tts_amd.text import (COMMA_MS, ELLIPSIS_MS, parse_explicit_pauses, parse_natural_pauses,
                                     parse_text_with_pauses, silence_samples, strip_pause_markers)

    p = parse_explicit_pauses("Hello [pause:500ms] world")
    assert len(p) == 1 and p[0].duration_ms == 500 and p[0].original == "[pause:500ms]"
    p = parse_explicit_pauses("Test [pause:1s] and [pause:1.5s]")
    assert [x.duration_ms for x in p] == [1000, 1500]
    assert [x.duration_ms for x in parse_natural_pauses("Hello... world")] == [ELLIPSIS_MS]
    assert [x.duration_ms for x in parse_natural_pauses("Hello, world")] == [COMMA_MS]
    assert parse_natural_pauses("That costs 1,000 dollars") == []
    assert strip_pause_markers("Hello [pause:500ms] world [pause:1s] done") == "Hello   world   done"
    parsed = parse_text_with_pauses("Hello... [pause:500ms] world, done")
    assert parsed.clean_text == "Hello...   world, done" and len(parsed.pauses) == 3
    assert [x.position for x in parsed.pauses] == [5, 9, 16]
    assert silence_samples(500, 24000) == 12000 and silence_samples(1000, 24000) == 24000


def test_long_text_segments():
    """generate_stream_long's interleaving (tts_model.rs:1080-1108)."""
    from pocket_tts_amd.text import long_text_segments

    assert long_text_segments("Hello [pause:500ms] world") == [("text", "Hello "), ("pause", 500), ("text", " world")]
    assert long_text_segments("One, two... three") == [("text", "One"), ("pause", 200), ("text", " two"),
                                                        ("pause", 500), ("text", " three")]
    assert long_text_segments("[pause:1s]") == [("pause", 1000)]


# ------------------------------------------------------------------ GPU: text -> audio
@pytest.mark.gpu
def test_text_generation_matches_oracle(oracle):
    """TTSModel with a tokenizer: the first sentence chunk is generated from the tokenizer's ids
    (prepared text), frame for frame equal to the oracle; the pause becomes exact silence."""
    import pocket_tts_amd as pt
    from pocket_tts_amd.text import estimate_frames_after_eos, max_gen_len, prepare_text_prompt

    tok = synthetic_tokenizer()
    m = pt.TTSModel.load_with_params(temp=0.0, eos_threshold=float("inf"), tokenizer=tok, max_ctx=256)
    try:
        rng = np.random.default_rng(5)
        prompt = (0.11 * rng.standard_normal((6, 1024))).astype(np.float32)
        v = m.get_voice_state_from_prompt_tensor(prompt)
        text = "hello world"
        frames = list(m.generate_stream(text, v))
        prepared = prepare_text_prompt(text)
        assert len(frames) == max_gen_len(prepared) == 52 and estimate_frames_after_eos(text) == 5
        ids = np.asarray(tok(prepared), np.int32)
        s = oracle.new_state(256)
        s.prefill(prompt)
        s.prefill_tokens(ids)
        lat = None
        for i in range(3):
            ref = s.step(lat)
            lat = ref["latent"]
            d = frames[i][0, 0] - ref["pcm"]
            assert np.sqrt(np.mean(d.astype(np.float64) ** 2)) <= 1e-4, i
        audio = m.generate_with_pauses("hello [pause:250ms] world", v)
        n_text = [max_gen_len(prepare_text_prompt(t)) for t in ("hello ", " world")]
        assert audio.shape == (1, sum(n_text) * 1920 + 6000)
        assert not audio[0, n_text[0] * 1920:n_text[0] * 1920 + 6000].any()
    finally:
        m.engine.close()
