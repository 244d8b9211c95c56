#!/usr/bin/env python3
"""Golden token ids for the text front end, from the HuggingFace
`tokenizers` library: the Python binding of the `tokenizers` crate the reference links
(0.21.4 in Cargo.lock; 0.22.2 here), configured exactly as the reference's native loader
builds it (conditioners/text.rs:58-79: Unigram(vocab, unk_id, byte_fallback = true), Metaspace
'▁' prepend Always, no split, no post-processor), and as `Tokenizer::from_file` reads the
reference's tokenizer.json (crates/pocket-tts/assets/tokenizer.json, the WASM copy).

Two vocabularies:
  * `synthetic`: a small Unigram vocabulary generated here (with the 256 byte pieces), committed
    inside the fixture, so the test runs anywhere;
  * `reference`: the reference's tokenizer.json vocabulary (4000 pieces; not committed, the test
    reads it from /root/reference when present). The real tokenizer.model is gated offline.

RUN HERE ONLY. Usage: python tests/golden/gen_text_golden.py
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF_JSON = Path("/root/reference/crates/pocket-tts/assets/tokenizer.json")

TEXTS = [
    "Hello, world!",
    "        Hello, world!",
    "        Hello world.",
    "One two three four five.",
    "The quick brown fox jumps over the lazy dog; it was 1,000 times faster: wow?",
    "  leading and   multiple   spaces  ",
    "Numbers 3.14159 and 2,718 and -42.",
    "Café naïve résumé über Straße.",
    "Emoji \U0001F600 and 中文 and 日本語 text.",
    "Line one.\nLine two.\rDone",
    "Unknown ☃☃☃ snowmen fused.",
    "Quotes \"double\" and 'single' (parens) [brackets] {braces}.",
    "<s> literal special </s> tokens <unk>",
    "a",
    ".",
    "Supercalifragilisticexpialidocious antidisestablishmentarianism.",
    "Hello... world... and more...",
    "It's a test-case with hyphen-ated words & symbols #1 @home 100%.",
]


def synthetic_vocab(seed=11):
    rng = np.random.default_rng(seed)
    words = ["hello", "world", "the", "quick", "brown", "fox", "test", "one", "two", "three", "numbers",
             "and", "caf", "line", "done", "super", "cal", "ing", "ed", "er", "s", "a", "e", "o", "l", "t"]
    pieces = {}
    for w in words:
        for s in ("▁" + w, w):
            for i in range(len(s)):
                for j in range(i + 1, min(len(s), i + 5) + 1):
                    pieces[s[i:j]] = None
    for ch in ".,!?;:'\"-()0123456789HOTLNCSEUQ▁é":
        pieces[ch] = None
    pieces["▁▁"] = None
    pieces["▁▁▁▁"] = None
    vocab = [["<unk>", 0.0], ["<s>", 0.0], ["</s>", 0.0], ["<pad>", 0.0]]
    vocab += [[f"<0x{b:02X}>", 0.0] for b in range(256)]
    for p in pieces:
        vocab.append([p, float(-1.0 - 9.0 * rng.random() - 0.3 * len(p) * rng.random())])
    return vocab


def native(vocab, unk_id=0):
    from tokenizers import Tokenizer, models, pre_tokenizers

    tok = Tokenizer(models.Unigram([tuple(v) for v in vocab], unk_id, True))
    tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="always", split=False)
    return tok


def main():
    from tokenizers import Tokenizer

    out = {"texts": TEXTS}
    vs = synthetic_vocab()
    tok = native(vs)
    out["synthetic"] = {"vocab": vs, "unk_id": 0, "native_ids": [tok.encode(t).ids for t in TEXTS]}
    if REF_JSON.exists():
        cfg = json.loads(REF_JSON.read_text())
        tok = native(cfg["model"]["vocab"], cfg["model"]["unk_id"])
        jt = Tokenizer.from_file(str(REF_JSON))
        out["reference"] = {"native_ids": [tok.encode(t).ids for t in TEXTS],
                            "json_ids": [jt.encode(t).ids for t in TEXTS],
                            "vocab_size": len(cfg["model"]["vocab"])}
    (HERE / "text_ids.json").write_text(json.dumps(out, ensure_ascii=False))
    print("wrote", HERE / "text_ids.json")


if __name__ == "__main__":
    main()
