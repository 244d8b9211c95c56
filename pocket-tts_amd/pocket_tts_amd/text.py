"""Text front end, host side: tokenizer, prompt preparation, sentence
chunking and pause markers. Host string work only; the token ids it produces feed the engine's
text prefill (`ptts_slot_open` / `ptts_slots_open`).

Reference behaviour restated here (crates/pocket-tts/src):
  * `Tokenizer`: the native tokenizer of `LUTConditioner` (conditioners/text.rs:18-107) = a
    SentencePiece Unigram model loaded from `tokenizer.model` (protobuf vocabulary, text.rs:81-217)
    into the `tokenizers` crate (0.21.4, Cargo.lock) with byte fallback, and a Metaspace
    pre-tokenizer ('▁', prepend always, no split), no normalizer and no special tokens added.
    The crate's Unigram encode is restated: Viterbi over the UTF-8 bytes with every vocabulary
    piece as a candidate (a prefix trie), unknown characters scored min_score - 10, consecutive
    unknowns fused into one piece, and unknown pieces emitted as `<0xXX>` byte tokens when the
    vocabulary has all of them (else the unk id). A `tokenizer.json` is read as `Tokenizer::from_file`
    does: its own pre-tokenizer, added special tokens and TemplateProcessing post-processor
    (the WASM build's file, crates/pocket-tts/assets/tokenizer.json, adds `<s>`).
  * `prepare_text_prompt` (tts_model.rs:1194-1227), `estimate_frames_after_eos` (:1230-1237),
    `max_gen_len` (:968), `split_into_best_sentences` (:601-684, the Rust algorithm: split after
    . ! ? ; :, pack sentences up to 50 tokens, 35-word batches for longer sentences).
  * pause markers (pause.rs:1-185): `[pause:Xms]` / `[pause:Xs]`, ellipses and commas, and the
    segmentation of `generate_stream_long` (tts_model.rs:1074-1131).
String positions are Python character offsets where the reference uses byte offsets; every
position is used only to slice the same string, and the markers are ASCII, so the results agree.
"""

from __future__ import annotations

import json
import re
import struct
from dataclasses import dataclass
from pathlib import Path
from typing import Sequence

META = "▁"  # '▁'
K_UNK_PENALTY = 10.0  # tokenizers::models::unigram::model::K_UNK_PENALTY
MAX_TOKENS_PER_CHUNK = 50  # tts_model.rs:604
WORDS_PER_BATCH = 35  # tts_model.rs:639


# =============================================================================================
# SentencePiece protobuf vocabulary (text.rs:81-217)
class TokenizerError(ValueError):
    pass


def read_varint(data: bytes, pos: int) -> tuple[int, int]:
    """text.rs:195-216."""
    result, shift = 0, 0
    while True:
        if pos >= len(data):
            raise TokenizerError("Unexpected end of data while reading varint")
        b = data[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift >= 64:
            raise TokenizerError("Varint too large")


def _skip(data: bytes, pos: int, wire: int) -> int | None:
    if wire == 0:
        return read_varint(data, pos)[1]
    if wire == 2:
        n, pos = read_varint(data, pos)
        return pos + n
    if wire == 5:
        return pos + 4
    if wire == 1:
        return pos + 8
    return None


def parse_sentencepiece_vocab(data: bytes) -> tuple[list[tuple[str, float]], int]:
    """ModelProto.pieces (field 1) -> [(piece, score)], unk id (type == 2). Pieces with an empty
    string are dropped, as in text.rs:166-168."""
    vocab: list[tuple[str, float]] = []
    unk_id, pos = 0, 0
    while pos < len(data):
        tag, pos = read_varint(data, pos)
        field, wire = tag >> 3, tag & 7
        if field == 1 and wire == 2:
            n, pos = read_varint(data, pos)
            end = pos + n
            piece, score, inner = "", 0.0, pos
            while inner < end:
                t, inner = read_varint(data, inner)
                f, w = t >> 3, t & 7
                if f == 1 and w == 2:
                    ln, inner = read_varint(data, inner)
                    piece = data[inner:inner + ln].decode("utf-8", errors="replace")
                    inner += ln
                elif f == 2 and w == 5:
                    if inner + 4 <= len(data):
                        score = struct.unpack_from("<f", data, inner)[0]
                        inner += 4
                elif f == 3 and w == 0:
                    typ, inner = read_varint(data, inner)
                    if typ == 2:
                        unk_id = len(vocab)
                else:
                    nxt = _skip(data, inner, w)
                    inner = end if nxt is None else nxt
            if piece:
                vocab.append((piece, float(score)))
            pos = end
        else:
            nxt = _skip(data, pos, wire)
            if nxt is None:
                break
            pos = nxt
    if not vocab:
        raise TokenizerError("No vocabulary found in SentencePiece model")
    return vocab, unk_id


# =============================================================================================
# Unigram model (tokenizers crate, models/unigram/model.rs: encode_optimized + tokenize)
class Unigram:
    def __init__(self, vocab: Sequence[tuple[str, float]], unk_id: int | None, byte_fallback: bool,
                 fuse_unk: bool = True):
        if not vocab:
            raise TokenizerError("empty vocabulary")
        self.vocab = [(p, float(s)) for p, s in vocab]
        self.token_to_id: dict[str, int] = {}
        for i, (p, _) in enumerate(self.vocab):
            self.token_to_id[p] = i
        # candidate pieces keyed by their UTF-8 bytes (the crate's trie holds every vocab entry)
        self.by_bytes: dict[bytes, int] = {p.encode(): self.token_to_id[p] for p, _ in self.vocab}
        self.max_len = max(len(k) for k in self.by_bytes)
        self.min_score = min(s for _, s in self.vocab)
        self.unk_id = unk_id
        self.byte_fallback = byte_fallback
        self.fuse_unk = fuse_unk
        self.byte_ids = None
        if byte_fallback:
            ids = [self.token_to_id.get(f"<0x{b:02X}>") for b in range(256)]
            self.byte_ids = ids

    def _viterbi(self, s: bytes) -> list[bytes]:
        size = len(s)
        unk_score = self.min_score - K_UNK_PENALTY
        best_score = [0.0] * (size + 1)
        best_start = [-1] * (size + 1)
        best_id = [0] * (size + 1)
        best_start[0] = 0
        pos = 0
        while pos < size:
            here = best_score[pos]
            mblen = _utf8_len(s[pos])
            single = False
            for ln in range(1, min(self.max_len, size - pos) + 1):
                tid = self.by_bytes.get(s[pos:pos + ln])
                if tid is None:
                    continue
                end = pos + ln
                cand = self.vocab[tid][1] + here
                if best_start[end] < 0 or cand > best_score[end]:
                    best_score[end], best_start[end], best_id[end] = cand, pos, tid
                if ln == mblen:
                    single = True
            if not single:
                end = pos + mblen
                cand = unk_score + here
                if best_start[end] < 0 or cand > best_score[end]:
                    best_score[end], best_start[end], best_id[end] = cand, pos, -1 if self.unk_id is None else self.unk_id
            pos += mblen
        out: list[bytes] = []
        unk_run: list[bytes] = []
        end = size
        while end > 0:
            start = best_start[end]
            piece = s[start:end]
            if self.fuse_unk and self.unk_id is not None and best_id[end] == self.unk_id:
                unk_run.append(piece)
            else:
                if unk_run:
                    out.append(b"".join(reversed(unk_run)))
                    unk_run = []
                out.append(piece)
            end = start
        if unk_run:
            out.append(b"".join(reversed(unk_run)))
        out.reverse()
        return out

    def tokenize(self, text: str) -> list[int]:
        ids: list[int] = []
        for piece in self._viterbi(text.encode("utf-8")):
            tid = self.by_bytes.get(piece)
            if tid is not None:
                ids.append(tid)
                continue
            if self.byte_fallback and all(self.byte_ids[b] is not None for b in piece):
                ids.extend(self.byte_ids[b] for b in piece)
                continue
            if self.unk_id is None:
                raise TokenizerError("unknown piece and no unk id")
            ids.append(self.unk_id)
        return ids


def _utf8_len(first_byte: int) -> int:
    if first_byte < 0x80:
        return 1
    if first_byte >> 5 == 0b110:
        return 2
    if first_byte >> 4 == 0b1110:
        return 3
    return 4


# =============================================================================================
@dataclass
class Metaspace:
    replacement: str = META
    prepend_scheme: str = "always"  # always | first | never
    split: bool = False

    def __call__(self, text: str) -> list[str]:
        s = text.replace(" ", self.replacement)
        if self.prepend_scheme in ("always", "first") and not s.startswith(self.replacement):
            s = self.replacement + s
        if not self.split:
            return [s]
        out, cur = [], ""
        for ch in s:  # MergedWithNext: every replacement char starts a new word
            if ch == self.replacement and cur:
                out.append(cur)
                cur = ""
            cur += ch
        return out + ([cur] if cur else [])


class Tokenizer:
    """The `tokenizers::Tokenizer` pipeline the reference builds (see module doc)."""

    def __init__(self, model: Unigram, pre: Metaspace, added: dict[str, int] | None = None,
                 template: list[tuple[str, object]] | None = None):
        self.model, self.pre = model, pre
        self.added = dict(added or {})
        self.template = template  # [("special", id) | ("seq", None)] of TemplateProcessing.single
        self._added_re = (re.compile("|".join(re.escape(t) for t in sorted(self.added, key=len, reverse=True)))
                          if self.added else None)

    # -- loaders (text.rs:26-38, 219-257)
    @classmethod
    def from_sentencepiece(cls, data: bytes) -> "Tokenizer":
        vocab, unk = parse_sentencepiece_vocab(data)
        return cls(Unigram(vocab, unk, byte_fallback=True), Metaspace(META, "always", False))

    @classmethod
    def from_json(cls, data: str | bytes, native: bool = False) -> "Tokenizer":
        """tokenizer.json as `Tokenizer::from_file` reads it; native=True applies the settings of
        the reference's .model path instead (prepend always, no added/special tokens)."""
        cfg = json.loads(data)
        m = cfg["model"]
        if m.get("type") != "Unigram":
            raise TokenizerError(f"unsupported tokenizer model {m.get('type')!r}")
        model = Unigram([(p, s) for p, s in m["vocab"]], m.get("unk_id"), bool(m.get("byte_fallback", False)))
        if native:
            return cls(model, Metaspace(META, "always", False))
        pre = cfg.get("pre_tokenizer") or {}
        if pre and pre.get("type") != "Metaspace":
            raise TokenizerError(f"unsupported pre-tokenizer {pre.get('type')!r}")
        meta = (Metaspace(pre.get("replacement", META), pre.get("prepend_scheme", "always"), bool(pre.get("split", True)))
                if pre else Metaspace(META, "never", False))
        added = {t["content"]: t["id"] for t in cfg.get("added_tokens") or []}
        template = None
        post = cfg.get("post_processor")
        if post:
            if post.get("type") != "TemplateProcessing":
                raise TokenizerError(f"unsupported post-processor {post.get('type')!r}")
            specials = post.get("special_tokens", {})
            template = []
            for item in post["single"]:
                if "SpecialToken" in item:
                    template.append(("special", specials[item["SpecialToken"]["id"]]["ids"]))
                else:
                    template.append(("seq", None))
        return cls(model, meta, added, template)

    @classmethod
    def from_file(cls, path, native: bool | None = None) -> "Tokenizer":
        p = Path(path)
        data = p.read_bytes()
        if p.suffix == ".model":
            return cls.from_sentencepiece(data)
        return cls.from_json(data, native=bool(native))

    # -- encode (Tokenizer::encode(text, add_special_tokens = true), text.rs:259-267)
    def encode(self, text: str) -> list[int]:
        parts: list[tuple[str, int | None]] = []
        if self._added_re is not None:
            last = 0
            for mt in self._added_re.finditer(text):
                if mt.start() > last:
                    parts.append((text[last:mt.start()], None))
                parts.append((mt.group(0), self.added[mt.group(0)]))
                last = mt.end()
            if last < len(text):
                parts.append((text[last:], None))
        else:
            parts = [(text, None)]
        ids: list[int] = []
        for seg, special in parts:
            if special is not None:
                ids.append(special)
                continue
            for word in self.pre(seg):
                ids.extend(self.model.tokenize(word))
        if self.template:
            out: list[int] = []
            for kind, val in self.template:
                out.extend(val if kind == "special" else ids)
            ids = out
        return ids

    __call__ = encode

    def count_tokens(self, text: str) -> int:
        """text.rs:305-313."""
        return len(self.encode(text))

    @property
    def vocab_size(self) -> int:
        return len(self.model.vocab)


def load_tokenizer(path, native: bool | None = None) -> Tokenizer:
    return Tokenizer.from_file(path, native)


# =============================================================================================
# pause markers (pause.rs)
ELLIPSIS_MS, COMMA_MS, PERIOD_MS, SEMICOLON_MS = 500, 200, 400, 300  # pause.rs:22-31
EXPLICIT_PAUSE = re.compile(r"\[pause:(\d+(?:\.\d+)?)(ms|s)\]")  # pause.rs:34-37
ELLIPSIS = re.compile(r"\.{3,}")  # pause.rs:39


@dataclass
class PauseMarker:
    original: str
    duration_ms: int
    position: int


def _ascii_float(s: str) -> float | None:
    """Rust's f64::from_str accepts ASCII digits only (\\d in the regex also matches others)."""
    return float(s) if s.isascii() else None


def _duration_ms(value: float, unit: str) -> int:
    ms = value if unit == "ms" else value * 1000.0
    return int(min(max(ms, 0.0), 4294967295.0))  # `as u32`: truncating, saturating


def parse_explicit_pauses(text: str) -> list[PauseMarker]:
    """pause.rs:52-73."""
    out = []
    for mt in EXPLICIT_PAUSE.finditer(text):
        v = _ascii_float(mt.group(1))
        if v is None:
            continue
        out.append(PauseMarker(mt.group(0), _duration_ms(v, mt.group(2)), mt.start()))
    return out


def parse_natural_pauses(text: str) -> list[PauseMarker]:
    """pause.rs:76-112: ellipses, and commas not between two ASCII digits."""
    out = [PauseMarker(mt.group(0), ELLIPSIS_MS, mt.start()) for mt in ELLIPSIS.finditer(text)]
    for i, ch in enumerate(text):
        if ch == ",":
            prev_digit = i > 0 and text[i - 1] in "0123456789"
            next_digit = i + 1 < len(text) and text[i + 1] in "0123456789"
            if not prev_digit or not next_digit:
                out.append(PauseMarker(",", COMMA_MS, i))
    out.sort(key=lambda p: p.position)
    return out


def strip_pause_markers(text: str) -> str:
    """pause.rs:115-117."""
    return EXPLICIT_PAUSE.sub(" ", text)


@dataclass
class ParsedText:
    clean_text: str
    pauses: list[PauseMarker]


def parse_text_with_pauses(text: str) -> ParsedText:
    """pause.rs:129-180: natural pauses of the clean text, plus explicit pauses moved to their
    clean-text positions (each marker became one space)."""
    clean = strip_pause_markers(text)
    pauses = parse_natural_pauses(clean)
    offset = 0
    for mt in EXPLICIT_PAUSE.finditer(text):
        v = _ascii_float(mt.group(1))
        ms = _duration_ms(v, mt.group(2)) if v is not None else 0
        if ms > 0:
            pauses.append(PauseMarker(mt.group(0), ms, max(mt.start() - offset, 0)))
        offset += len(mt.group(0)) - 1
    pauses.sort(key=lambda p: p.position)
    return ParsedText(clean, pauses)


def silence_samples(duration_ms: int, sample_rate: int) -> int:
    """pause.rs:183-185."""
    return duration_ms * sample_rate // 1000


def long_text_segments(text: str) -> list[tuple[str, object]]:
    """generate_stream_long's interleaving (tts_model.rs:1080-1108): [("text", str) | ("pause", ms)]."""
    parsed = parse_text_with_pauses(text)
    clean, segs, last = parsed.clean_text, [], 0
    for p in parsed.pauses:
        if p.position > last:
            seg = clean[last:p.position]
            if seg.strip():
                segs.append(("text", seg))
        segs.append(("pause", p.duration_ms))
        last = p.position + 1 if p.original.startswith("[pause:") else p.position + len(p.original)
    if last < len(clean):
        seg = clean[last:]
        if seg.strip():
            segs.append(("text", seg))
    return segs


# =============================================================================================
# prompt preparation and chunking (tts_model.rs)
def prepare_text_prompt(text: str) -> str:
    """tts_model.rs:1194-1227."""
    text = strip_pause_markers(text).strip()
    if not text:
        return "."
    text = text.replace("\n", " ").replace("\r", " ").replace("  ", " ")
    words = len(text.split())
    if not text[0].isupper():
        text = text[0].upper() + text[1:]
    if text[-1].isalnum():
        text += "."
    if words < 5:
        text = " " * 8 + text
    return text


def estimate_frames_after_eos(text: str) -> int:
    """tts_model.rs:1230-1237."""
    return 5 if len(text.split()) <= 4 else 3


def max_gen_len(prepared_text: str) -> int:
    """tts_model.rs:968: (words + 2) * 13 frames."""
    return (len(prepared_text.split()) + 2) * 13


_SENTENCE_END = re.compile(r"[^.!?;:]*[.!?;:]|[^.!?;:]+$")


def split_into_best_sentences(text: str, count_tokens) -> list[str]:
    """tts_model.rs:601-684 (the Rust algorithm; Python's differs)."""
    prepared = prepare_text_prompt(text)
    raw = [s.strip() for s in _SENTENCE_END.findall(prepared)]
    raw = [s for s in raw if s]
    if not raw:
        return [prepared]

    def count(s: str) -> int:
        try:
            return count_tokens(s)
        except Exception:
            return MAX_TOKENS_PER_CHUNK  # .unwrap_or(MAX_TOKENS_PER_CHUNK)

    chunks: list[str] = []
    cur, cur_n = "", 0
    for sentence in raw:
        n = count(sentence)
        if n > MAX_TOKENS_PER_CHUNK:
            if cur:
                chunks.append(cur)
                cur, cur_n = "", 0
            words = sentence.split()
            for i in range(0, len(words), WORDS_PER_BATCH):
                batch = words[i:i + WORDS_PER_BATCH]
                s = " ".join(batch)
                if count(s) <= MAX_TOKENS_PER_CHUNK:
                    chunks.append(s)
                else:
                    mid = len(batch) // 2
                    chunks.append(" ".join(batch[:mid]))
                    chunks.append(" ".join(batch[mid:]))
            continue
        if not cur:
            cur, cur_n = sentence, n
        elif cur_n + n > MAX_TOKENS_PER_CHUNK:
            chunks.append(cur)
            cur, cur_n = sentence, n
        else:
            cur += " " + sentence
            cur_n += n
    if cur:
        chunks.append(cur)
    return chunks
