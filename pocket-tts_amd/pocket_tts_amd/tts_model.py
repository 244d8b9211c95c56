"""Host-side mirror of the reference's `TTSModel` API (crates/pocket-tts/src/tts_model.rs),
running the generation hot path through the HIP engine.

Reference surface kept:
  * `TTSModel.load / load_with_params`, public fields `temp`, `lsd_decode_steps`,
    `eos_threshold`, `noise_clamp`, `sample_rate`, `voice_prompt_chunk_frames` (:22-49, :417);
  * voices: `get_voice_state` (:446-463), `get_voice_state_from_bytes` (:428-444),
    `get_voice_state_from_tensor` (:504-577), `get_voice_state_from_prompt_file / _bytes /
    _tensor` (:465-501). WAV decode on the host (audio.py), resampling and the Mimi encoder on
    the GPU;
  * generation: `generate` (:687-703), `generate_stream` (:894-913: sentence chunks of at most
    50 tokens, one segment each from a fresh copy of the voice state), `generate_stream_long`
    and `generate_with_pauses` (:856-883, 1074-1131: pause markers become silence), one
    [1, 1, 1920] frame per item; `split_into_best_sentences` (:601-684),
    `estimate_generation_steps` (:1187-1190).
Text goes through the text front end (text.py: tokenizer, prompt preparation); token-id input
is accepted too (one segment, no splitting).
"""

from __future__ import annotations

from typing import Callable, Iterator, Sequence

import numpy as np

from ._lib import FRAME, QUANT_ALL, QUANT_FLOW_LM, QUANT_NONE, SAMPLE_RATE
from .audio import read_wav, read_wav_from_bytes
from .engine import Engine, GenerationParams, Voice
from .text import (estimate_frames_after_eos, load_tokenizer, long_text_segments, max_gen_len,
                   prepare_text_prompt, silence_samples, split_into_best_sentences)

DEFAULT_VARIANT = "b6369a24"

__all__ = ["TTSModel", "prepare_text_prompt", "estimate_frames_after_eos", "max_gen_len", "DEFAULT_VARIANT"]


def _mono(audio: np.ndarray) -> np.ndarray:
    """[channels, n] -> [n]. The reference's Mimi encoder has one input channel, so a multi-channel
    prompt is an error there too (get_voice_state_from_tensor on [1, C, T])."""
    if audio.shape[0] != 1:
        raise ValueError(f"voice prompt must be mono, got {audio.shape[0]} channels")
    return audio[0]


class TTSModel:
    def __init__(self, engine: Engine, temp: float, lsd_decode_steps: int, eos_threshold: float,
                 noise_clamp: float | None, tokenizer: Callable[[str], Sequence[int]] | None = None):
        self.engine = engine
        self.temp = temp
        self.lsd_decode_steps = lsd_decode_steps
        self.eos_threshold = eos_threshold
        self.noise_clamp = noise_clamp
        self.sample_rate = SAMPLE_RATE
        self.tokenizer = tokenizer
        self.voice_prompt_chunk_frames: int | None = None  # tts_model.rs:417 (None = adaptive rule)
        # voice-prompt resampler for rates other than 24 kHz: "poly" (resample_poly, the rule of the
        # reference's ref.wav fixture pair) or "rubato" (the Rust driver's FastFixedIn / Septic,
        # audio.rs:197-255; restated, parity unpinned)
        self.voice_resampler: str = "poly"
        self._seed = 0

    @classmethod
    def load(cls, variant: str = DEFAULT_VARIANT, **kw) -> "TTSModel":
        return cls.load_with_params(variant, **kw)

    @classmethod
    def load_with_params(cls, variant: str = DEFAULT_VARIANT, temp: float = 0.7, lsd_decode_steps: int = 1,
                         eos_threshold: float = -4.0, noise_clamp: float | None = None, *,
                         weights_path: str | None = None, tokenizer_path: str | None = None, seed: int = 0x5EED,
                         device: int = 0, max_ctx: int = 1024, tokenizer=None,
                         weight_quant: int = QUANT_NONE) -> "TTSModel":
        """weights_path: local safetensors with the TTSModel state-dict names (synthetic weights
        from `seed` when None); tokenizer_path: tokenizer.model (SentencePiece) or tokenizer.json."""
        if variant != DEFAULT_VARIANT:
            raise ValueError(f"unsupported variant {variant!r} (only {DEFAULT_VARIANT})")
        if tokenizer is None and tokenizer_path:
            tokenizer = load_tokenizer(tokenizer_path)
        eng = Engine(device=device, max_slots=1, max_ctx=max_ctx, lsd_decode_steps=lsd_decode_steps, seed=seed,
                     weights_path=weights_path, weight_quant=weight_quant)
        return cls(eng, temp, lsd_decode_steps, eos_threshold, noise_clamp, tokenizer)

    # ---- quantized loading (tts_model.rs:108-181, feature "quantized"). The reference's version
    # is a placeholder that returns the f32 model (is_quantized() == false); here the weights get
    # quantize_weights() with QuantizeConfig::default() (quantize.rs) and the FlowLM step GEMMs
    # stream the int8 codes. scope: QUANT_FLOW_LM (default) or QUANT_ALL.
    @classmethod
    def load_quantized(cls, variant: str = DEFAULT_VARIANT, **kw) -> "TTSModel":
        return cls.load_quantized_with_params(variant, **kw)

    @classmethod
    def load_quantized_with_params(cls, variant: str = DEFAULT_VARIANT, temp: float = 0.7,
                                   lsd_decode_steps: int = 1, eos_threshold: float = -4.0,
                                   noise_clamp: float | None = None, *, scope: int = QUANT_FLOW_LM,
                                   **kw) -> "TTSModel":
        if scope not in (QUANT_FLOW_LM, QUANT_ALL):
            raise ValueError("scope must be QUANT_FLOW_LM or QUANT_ALL")
        return cls.load_with_params(variant, temp, lsd_decode_steps, eos_threshold, noise_clamp,
                                    weight_quant=scope, **kw)

    def is_quantized(self) -> bool:
        return self.engine.weight_quant != QUANT_NONE

    # ---- voice states
    def get_voice_state_from_prompt_tensor(self, prompt: np.ndarray) -> Voice:
        return self.engine.voice_from_prompt(np.asarray(prompt, np.float32).reshape(-1, 1024))

    def get_voice_state_from_tensor(self, audio: np.ndarray, sample_rate: int = SAMPLE_RATE) -> Voice:
        """tts_model.rs:504-577 (24 kHz mono PCM); other rates are resampled on the GPU first."""
        return self.engine.voice_from_audio(np.asarray(audio, np.float32).reshape(-1), sample_rate,
                                            self.voice_prompt_chunk_frames or 0, self.voice_resampler)

    def get_voice_state_from_bytes(self, data: bytes) -> Voice:
        """tts_model.rs:428-444: WAV bytes -> (GPU) resample -> encode -> prompt prefill."""
        audio, sr = read_wav_from_bytes(data)
        return self.get_voice_state_from_tensor(_mono(audio), sr)

    def get_voice_state(self, path: str) -> Voice:
        """tts_model.rs:446-463."""
        audio, sr = read_wav(path)
        return self.get_voice_state_from_tensor(_mono(audio), sr)

    def get_voice_state_from_prompt_file(self, path: str) -> Voice:
        """tts_model.rs:465-477: a safetensors file holding `audio_prompt` [1, F, 1024]."""
        from safetensors.numpy import load_file

        t = load_file(str(path))
        if "audio_prompt" not in t:
            raise KeyError("'audio_prompt' not found in safetensors file")
        return self.get_voice_state_from_prompt_tensor(t["audio_prompt"])

    def get_voice_state_from_prompt_bytes(self, data: bytes) -> Voice:
        """tts_model.rs:479-487."""
        from safetensors.numpy import load

        t = load(data)
        if "audio_prompt" not in t:
            raise KeyError("'audio_prompt' not found in safetensors bytes")
        return self.get_voice_state_from_prompt_tensor(t["audio_prompt"])

    # ---- text
    def _tok(self):
        if self.tokenizer is None:
            raise ValueError("text input needs a tokenizer (TTSModel.load(..., tokenizer_path=...) or "
                             "tokenizer=callable); or pass token ids")
        return self.tokenizer

    def count_tokens(self, text: str) -> int:
        tok = self._tok()
        return tok.count_tokens(text) if hasattr(tok, "count_tokens") else len(tok(text))

    def split_into_best_sentences(self, text: str) -> list[str]:
        return split_into_best_sentences(text, self.count_tokens)

    def estimate_generation_steps(self, text: str) -> int:
        return max_gen_len(prepare_text_prompt(text))

    # ---- generation
    def _params(self, max_frames: int, frames_after_eos: int) -> GenerationParams:
        self._seed += 1
        return GenerationParams(temp=self.temp, eos_threshold=self.eos_threshold, noise_clamp=self.noise_clamp,
                                frames_after_eos=frames_after_eos, max_frames=max_frames, seed=self._seed)

    def _segment(self, ids: np.ndarray, voice_state: Voice, max_frames: int, frames_after_eos: int
                 ) -> Iterator[np.ndarray]:
        """generate_stream_segment (tts_model.rs:935-1071) on engine row 0."""
        if self.lsd_decode_steps != self.engine.lsd_decode_steps:
            raise ValueError("lsd_decode_steps is fixed at engine creation")
        self.engine.open(0, voice_state, ids, self._params(max_frames, frames_after_eos))
        lag, delay = self.engine.frame_lag()  # overlapped stepping: frames arrive lag (+ delay) calls late
        lead = lag + delay
        while True:
            r = self.engine.step(1)
            if not r.valid[0]:
                if lead > 0:
                    lead -= 1
                    continue
                return
            lead = 0
            yield r.pcm[0].reshape(1, 1, FRAME).copy()
            if r.last[0]:
                return

    def generate_stream(self, text_or_ids, voice_state: Voice, max_frames: int | None = None,
                        words: int | None = None) -> Iterator[np.ndarray]:
        """tts_model.rs:894-913. Text: one segment per sentence chunk; max_gen_len and the EOS tail
        from each chunk (:968-969). Token ids (an extension for callers with their own tokenizer):
        one segment; ids carry no word count, so the caller passes `words` (the reference's rules
        then apply: max_gen_len = (words + 2) * 13, tail 5 frames up to 4 words else 3) or an
        explicit max_frames (tail 3)."""
        if not isinstance(text_or_ids, str):
            ids = np.asarray(text_or_ids, np.int32).reshape(-1)
            if words is None and max_frames is None:
                raise ValueError("token ids carry no word count: pass words= or max_frames=")
            fae = 3 if words is None else (5 if words <= 4 else 3)
            yield from self._segment(ids, voice_state, max_frames or (words + 2) * 13, fae)
            return
        tok = self._tok()
        for chunk in self.split_into_best_sentences(text_or_ids):
            prepared = prepare_text_prompt(chunk)
            ids = np.asarray(tok(prepared), np.int32)
            yield from self._segment(ids, voice_state, max_frames or max_gen_len(prepared),
                                     estimate_frames_after_eos(chunk))

    def generate(self, text_or_ids, voice_state: Voice, max_frames: int | None = None,
                 words: int | None = None) -> np.ndarray:
        """tts_model.rs:687-703: all frames concatenated, [1, N*1920]."""
        frames = list(self.generate_stream(text_or_ids, voice_state, max_frames, words))
        if not frames:
            raise RuntimeError("No audio generated")
        return np.concatenate(frames, axis=2)[0]

    def generate_stream_long(self, text: str, voice_state: Voice) -> Iterator[np.ndarray]:
        """tts_model.rs:1074-1131: text segments between pause markers, silence for each pause."""
        for kind, val in long_text_segments(text):
            if kind == "text":
                yield from self.generate_stream(val, voice_state)
            else:
                yield np.zeros((1, 1, silence_samples(val, self.sample_rate)), np.float32)

    def generate_with_pauses(self, text: str, voice_state: Voice) -> np.ndarray:
        """tts_model.rs:856-883."""
        chunks = list(self.generate_stream_long(text, voice_state))
        if not chunks:
            raise RuntimeError("No audio generated")
        return np.concatenate(chunks, axis=2)[0]
