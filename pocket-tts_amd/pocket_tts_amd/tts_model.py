"""Host-side mirror of the reference's `TTSModel` API (crates/pocket-tts/src/tts_model.rs),
running the generation hot path through the HIP engine.

Reference surface kept: `TTSModel.load / load_with_params`, public fields `temp`,
`lsd_decode_steps`, `eos_threshold`, `noise_clamp`, `sample_rate`,
`get_voice_state_from_prompt_tensor` (:490-501), `get_voice_state_from_tensor` (:504-560),
`get_voice_state` (:449-463, 24 kHz mono WAV), `generate` (:687-703) and `generate_stream`
(:894-913, one frame of 1920 samples per item). Text enters as token ids; the SentencePiece
tokenizer and sentence splitting are the next row of the build, so a
`tokenizer` callable may be supplied for text input.
"""

from __future__ import annotations

from typing import Callable, Iterator, Sequence

import numpy as np

from ._lib import FRAME, SAMPLE_RATE
from .audio import read_wav, read_wav_from_bytes
from .engine import Engine, GenerationParams, Voice

DEFAULT_VARIANT = "b6369a24"


def prepare_text_prompt(text: str) -> str:
    """tts_model.rs:1194-1227 (pause markers are not parsed here)."""
    text = text.strip()
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
    """tts_model.rs:968."""
    return (len(prepared_text.split()) + 2) * 13


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
        self._seed = 0

    @classmethod
    def load(cls, variant: str = DEFAULT_VARIANT, **kw) -> "TTSModel":
        return cls.load_with_params(variant, **kw)

    @classmethod
    def load_with_params(cls, variant: str = DEFAULT_VARIANT, temp: float = 0.7, lsd_decode_steps: int = 1,
                         eos_threshold: float = -4.0, noise_clamp: float | None = None, *,
                         weights_path: str | None = None, seed: int = 0x5EED, device: int = 0,
                         max_ctx: int = 1024, tokenizer=None) -> "TTSModel":
        if variant != DEFAULT_VARIANT:
            raise ValueError(f"unsupported variant {variant!r} (only {DEFAULT_VARIANT})")
        eng = Engine(device=device, max_slots=1, max_ctx=max_ctx, lsd_decode_steps=lsd_decode_steps, seed=seed,
                     weights_path=weights_path)
        return cls(eng, temp, lsd_decode_steps, eos_threshold, noise_clamp, tokenizer)

    # ---- voice states
    def get_voice_state_from_prompt_tensor(self, prompt: np.ndarray) -> Voice:
        return self.engine.voice_from_prompt(np.asarray(prompt, np.float32).reshape(-1, 1024))

    def get_voice_state_from_tensor(self, audio: np.ndarray, sample_rate: int = SAMPLE_RATE) -> Voice:
        """tts_model.rs:504-577 (24 kHz mono PCM); other rates are resampled on the GPU first."""
        return self.engine.voice_from_audio(np.asarray(audio, np.float32).reshape(-1), sample_rate,
                                            self.voice_prompt_chunk_frames or 0)

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

    # ---- generation
    def _ids(self, text_or_ids) -> tuple[np.ndarray, int, int]:
        if isinstance(text_or_ids, str):
            if self.tokenizer is None:
                raise ValueError("text input needs a tokenizer callable (TTSModel(..., tokenizer=...)); "
                                 "or pass token ids")
            prepared = prepare_text_prompt(text_or_ids)
            ids = np.asarray(self.tokenizer(prepared), np.int32)
            return ids, max_gen_len(prepared), estimate_frames_after_eos(text_or_ids)
        ids = np.asarray(text_or_ids, np.int32).reshape(-1)
        return ids, (max(1, ids.size // 2) + 2) * 13, 3

    def _params(self, max_frames: int, frames_after_eos: int) -> GenerationParams:
        self._seed += 1
        return GenerationParams(temp=self.temp, eos_threshold=self.eos_threshold, noise_clamp=self.noise_clamp,
                                frames_after_eos=frames_after_eos, max_frames=max_frames, seed=self._seed)

    def generate_stream(self, text_or_ids, voice_state: Voice, max_frames: int | None = None) -> Iterator[np.ndarray]:
        if self.lsd_decode_steps != self.engine.lsd_decode_steps:
            raise ValueError("lsd_decode_steps is fixed at engine creation")
        ids, mgl, fae = self._ids(text_or_ids)
        p = self._params(max_frames or mgl, fae)
        self.engine.open(0, voice_state, ids, p)
        first = True
        while True:
            r = self.engine.step(1)
            if not r.valid[0]:
                if first and self.engine.pipeline:  # overlapped stepping: frames arrive one call late
                    first = False
                    continue
                return
            first = False
            yield r.pcm[0].reshape(1, 1, FRAME).copy()
            if r.last[0]:
                return

    def generate(self, text_or_ids, voice_state: Voice, max_frames: int | None = None) -> np.ndarray:
        frames = list(self.generate_stream(text_or_ids, voice_state, max_frames))
        if not frames:
            raise RuntimeError("No audio generated")
        return np.concatenate(frames, axis=2)[0]
