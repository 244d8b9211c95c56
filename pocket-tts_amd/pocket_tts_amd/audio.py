"""Audio I/O of the voice-cloning front end, host side.

Mirrors crates/pocket-tts/src/audio.rs:
  * `read_wav` / `read_wav_from_bytes` (audio.rs:12-108, hound): RIFF/WAVE with integer PCM
    (8/16/24/32 bit, value / 2^(bits-1); 8-bit data is unsigned on disk) or IEEE float32, plain
    or WAVE_FORMAT_EXTENSIBLE; interleaved channels -> [channels, samples]; a data chunk cut short
    keeps the whole samples read so far (the reference accepts truncated files, audio.rs:33-49).
  * `pcm_i16_le_bytes` (audio.rs:110-146): clamp to [-1, 1], x 32767, truncate toward zero,
    channels interleaved.
  * `write_wav` / `wav_bytes` (audio.rs:148-185): 16-bit integer PCM RIFF/WAVE.
  * `normalize_peak` (audio.rs:187-194).
Resampling to 24 kHz is not here: it runs on the GPU inside `ptts_voice_from_audio`
(the polyphase resampler of pocket-tts_amd/csrc/kernels.hip).
"""

from __future__ import annotations

import struct
from pathlib import Path

import numpy as np

WAVE_FORMAT_PCM = 0x0001
WAVE_FORMAT_IEEE_FLOAT = 0x0003
WAVE_FORMAT_EXTENSIBLE = 0xFFFE


class WavError(ValueError):
    pass


def read_wav_from_bytes(data: bytes) -> tuple[np.ndarray, int]:
    """-> (samples float32 [channels, n], sample_rate)."""
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise WavError("not a RIFF/WAVE file")
    pos, fmt, body = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack_from("<I", data, pos + 4)[0]
        start = pos + 8
        if cid == b"fmt ":
            if size < 16:
                raise WavError("fmt chunk too short")
            tag, ch, sr, _, align, bits = struct.unpack_from("<HHIIHH", data, start)
            if tag == WAVE_FORMAT_EXTENSIBLE:
                if size < 40:
                    raise WavError("extensible fmt chunk too short")
                tag = struct.unpack_from("<H", data, start + 24)[0]  # first 2 bytes of the subformat GUID
            fmt = (tag, ch, sr, align, bits)
        elif cid == b"data":
            body = data[start:start + size]  # may be shorter than `size`: truncated file
            break
        pos = start + size + (size & 1)  # chunks are word aligned
    if fmt is None:
        raise WavError("missing fmt chunk")
    if body is None:
        raise WavError("missing data chunk")
    tag, ch, sr, align, bits = fmt
    if ch < 1:
        raise WavError("zero channels")
    width = (bits + 7) // 8
    if tag == WAVE_FORMAT_IEEE_FLOAT:
        if bits != 32:
            raise WavError(f"unsupported float width {bits}")
    elif tag != WAVE_FORMAT_PCM or bits not in (8, 16, 24, 32):
        raise WavError(f"unsupported WAV format tag {tag:#x} / {bits} bits")
    frame = width * ch
    n = len(body) // frame
    if n == 0 and len(body) > 0:
        raise WavError("truncated WAV data")
    raw = np.frombuffer(body[:n * frame], np.uint8).reshape(n * ch, width)
    if tag == WAVE_FORMAT_IEEE_FLOAT:
        x = raw.copy().view("<f4").reshape(-1)
    elif bits == 8:
        x = (raw[:, 0].astype(np.int32) - 128).astype(np.float32) / np.float32(128.0)
    else:
        v = np.zeros(n * ch, np.int64)
        for b in range(width):
            v |= raw[:, b].astype(np.int64) << (8 * b)
        sign = np.int64(1) << (bits - 1)
        v = (v ^ sign) - sign
        x = v.astype(np.float32) / np.float32(1 << (bits - 1))
    return np.ascontiguousarray(x.reshape(n, ch).T, np.float32), int(sr)


def read_wav(path) -> tuple[np.ndarray, int]:
    return read_wav_from_bytes(Path(path).read_bytes())


def pcm_i16_le_bytes(audio: np.ndarray) -> bytes:
    """audio [channels, n] (or [n] mono) -> interleaved little-endian int16."""
    a = np.asarray(audio, np.float32)
    a = a.reshape(1, -1) if a.ndim == 1 else a
    x = np.clip(a.T, -1.0, 1.0) * np.float32(32767.0)
    return x.astype(np.int16).astype("<i2").tobytes()  # float -> int casts truncate toward zero


def wav_bytes(audio: np.ndarray, sample_rate: int = 24000) -> bytes:
    a = np.asarray(audio, np.float32)
    ch = 1 if a.ndim == 1 else a.shape[0]
    data = pcm_i16_le_bytes(a)
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, WAVE_FORMAT_PCM, ch, sample_rate, sample_rate * 2 * ch, 2 * ch, 16)
    hdr += b"data" + struct.pack("<I", len(data))
    return hdr + data


def write_wav(path, audio: np.ndarray, sample_rate: int = 24000) -> None:
    Path(path).write_bytes(wav_bytes(audio, sample_rate))


def normalize_peak(audio: np.ndarray) -> np.ndarray:
    a = np.asarray(audio, np.float32)
    m = float(np.abs(a).max()) if a.size else 0.0
    return (a * np.float32(1.0 / m)).astype(np.float32) if m > 0 else a.copy()
