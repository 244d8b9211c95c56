"""Deterministic synthetic weights for variant b6369a24 (numpy restatement).

Real checkpoints (hf://kyutai/pocket-tts, `config/b6369a24.yaml:3-4`) are gated
and unavailable offline, so every parity fixture and every benchmark runs on
weights drawn from a counter-based PRNG that is restated bit-identically in

  * this file (numpy; used to fill the Python reference modules when the
    golden fixtures are generated),
  * `oracle/ptts_oracle.c` (`synth_fill`), and
  * `pocket-tts_amd/csrc/weights.cpp` (`synth_fill`).

Element i of the tensor named `name` (TTSModel state-dict key, e.g.
"flow_lm.transformer.layers.0.self_attn.in_proj.weight") is

    key = fnv1a64(name)
    z   = splitmix64_finalize(seed * 0x9E3779B97F4A7C15 + key + i * 0xD1B54A32D192ED03)
    u   = (z >> 40) / 2**24                         # exact in f64
    v   = float32(center + (2u - 1) * halfwidth)    # f64 arithmetic, one rounding

The (center, halfwidth) per tensor comes from `init_rule(name, shape)`.
Only integer and IEEE f64 add/mul are involved, so C and numpy agree bit for bit.
"""

from __future__ import annotations

import math

import numpy as np

M64 = (1 << 64) - 1
C_SEED = 0x9E3779B97F4A7C15
C_IDX = 0xD1B54A32D192ED03


def fnv1a64(name: str) -> int:
    h = 0xCBF29CE484222325
    for b in name.encode():
        h ^= b
        h = (h * 0x100000001B3) & M64
    return h


def _splitmix_finalize(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform01(seed: int, name: str, n: int) -> np.ndarray:
    """u in [0,1) as float64, 24-bit resolution."""
    base = ((seed * C_SEED) + fnv1a64(name)) & M64
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(base) + idx * np.uint64(C_IDX)
        z = _splitmix_finalize(z)
    return (z >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)


def init_rule(name: str, shape: tuple[int, ...]) -> tuple[float, float] | None:
    """(center, halfwidth) of the uniform init for a parameter, None = leave as is.

    Mirrors torch's default init scale (U(+-1/sqrt(fan_in))) for matrices, and
    perturbs every norm/scale vector away from its identity value so that a
    kernel that drops an affine term cannot pass parity.
    """
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "freqs":  # TimestepEmbedder buffer, computed (mlp.py:73)
        return None
    if name.endswith("emb_std"):
        return (1.0, 0.1)
    if name.endswith("emb_mean"):
        return (0.0, 0.1)
    if name.endswith("bos_emb"):
        return (0.0, math.sqrt(3.0))
    if name.endswith("conditioner.embed.weight"):
        return (0.0, 1.0)
    if leaf == "alpha":  # RMSNorm
        return (1.0, 0.1)
    if leaf == "scale" and "layer_scale" in name:
        return (0.01, 0.005)
    is_norm = any(t in name for t in ("norm1.", "norm2.", "out_norm.", "in_ln."))
    if is_norm and leaf == "weight":
        return (1.0, 0.1)
    if is_norm and leaf == "bias":
        return (0.0, 0.1)
    if leaf == "bias":
        return (0.0, 0.05)
    if len(shape) >= 2:
        fan = int(np.prod(shape[1:]))
        return (0.0, 1.0 / math.sqrt(fan))
    raise ValueError(f"no init rule for {name} {shape}")


def synth_tensor(seed: int, name: str, shape: tuple[int, ...]) -> np.ndarray | None:
    rule = init_rule(name, shape)
    if rule is None:
        return None
    c, hw = rule
    n = int(np.prod(shape)) if shape else 1
    u = uniform01(seed, name, n)
    v = (c + (2.0 * u - 1.0) * hw).astype(np.float32)
    return v.reshape(shape)


def gaussian(seed: int, name: str, n: int, std: float) -> np.ndarray:
    """Box-Muller normal (used only for inputs stored inside fixtures)."""
    u1 = uniform01(seed, name + "#u1", n)
    u2 = uniform01(seed, name + "#u2", n)
    r = np.sqrt(-2.0 * np.log(u1 + (0.5 / 16777216.0)))
    return (std * r * np.cos(2.0 * math.pi * u2)).astype(np.float32)
