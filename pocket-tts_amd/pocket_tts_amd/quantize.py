"""Weight quantization API of the reference (crates/pocket-tts/src/quantize.rs, re-exported at
lib.rs:16): QuantizeConfig, QuantizedTensor, quantize_weights, calculate_snr.

The arithmetic is the engine's own C++ restatement (`ptts_quantize_tensor`, host only, no GPU):
symmetric per-tensor levels, scale = max|x| / (levels/2 - 1), data = clamp(round(x / scale)) *
scale in f32 with round half away from zero. The engine applies the same function while packing
weights (`weight_quant`), so `quantize_weights(state_dict)` here and a quantized engine hold the
same values; on the GPU the FlowLM step GEMMs then stream the int8 codes.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from ._lib import F32P, check, lib


@dataclass
class QuantizeConfig:
    """QuantizeConfig (quantize.rs:17-41); the defaults are QuantizeConfig::default()."""

    skip_layers: list[str] = field(default_factory=lambda: ["embed", "lut", "out_proj", "eos_head"])
    min_size: int = 1024
    num_levels: int = 256


@dataclass
class QuantizedTensor:
    """QuantizedTensor (quantize.rs:43-118): simulated values stored as f32."""

    data: np.ndarray
    scale: float
    zero_point: float = 0.0
    num_levels: int = 256

    @classmethod
    def quantize(cls, tensor: np.ndarray, num_levels: int = 256) -> "QuantizedTensor":
        x = np.ascontiguousarray(tensor, np.float32)
        out = np.empty_like(x)
        sc = C.c_float()
        check(lib().ptts_quantize_tensor(x.ctypes.data_as(F32P), x.size, int(num_levels), out.ctypes.data_as(F32P),
                                         C.byref(sc)))
        return cls(out, float(sc.value), 0.0, int(num_levels))

    def theoretical_memory_savings(self) -> float:
        return {256: 4.0, 65536: 2.0}.get(self.num_levels, 1.0)


def should_skip_layer(name: str, config: QuantizeConfig) -> bool:
    """quantize.rs:120-123: substring match against skip_layers."""
    return any(s in name for s in config.skip_layers)


def quantize_weights(weights: dict[str, np.ndarray], config: QuantizeConfig | None = None
                     ) -> dict[str, QuantizedTensor]:
    """quantize.rs:126-150: small or skipped tensors pass through with num_levels 0, scale 1."""
    config = config or QuantizeConfig()
    out = {}
    for name, t in weights.items():
        t = np.asarray(t, np.float32)
        if t.size < config.min_size or should_skip_layer(name, config):
            out[name] = QuantizedTensor(t.copy(), 1.0, 0.0, 0)
        else:
            out[name] = QuantizedTensor.quantize(t, config.num_levels)
    return out


def calculate_snr(original: np.ndarray, quantized: np.ndarray) -> float:
    """quantize.rs:153-168: 10 log10(mean(x^2) / mean((x - q)^2)), +inf when exact."""
    o = np.asarray(original, np.float32)
    q = np.asarray(quantized, np.float32)
    signal = float(np.mean(o * o, dtype=np.float32))
    noise = float(np.mean((o - q) * (o - q), dtype=np.float32))
    if noise <= 0.0:
        return float("inf")
    return float(10.0 * np.log10(signal / noise))
