"""ctypes binding of the CPU oracle (oracle/libptts_oracle.so) - test infrastructure only."""

from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE = "libptts_oracle.so"  # the checker
CPU_FAST = "libptts_cpu_fast.so"  # same source, -DORC_FAST: the CPU-baseline build (bench only)
_LIBS: dict = {}
F32P = C.POINTER(C.c_float)


def lib(name: str = ORACLE) -> C.CDLL:
    if name not in _LIBS:
        path = ROOT / "oracle" / name
        if not path.exists():
            raise FileNotFoundError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(str(path))
        L.orc_model_create.restype = C.c_void_p
        L.orc_model_create.argtypes = [C.c_uint64]
        L.orc_model_create_ex.restype = C.c_void_p
        L.orc_model_create_ex.argtypes = [C.c_uint64, C.c_int]
        L.orc_quantize.restype = C.c_float
        L.orc_quantize.argtypes = [F32P, C.c_int64, C.c_int, F32P]
        L.orc_quant_applies.argtypes = [C.c_char_p, C.c_int64, C.c_int]
        L.orc_model_destroy.argtypes = [C.c_void_p]
        L.orc_synth_head.argtypes = [C.c_uint64, C.c_char_p, C.POINTER(C.c_int64), C.c_int, F32P, C.c_int64]
        L.orc_state_create.restype = C.c_void_p
        L.orc_state_create.argtypes = [C.c_void_p, C.c_int]
        L.orc_state_destroy.argtypes = [C.c_void_p]
        L.orc_state_pos.argtypes = [C.c_void_p]
        L.orc_prefill.argtypes = [C.c_void_p, C.c_void_p, F32P, C.c_int]
        L.orc_prefill_tokens.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int]
        L.orc_embed_tokens.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int, F32P]
        L.orc_step.argtypes = [C.c_void_p, C.c_void_p, F32P, F32P, C.c_int] + [F32P] * 7
        L.orc_mimi_decode.argtypes = [C.c_void_p, C.c_void_p, F32P, F32P]
        L.orc_encode.argtypes = [C.c_void_p, F32P, C.c_int, F32P, F32P, F32P, F32P]
        L.orc_encode_ex.argtypes = [C.c_void_p, F32P, C.c_int, C.c_int, F32P, F32P, F32P, F32P]
        L.orc_resample_len.argtypes = [C.c_int, C.c_int, C.c_int]
        L.orc_resample.argtypes = [F32P, C.c_int, C.c_int, C.c_int, F32P]
        L.orc_resample_septic_len.argtypes = [C.c_int, C.c_int, C.c_int]
        L.orc_resample_septic.argtypes = [F32P, C.c_int, C.c_int, C.c_int, F32P]
        L.orc_time_embeddings.argtypes = [C.c_void_p, C.c_int, F32P]
        L.orc_bench.restype = C.c_double
        L.orc_bench.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        _LIBS[name] = L
    return _LIBS[name]


def fp(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(F32P)


class Oracle:
    """One synthetic-weight model (seed) on the CPU; quant = weight quantization scope
    (0 none, 1 flow_lm.*, 2 all: the oracle's quantize.rs restatement)."""

    def __init__(self, seed: int = 0x5EED, quant: int = 0, lib_name: str = ORACLE):
        self.L = lib(lib_name)
        self.m = self.L.orc_model_create_ex(seed, quant)

    def __del__(self):
        if getattr(self, "m", None):
            self.L.orc_model_destroy(self.m)
            self.m = None

    def synth_head(self, seed, name, shape, n):
        out = np.zeros(n, np.float32)
        sh = (C.c_int64 * len(shape))(*shape)
        rc = self.L.orc_synth_head(seed, name.encode(), sh, len(shape), fp(out), n)
        assert rc == 0
        return out

    def new_state(self, max_ctx=1024):
        return OracleState(self, max_ctx)

    def time_embeddings(self, n):
        out = np.zeros((n, 512), np.float32)
        self.L.orc_time_embeddings(self.m, n, fp(out))
        return out

    def encode(self, pcm: np.ndarray, chunk_frames: int = -1):
        """chunk_frames <= 0: one pass (Python reference); else the Rust chunked encode."""
        pcm = np.ascontiguousarray(pcm, np.float32)
        F = pcm.size // 1920
        T = pcm.size // 120
        cond = np.zeros((F, 1024), np.float32)
        enc = np.zeros((T, 512), np.float32)
        tr = np.zeros((T, 512), np.float32)
        lat = np.zeros((F, 512), np.float32)
        self.L.orc_encode_ex(self.m, fp(pcm), pcm.size, chunk_frames, fp(cond), fp(enc), fp(tr), fp(lat))
        return cond, enc, tr, lat

    def bench(self, n_utt, F, S, n_frames, threads):
        return self.L.orc_bench(self.m, n_utt, F, S, n_frames, threads)


def quantize(x: np.ndarray, num_levels: int = 256):
    """The oracle's QuantizedTensor::quantize restatement: (simulated values, scale)."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    sc = lib().orc_quantize(fp(x), x.size, num_levels, fp(out))
    return out, float(sc)


def quant_applies(name: str, numel: int, mode: int) -> bool:
    return bool(lib().orc_quant_applies(name.encode(), numel, mode))


def resample(x: np.ndarray, sr_from: int, sr_to: int = 24000) -> np.ndarray:
    """The oracle's restatement of the reference resampler (scipy resample_poly rule)."""
    L = lib()
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    y = np.zeros(max(L.orc_resample_len(x.size, sr_from, sr_to), 1), np.float32)
    n = L.orc_resample(fp(x), x.size, sr_from, sr_to, fp(y))
    return y[:n]


def resample_septic(x: np.ndarray, sr_from: int, sr_to: int = 24000) -> np.ndarray:
    """The oracle's restatement of the Rust driver's resampler (rubato FastFixedIn / Septic)."""
    L = lib()
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    y = np.zeros(max(L.orc_resample_septic_len(x.size, sr_from, sr_to), 1), np.float32)
    n = L.orc_resample_septic(fp(x), x.size, sr_from, sr_to, fp(y))
    return y[:n]


class OracleState:
    def __init__(self, o: Oracle, max_ctx: int):
        self.o = o
        self.s = o.L.orc_state_create(o.m, max_ctx)

    def __del__(self):
        if getattr(self, "s", None):
            self.o.L.orc_state_destroy(self.s)
            self.s = None

    @property
    def pos(self):
        return self.o.L.orc_state_pos(self.s)

    def prefill(self, x: np.ndarray):
        x = np.ascontiguousarray(x, np.float32)
        self.o.L.orc_prefill(self.o.m, self.s, fp(x), x.shape[0])

    def prefill_tokens(self, ids):
        ids = np.ascontiguousarray(ids, np.int32)
        self.o.L.orc_prefill_tokens(self.o.m, self.s, ids.ctypes.data_as(C.POINTER(C.c_int32)), ids.size)

    def step(self, latent_in=None, noise=None, lsd_steps=1, intermediates=False):
        out = dict(tout=np.zeros(1024, np.float32), eos_logit=np.zeros(1, np.float32),
                   latent=np.zeros(32, np.float32), pcm=np.zeros(1920, np.float32))
        if intermediates:
            out.update(quantized=np.zeros(512, np.float32), after_upsample=np.zeros((16, 512), np.float32),
                       after_tr=np.zeros((16, 512), np.float32))
        li = None if latent_in is None else np.ascontiguousarray(latent_in, np.float32)
        nz = None if noise is None else np.ascontiguousarray(noise, np.float32)
        self.o.L.orc_step(self.o.m, self.s, fp(li), fp(nz), lsd_steps, fp(out["tout"]), fp(out["eos_logit"]),
                          fp(out["latent"]), fp(out["pcm"]), fp(out.get("quantized")),
                          fp(out.get("after_upsample")), fp(out.get("after_tr")))
        out["eos_logit"] = float(out["eos_logit"][0])
        return out
