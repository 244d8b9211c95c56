"""ctypes binding of libpocket_tts_hip.so (include/pocket_tts.h). No CPU fallback exists:
if the HIP library is missing or no GPU is visible, every entry point raises."""

from __future__ import annotations

import ctypes as C
import hashlib
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = Path(os.environ.get("PTTS_LIB", PKG_ROOT / "lib" / "libpocket_tts_hip.so"))

PTTS_OK = 0
ERRORS = {1: "invalid argument", 2: "HIP error", 3: "invalid state", 4: "I/O error"}
FRAME = 1920
LDIM = 32
DIM = 1024
SAMPLE_RATE = 24000
QUANT_NONE, QUANT_FLOW_LM, QUANT_ALL = 0, 1, 2
BACK_F32, BACK_BF16, BACK_F32X6 = 0, 1, 2  # ptts_engine_config.back_mfma (PTTS_BACK_*)
ABI_VERSION = 6  # PTTS_ABI_VERSION of include/pocket_tts.h that the structs below mirror

F32P = C.POINTER(C.c_float)
U8P = C.POINTER(C.c_uint8)
I32P = C.POINTER(C.c_int32)


class EngineConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int),
        ("max_slots", C.c_int),
        ("max_ctx", C.c_int),
        ("lsd_decode_steps", C.c_int),
        ("synth_seed", C.c_uint64),
        ("weights_path", C.c_char_p),
        ("weight_blob", C.c_void_p),
        ("defer_weights", C.c_int),
        ("pipeline", C.c_int),
        ("weight_quant", C.c_int),
        ("fp8_gemm", C.c_int),
        ("cfg_yaml", C.c_char_p),
        ("back_frames", C.c_int),
        ("back_mfma", C.c_int),
    ]


class GenParams(C.Structure):
    _fields_ = [
        ("temp", C.c_float),
        ("eos_threshold", C.c_float),
        ("noise_clamp", C.c_float),
        ("frames_after_eos", C.c_int),
        ("max_frames", C.c_int),
        ("seed", C.c_uint64),
    ]


# (name, restype, argtypes) for every symbol include/pocket_tts.h (the boundary) and
# include/pocket_tts_probe.h (measurement / test hooks) declare
SIGNATURES = [
    ("ptts_abi_version", C.c_int, []),
    ("ptts_build_id", C.c_char_p, []),
    ("ptts_weight_blob_bytes", C.c_size_t, []),
    ("ptts_pack_weights", C.c_int, [C.c_uint64, C.c_char_p, F32P, C.c_size_t]),
    ("ptts_pack_weights_ex", C.c_int, [C.c_uint64, C.c_char_p, C.c_int, F32P, C.c_size_t]),
    ("ptts_weight_manifest", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("ptts_quantize_tensor", C.c_int, [F32P, C.c_size_t, C.c_int, F32P, F32P]),
    ("ptts_quant_applies", C.c_int, [C.c_char_p, C.c_size_t, C.c_int]),
    ("ptts_engine_int8_matrices", C.c_int, [C.c_void_p]),
    ("ptts_engine_fp8_matrices", C.c_int, [C.c_void_p]),
    ("ptts_engine_create", C.c_int, [C.POINTER(EngineConfig), C.POINTER(C.c_void_p)]),
    ("ptts_config_check", C.c_int, [C.c_char_p]),
    ("ptts_engine_finalize", C.c_int, [C.c_void_p]),
    ("ptts_engine_load_blob", C.c_int, [C.c_void_p, F32P, C.c_size_t]),
    ("ptts_engine_destroy", None, [C.c_void_p]),
    ("ptts_engine_weight_blob", C.c_void_p, [C.c_void_p]),
    ("ptts_voice_from_prompt", C.c_int, [C.c_void_p, F32P, C.c_int, C.POINTER(C.c_void_p)]),
    ("ptts_voice_from_pcm", C.c_int, [C.c_void_p, F32P, C.c_int, C.POINTER(C.c_void_p)]),
    ("ptts_voice_from_audio", C.c_int, [C.c_void_p, F32P, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("ptts_resample_len", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("ptts_resample", C.c_int, [C.c_void_p, F32P, C.c_int, C.c_int, C.c_int, F32P]),
    ("ptts_resample_len_ex", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int]),
    ("ptts_resample_ex", C.c_int, [C.c_void_p, F32P, C.c_int, C.c_int, C.c_int, C.c_int, F32P]),
    ("ptts_voice_from_audio_ex", C.c_int, [C.c_void_p, F32P, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(C.c_void_p)]),
    ("ptts_flush_async", C.c_int, [C.c_void_p, C.c_int]),
    ("ptts_test_gemm", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, F32P, F32P, F32P]),
    ("ptts_voice_len", C.c_int, [C.c_void_p]),
    ("ptts_voice_conditioning", C.c_int, [C.c_void_p, F32P, C.c_int]),
    ("ptts_voice_destroy", None, [C.c_void_p]),
    ("ptts_slot_open", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, I32P, C.c_int, C.POINTER(GenParams)]),
    ("ptts_slots_open", C.c_int, [C.c_void_p, C.c_int, I32P, C.POINTER(C.c_void_p), I32P, I32P,
                                  C.POINTER(GenParams)]),
    ("ptts_probe_overlap", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    ("ptts_slot_close", C.c_int, [C.c_void_p, C.c_int]),
    ("ptts_step", C.c_int, [C.c_void_p, C.c_int, F32P, U8P, U8P, F32P, F32P]),
    ("ptts_step_async", C.c_int, [C.c_void_p, C.c_int]),
    ("ptts_sync", C.c_int, [C.c_void_p]),
    ("ptts_fetch", C.c_int, [C.c_void_p, C.c_int, F32P, U8P, U8P, F32P, F32P]),
    ("ptts_frame_lag", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("ptts_fetch_prev", C.c_int, [C.c_void_p, C.c_int, C.c_int, F32P, U8P, U8P, F32P, F32P]),
    ("ptts_preview_enable", C.c_int, [C.c_void_p, C.c_int]),
    ("ptts_fetch_ready", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    ("ptts_front_done", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    ("ptts_preview_fetch", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), F32P, C.POINTER(C.c_int)]),
    ("ptts_slot_set_latent", C.c_int, [C.c_void_p, C.c_int, F32P]),
    ("ptts_decode_latents", C.c_int, [C.c_void_p, C.c_int, F32P, C.c_int, F32P, F32P, F32P, F32P]),
    ("ptts_generate", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, I32P, C.c_int, C.POINTER(GenParams), F32P, C.c_int,
                                C.POINTER(C.c_int)]),
    ("ptts_time_kernel", C.c_int, [C.c_void_p, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_double)]),
    ("ptts_plan_ops", C.c_int, [C.c_void_p, C.c_int, C.c_char_p, C.c_int]),
    ("ptts_last_error", C.c_char_p, []),
]

_LIB: C.CDLL | None = None


class PocketTTSError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, 'error')} ({code}): {msg}")
        self.code = code


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"HIP extension {LIB_PATH} is missing: build it with `make -C pocket-tts_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(str(LIB_PATH))
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        abi = L.ptts_abi_version()
        if abi != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH} has C ABI version {abi}, these bindings mirror {ABI_VERSION}: rebuild it")
        _LIB = L
    return _LIB


def build_id() -> str:
    """Build id compiled into the loaded library (ptts_build_id)."""
    return lib().ptts_build_id().decode()


def source_build_id() -> str:
    """The build id the checked-out sources produce (the Makefile's BUILD_ID rule: sha256 over the
    sorted csrc/*.{hip,cpp,h}, include/pocket_tts.h, include/pocket_tts_probe.h and the Makefile,
    first 16 hex digits)."""
    csrc = PKG_ROOT / "csrc"
    files = sorted(p for ext in ("*.hip", "*.cpp", "*.h") for p in csrc.glob(ext))
    files += [PKG_ROOT.parent / "include" / "pocket_tts.h", PKG_ROOT.parent / "include" / "pocket_tts_probe.h",
              PKG_ROOT / "Makefile"]
    h = hashlib.sha256()
    for f in files:
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def check_build_id() -> str:
    """Raise unless the loaded library was built from the checked-out sources (a stale prebuilt
    binary, or a -DPTTS_PROBES measurement build, fails loudly). Returns the id."""
    got, want = build_id(), source_build_id()
    if got != want:
        raise RuntimeError(f"{LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                           "run `make -C pocket-tts_amd`")
    return got


def check(rc: int) -> None:
    if rc != PTTS_OK:
        raise PocketTTSError(rc, lib().ptts_last_error().decode(errors="replace"))


def fptr(a):
    return None if a is None else a.ctypes.data_as(F32P)


def u8ptr(a):
    return None if a is None else a.ctypes.data_as(U8P)
