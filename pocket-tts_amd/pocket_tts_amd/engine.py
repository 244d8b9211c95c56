"""Batched engine over the C ABI: one engine per GPU, `max_slots` concurrent utterances."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import (BACK_BF16, BACK_F32, BACK_F32X6, DIM, F32P, FRAME, LDIM, EngineConfig, GenParams, check, fptr, lib,
                   u8ptr)


@dataclass
class GenerationParams:
    """Per-utterance knobs; field meaning follows TTSModel (tts_model.rs:22-49, 968-969)."""

    temp: float = 0.7
    eos_threshold: float = -4.0
    noise_clamp: float | None = None
    frames_after_eos: int = 3
    max_frames: int = 250
    seed: int = 0

    def to_c(self) -> GenParams:
        return GenParams(float(self.temp), float(self.eos_threshold),
                         float(self.noise_clamp) if self.noise_clamp is not None else 0.0,
                         int(self.frames_after_eos), int(self.max_frames), int(self.seed) & (2**64 - 1))


class Voice:
    """Immutable FlowLM KV prefix of a voice prompt (the reference's ModelState)."""

    def __init__(self, engine: "Engine", handle: int):
        self._engine = engine
        self.handle = C.c_void_p(handle)

    @property
    def n_frames(self) -> int:
        return lib().ptts_voice_len(self.handle)

    def conditioning(self) -> np.ndarray:
        out = np.zeros((self.n_frames, DIM), np.float32)
        check(lib().ptts_voice_conditioning(self.handle, fptr(out), out.shape[0]))
        return out

    def close(self):
        if self.handle:
            lib().ptts_voice_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class StepResult:
    pcm: np.ndarray  # [n_rows, 1920]
    valid: np.ndarray  # [n_rows] bool, row produced a frame this step
    last: np.ndarray  # [n_rows] bool, that frame was the row's final one
    eos_logits: np.ndarray  # [n_rows]
    latents: np.ndarray  # [n_rows, 32]


RESAMPLERS = {"poly": 0, "rubato": 1}  # PTTS_RESAMPLE_POLY, PTTS_RESAMPLE_RUBATO_SEPTIC


def resampler_code(name: str) -> int:
    if name not in RESAMPLERS:
        raise ValueError(f"resampler must be one of {sorted(RESAMPLERS)}, got {name!r}")
    return RESAMPLERS[name]


class Engine:
    def __init__(self, device: int = 0, max_slots: int = 1, max_ctx: int = 1024, lsd_decode_steps: int = 1,
                 seed: int = 0x5EED, weights_path: str | None = None, weight_blob: int | None = None,
                 defer_weights: bool = False, pipeline: bool = False, weight_quant: int = 0, fp8_gemm: bool = False,
                 cfg_yaml: str | None = None, back_frames: int = 1, back_bf16: bool = False,
                 back_mfma: int | None = None):
        """pipeline=True: overlapped stepping, each step() returns the frame produced by the
        previous call (see ptts_engine_config.pipeline). weight_quant: QUANT_NONE / QUANT_FLOW_LM /
        QUANT_ALL, the reference's simulated int8 weight quantization (quantize.rs), with the
        FlowLM step GEMMs streaming int8 codes. fp8_gemm=True: the large FlowLM step GEMMs run as
        fp8 W8A8 MFMA (accuracy-gated; see ptts_engine_config.fp8_gemm). cfg_yaml: the reference's
        model config (config/b6369a24.yaml), checked against the compiled dimensions.
        back_frames=n, 2 or 4 (pipelined only): n frames per Mimi-decode pass; a step() returns the
        frame computed 2 n - 1 calls earlier (`frame_lag`). back_mfma (ptts_engine_config.back_mfma): how the
        Mimi decode's GEMMs and convs use the matrix cores, BACK_F32 (exact f32 FMA chain), BACK_F32X6
        (f32 products as six bf16 piece products, f32 accuracy) or BACK_BF16 (operands rounded to
        bf16: a variant gated on PCM accuracy); back_bf16=True is BACK_BF16."""
        if back_mfma is None:
            back_mfma = BACK_BF16 if back_bf16 else BACK_F32
        elif back_bf16 and back_mfma != BACK_BF16:
            raise ValueError("back_bf16=True contradicts back_mfma=%d (pass one of them)" % back_mfma)
        cfg = EngineConfig(device, max_slots, max_ctx, lsd_decode_steps, seed,
                           weights_path.encode() if weights_path else None,
                           weight_blob or None, int(defer_weights), int(pipeline), int(weight_quant),
                           int(fp8_gemm), cfg_yaml.encode() if cfg_yaml else None, int(back_frames),
                           int(back_mfma))
        h = C.c_void_p()
        check(lib().ptts_engine_create(C.byref(cfg), C.byref(h)))
        self.handle = h
        self.weight_quant = int(weight_quant)
        self.max_slots = max_slots
        self.max_ctx = max_ctx
        self.lsd_decode_steps = lsd_decode_steps
        self.pipeline = bool(pipeline)
        self.back_frames = int(back_frames) if pipeline else 1
        self.back_mfma = int(back_mfma)
        self.back_bf16 = self.back_mfma == BACK_BF16

    def test_gemm(self, layout: int, x: np.ndarray, w: np.ndarray, splits: int = 1, tail_slices: int = 0) -> np.ndarray:
        """GEMM-core test hook (ptts_test_gemm): x [m][k] @ w [n][k]^T on tile `layout`; splits > 1
        returns the [splits][m][n] partial slabs."""
        x = np.ascontiguousarray(x, np.float32)
        w = np.ascontiguousarray(w, np.float32)
        m, k = x.shape
        n = w.shape[0]
        y = np.empty((splits, m, n) if splits > 1 else (m, n), np.float32)
        check(lib().ptts_test_gemm(self.handle, layout, m, n, k, splits, tail_slices, fptr(x), fptr(w), fptr(y)))
        return y

    def frame_lag(self) -> tuple[int, int]:
        """(lag, admit_delay): a frame arrives `lag` calls after the call that computed it; the
        rows of the latest admission start `admit_delay` calls late (ptts_frame_lag)."""
        d = C.c_int(0)
        lag = int(lib().ptts_frame_lag(self.handle, C.byref(d)))
        return lag, int(d.value)

    @staticmethod
    def check_config(cfg_yaml: str) -> None:
        """Raise PocketTTSError unless the reference model config at `cfg_yaml` states the
        dimensions this build implements (b6369a24); no GPU needed (ptts_config_check)."""
        check(lib().ptts_config_check(cfg_yaml.encode()))

    @staticmethod
    def weight_blob_bytes() -> int:
        return int(lib().ptts_weight_blob_bytes())

    @staticmethod
    def pack_weights(seed: int = 0x5EED, weights_path: str | None = None, weight_quant: int = 0) -> np.ndarray:
        """Packed weight blob (engine device layout) built on the host; no GPU needed.
        weight_quant applies the reference's quantize_weights (quantize.rs) while packing."""
        out = np.empty(Engine.weight_blob_bytes() // 4, np.float32)
        check(lib().ptts_pack_weights_ex(seed, weights_path.encode() if weights_path else None, int(weight_quant),
                                         out.ctypes.data_as(F32P), out.nbytes))
        return out

    @staticmethod
    def weight_manifest() -> list[tuple[str, tuple[int, ...]]]:
        """(checkpoint tensor name, shape) of every tensor the weight packer reads (host only)."""
        need = C.c_size_t(0)
        check(lib().ptts_weight_manifest(None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        check(lib().ptts_weight_manifest(buf, need.value, None))
        out = []
        for line in buf.value.decode().splitlines():
            name, dims = line.split("\t")
            out.append((name, tuple(int(x) for x in dims.split(",")) if dims else ()))
        return out

    @property
    def fp8_matrices(self) -> int:
        """FlowLM GEMM weight matrices on the fp8 W8A8 path (0 unless fp8_gemm)."""
        return int(lib().ptts_engine_fp8_matrices(self.handle))

    @property
    def int8_matrices(self) -> int:
        """FlowLM GEMM weight matrices streamed as int8 codes (0 unless weight_quant)."""
        return int(lib().ptts_engine_int8_matrices(self.handle))

    def weight_blob(self) -> int:
        return int(lib().ptts_engine_weight_blob(self.handle) or 0)

    def load_blob(self, blob: np.ndarray):
        """Fill a deferred engine's weights from a host blob (Engine.pack_weights)."""
        blob = np.ascontiguousarray(blob, np.float32)
        check(lib().ptts_engine_load_blob(self.handle, blob.ctypes.data_as(F32P), blob.nbytes))

    def finalize(self):
        check(lib().ptts_engine_finalize(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            lib().ptts_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- voices
    def voice_from_prompt(self, prompt: np.ndarray) -> Voice:
        p = np.ascontiguousarray(prompt, np.float32).reshape(-1, DIM)
        h = C.c_void_p()
        check(lib().ptts_voice_from_prompt(self.handle, fptr(p), p.shape[0], C.byref(h)))
        return Voice(self, h.value)

    def voice_from_pcm(self, pcm: np.ndarray) -> Voice:
        x = np.ascontiguousarray(pcm, np.float32).reshape(-1)
        h = C.c_void_p()
        check(lib().ptts_voice_from_pcm(self.handle, fptr(x), x.size, C.byref(h)))
        return Voice(self, h.value)

    def voice_from_audio(self, samples: np.ndarray, sample_rate: int, chunk_frames: int = 0,
                         resampler: str = "poly") -> Voice:
        """Mono samples at any rate -> GPU resample to 24 kHz -> chunked Mimi encode -> voice.
        chunk_frames: 0 = the reference's adaptive rule, > 0 = that many frames, < 0 = one pass.
        resampler: "poly" (resample_poly, the rule the reference's ref.wav fixture pair was made
        with) or "rubato" (the Rust driver's FastFixedIn / Septic, audio.rs:197-255)."""
        x = np.ascontiguousarray(samples, np.float32).reshape(-1)
        h = C.c_void_p()
        check(lib().ptts_voice_from_audio_ex(self.handle, fptr(x), x.size, int(sample_rate), int(chunk_frames),
                                             resampler_code(resampler), C.byref(h)))
        return Voice(self, h.value)

    def resample(self, x: np.ndarray, sr_from: int, sr_to: int = 24000, resampler: str = "poly") -> np.ndarray:
        """The GPU resampler on its own (ptts_resample_ex)."""
        x = np.ascontiguousarray(x, np.float32).reshape(-1)
        code = resampler_code(resampler)
        n = lib().ptts_resample_len_ex(x.size, int(sr_from), int(sr_to), code)
        y = np.zeros(max(n, 1), np.float32)
        check(lib().ptts_resample_ex(self.handle, fptr(x), x.size, int(sr_from), int(sr_to), code, fptr(y)))
        return y[:n]

    # -- slots
    def open(self, slot: int, voice: Voice, ids, params: GenerationParams):
        a = np.ascontiguousarray(np.asarray(ids, np.int32).reshape(-1))
        cp = params.to_c()
        check(lib().ptts_slot_open(self.handle, slot, voice.handle, a.ctypes.data_as(C.POINTER(C.c_int32)), a.size,
                                   C.byref(cp)))

    def open_many(self, slots, voices, ids_list, params_list):
        """Batched admission (ptts_slots_open): row slots[i] <- (voices[i], ids_list[i], params_list[i])."""
        n = len(slots)
        sl = np.ascontiguousarray(np.asarray(slots, np.int32))
        arrs = [np.asarray(x, np.int32).reshape(-1) for x in ids_list]
        nid = np.ascontiguousarray(np.array([a.size for a in arrs], np.int32))
        cat = np.ascontiguousarray(np.concatenate(arrs) if arrs else np.zeros(0, np.int32))
        vh = (C.c_void_p * n)(*[v.handle for v in voices])
        ps = (GenParams * n)(*[p.to_c() for p in params_list])
        i32 = C.POINTER(C.c_int32)
        check(lib().ptts_slots_open(self.handle, n, sl.ctypes.data_as(i32), vh, cat.ctypes.data_as(i32),
                                    nid.ctypes.data_as(i32), ps))

    def close_slot(self, slot: int):
        check(lib().ptts_slot_close(self.handle, slot))

    def set_latent(self, slot: int, latent: np.ndarray):
        v = np.ascontiguousarray(latent, np.float32).reshape(LDIM)
        check(lib().ptts_slot_set_latent(self.handle, slot, fptr(v)))

    def decode_latents(self, slot: int, latents: np.ndarray) -> dict:
        """MimiModel::decode_from_latent of n FlowLM latents [n, 32] on a reset slot (idle engine):
        pcm [n, 1920], quantized [n, 512], after_upsample / after_transformer [n, 16, 512]."""
        lat = np.ascontiguousarray(latents, np.float32).reshape(-1, LDIM)
        n = lat.shape[0]
        out = {"pcm": np.zeros((n, FRAME), np.float32), "quantized": np.zeros((n, 512), np.float32),
               "after_upsample": np.zeros((n, 16, 512), np.float32),
               "after_transformer": np.zeros((n, 16, 512), np.float32)}
        check(lib().ptts_decode_latents(self.handle, slot, fptr(lat), n, fptr(out["pcm"]), fptr(out["quantized"]),
                                        fptr(out["after_upsample"]), fptr(out["after_transformer"])))
        return out

    # -- the batched hot path
    def step(self, n_rows: int) -> StepResult:
        r = StepResult(np.zeros((n_rows, FRAME), np.float32), np.zeros(n_rows, np.uint8), np.zeros(n_rows, np.uint8),
                       np.zeros(n_rows, np.float32), np.zeros((n_rows, LDIM), np.float32))
        check(lib().ptts_step(self.handle, n_rows, fptr(r.pcm), u8ptr(r.valid), u8ptr(r.last), fptr(r.eos_logits),
                              fptr(r.latents)))
        r.valid = r.valid.astype(bool)
        r.last = r.last.astype(bool)
        return r

    def step_async(self, n_rows: int):
        check(lib().ptts_step_async(self.handle, n_rows))

    def flush_async(self, n_rows: int):
        """A pipelined call that starts no frame (ptts_flush_async): drains the frames already
        computed without running front parts whose frames would be discarded."""
        check(lib().ptts_flush_async(self.handle, n_rows))

    def sync(self):
        check(lib().ptts_sync(self.handle))

    def fetch(self, n_rows: int, calls_back: int = 0) -> StepResult:
        """Outputs of the latest call (calls_back = 0) or of the call before it (1: a driver that
        keeps one call in flight)."""
        r = StepResult(np.empty((n_rows, FRAME), np.float32), np.zeros(n_rows, np.uint8), np.zeros(n_rows, np.uint8),
                       np.zeros(n_rows, np.float32), np.zeros((n_rows, LDIM), np.float32))
        check(lib().ptts_fetch_prev(self.handle, calls_back, n_rows, fptr(r.pcm), u8ptr(r.valid), u8ptr(r.last),
                                    fptr(r.eos_logits), fptr(r.latents)))
        r.valid = r.valid.astype(bool)
        r.last = r.last.astype(bool)
        return r

    def fetch_ready(self, calls_back: int = 0) -> bool:
        """fetch(calls_back=...) would not block (ptts_fetch_ready)."""
        r = C.c_int(0)
        check(lib().ptts_fetch_ready(self.handle, calls_back, C.byref(r)))
        return bool(r.value)

    def front_done(self, calls_back: int = 1, wait: bool = False) -> bool:
        """The FlowLM step of the call calls_back calls before the latest has run (ptts_front_done);
        wait=True blocks until it has."""
        r = C.c_int(0)
        check(lib().ptts_front_done(self.handle, calls_back, int(wait), C.byref(r)))
        return bool(r.value)

    def enable_preview(self, max_rows: int = 8):
        """First-frame previews (ptts_preview_enable, pipelined engines): the first frame of up to
        max_rows rows starting in one call is decoded right after their first FlowLM step, alone,
        so it does not wait frame_lag() calls; fetch_previews() returns them. 0 disables."""
        check(lib().ptts_preview_enable(self.handle, int(max_rows)))
        self._pv_slots = np.zeros(64, np.int32)
        self._pv_pcm = np.zeros((64, FRAME), np.float32)

    def fetch_previews(self, wait: bool = False) -> list[tuple[int, np.ndarray]]:
        """Completed first-frame previews, oldest first: (slot, pcm [1920]) pairs (fresh arrays).
        wait=False never blocks."""
        n = C.c_int(0)
        check(lib().ptts_preview_fetch(self.handle, int(wait), len(self._pv_slots),
                                       self._pv_slots.ctypes.data_as(C.POINTER(C.c_int)), fptr(self._pv_pcm),
                                       C.byref(n)))
        return [(int(self._pv_slots[i]), self._pv_pcm[i].copy()) for i in range(n.value)]

    def generate(self, slot: int, voice: Voice, ids, params: GenerationParams) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(ids, np.int32).reshape(-1))
        cap = params.max_frames * FRAME
        out = np.zeros(cap, np.float32)
        n = C.c_int(0)
        cp = params.to_c()
        check(lib().ptts_generate(self.handle, slot, voice.handle, a.ctypes.data_as(C.POINTER(C.c_int32)), a.size,
                                  C.byref(cp), fptr(out), cap, C.byref(n)))
        return out[: n.value]

    # -- measurement
    def plan(self, n_rows: int) -> list[tuple[str, float, float]]:
        """The step plan: (op name, algorithmic flops, algorithmic bytes) per launch."""
        buf = C.create_string_buffer(1 << 17)
        check(lib().ptts_plan_ops(self.handle, n_rows, buf, len(buf)))
        out = []
        for line in buf.value.decode().split("\n"):
            if line:
                name, fl, by = line.split("\t")
                out.append((name, float(fl), float(by)))
        return out

    def plan_ops(self, n_rows: int) -> list[str]:
        return [n for n, _, _ in self.plan(n_rows)]

    def time_kernel(self, n_rows: int, name: str, reps: int = 50) -> float:
        us = C.c_double(0)
        check(lib().ptts_time_kernel(self.handle, n_rows, name.encode(), reps, C.byref(us)))
        return us.value
