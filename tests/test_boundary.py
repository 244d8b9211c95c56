"""CPU: the C-ABI library builds/loads, exports every symbol include/pocket_tts.h declares,
and fails loudly (no CPU fallback) when no GPU is visible. Host-logic KATs mirror the
reference's inline unit tests (tts_model.rs:1239-1299)."""

import ctypes as C
import re

import numpy as np
import pytest
from conftest import ROOT


def declared_symbols(header="pocket_tts.h"):
    text = (ROOT / "include" / header).read_text()
    return sorted(set(re.findall(r"\b(ptts_[a-z0-9_]+)\s*\(", text)))


PROBE_HOOKS = {"ptts_test_gemm", "ptts_time_kernel", "ptts_plan_ops", "ptts_probe_overlap"}


def test_boundary_header_holds_no_measurement_hooks():
    """pocket_tts.h is the drop-in boundary only; the measurement / test hooks live
    in pocket_tts_probe.h."""
    assert not PROBE_HOOKS & set(declared_symbols())
    assert set(declared_symbols("pocket_tts_probe.h")) == PROBE_HOOKS


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["ptts_engine_create", "ptts_voice_from_prompt", "ptts_voice_from_pcm", "ptts_slot_open", "ptts_step",
              "ptts_generate", "ptts_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from pocket_tts_amd import _lib

    L = _lib.lib()
    declared = set(declared_symbols()) | set(declared_symbols("pocket_tts_probe.h"))
    for s in declared:
        assert hasattr(L, s), s
    assert {n for n, _, _ in _lib.SIGNATURES} == declared


def test_blob_size_is_the_packed_model():
    from pocket_tts_amd import Engine

    n = Engine.weight_blob_bytes()
    # 89.4M FlowLM + 27.9M Mimi parameters, fp32, plus padding (<1%)
    assert 117_000_000 * 4 < n < 119_000_000 * 4


def test_engine_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import pocket_tts_amd as pt

    with pytest.raises(pt.PocketTTSError) as e:
        pt.Engine(device=0, max_slots=1, max_ctx=64)
    assert e.value.code == 2  # PTTS_ERR_HIP


def test_null_arguments_rejected():
    from pocket_tts_amd import _lib

    L = _lib.lib()
    assert L.ptts_engine_create(None, None) == 1
    assert L.ptts_step(None, 1, None, None, None, None, None) == 1
    assert b"null" in L.ptts_last_error()


def test_prepare_text_prompt_kats():
    from pocket_tts_amd import estimate_frames_after_eos, max_gen_len, prepare_text_prompt

    assert prepare_text_prompt("hello world") == "        Hello world."
    assert prepare_text_prompt("Hello world.") == "        Hello world."
    assert prepare_text_prompt("  hello  ") == "        Hello."
    assert prepare_text_prompt("one two three four five") == "One two three four five."
    assert estimate_frames_after_eos("Hello world") == 5
    assert estimate_frames_after_eos("One two three four five") == 3
    assert max_gen_len(prepare_text_prompt("Hello, world!")) == (2 + 2) * 13


def test_generation_params_marshalling():
    from pocket_tts_amd import GenerationParams

    p = GenerationParams(temp=0.5, eos_threshold=float("inf"), noise_clamp=None, frames_after_eos=5, max_frames=7,
                         seed=2**64 - 1).to_c()
    assert p.noise_clamp == 0.0 and p.max_frames == 7 and p.seed == 2**64 - 1 and np.isinf(p.eos_threshold)


def test_library_is_built_from_these_sources():
    """The .so carries the hash of the sources it was built from (Makefile BUILD_ID): a stale
    prebuilt binary (or a -DPTTS_PROBES measurement build) is refused by every GPU session."""
    import pocket_tts_amd as pt
    from pocket_tts_amd import _lib

    assert _lib.lib().ptts_abi_version() == _lib.ABI_VERSION == 6
    assert len(pt.source_build_id()) == 16
    assert pt.build_id() == pt.source_build_id()
    assert pt.check_build_id() == pt.build_id()
