"""Model config (SURVEY §8(b) cfg_yaml): the reference loads its dimensions from
config/b6369a24.yaml (config.rs:1-124, TTSModel::load config.rs:111-115); this build compiles
them into the kernels and checks a given config against them (csrc/config.cpp).
tests/golden/b6369a24.yaml is the reference's config file, kept as test data."""

from pathlib import Path

import pytest

import pocket_tts_amd as pt

GOLDEN = Path(__file__).parent / "golden" / "b6369a24.yaml"


def _variant(tmp_path, old, new):
    text = GOLDEN.read_text()
    assert old in text
    p = tmp_path / "variant.yaml"
    p.write_text(text.replace(old, new, 1))
    return str(p)


def test_reference_config_matches_build():
    pt.Engine.check_config(str(GOLDEN))


@pytest.mark.parametrize("old,new,key", [
    ("    num_layers: 6", "    num_layers: 12", "flow_lm.transformer.num_layers"),
    ("    depth: 6", "    depth: 4", "flow_lm.flow.depth"),
    ("    - 5\n", "    - 8\n", "mimi.seanet.ratios"),
    ("    context: 250", "    context: 500", "mimi.transformer.context"),
    ("  frame_rate: 12.5", "  frame_rate: 25", "mimi.frame_rate"),
    ("  dtype: float32\n  flow:", "  dtype: bfloat16\n  flow:", "flow_lm.dtype"),
    ("    pad_mode: constant", "    pad_mode: reflect", "mimi.seanet.pad_mode"),
])
def test_other_variant_is_rejected_naming_the_key(tmp_path, old, new, key):
    with pytest.raises(pt.PocketTTSError, match=key.replace(".", r"\.")):
        pt.Engine.check_config(_variant(tmp_path, old, new))


def test_equal_values_in_other_spellings_pass(tmp_path):
    pt.Engine.check_config(_variant(tmp_path, "  frame_rate: 12.5", "  frame_rate: 12.50  # Hz"))
    pt.Engine.check_config(_variant(tmp_path, "    max_period: 10000", "    max_period: 1e4"))


def test_hash_inside_a_value_is_not_a_comment(tmp_path):
    """'#' opens a comment only after whitespace and outside quotes."""
    with pytest.raises(pt.PocketTTSError, match=r"pad_mode = constant#x"):
        pt.Engine.check_config(_variant(tmp_path, "    pad_mode: constant", "    pad_mode: constant#x"))
    with pytest.raises(pt.PocketTTSError, match=r"mimi\.dtype = 'float32 # x'"):
        pt.Engine.check_config(_variant(tmp_path, "  dtype: float32\n  sample_rate", "  dtype: 'float32 # x'\n  sample_rate"))
    pt.Engine.check_config(_variant(tmp_path, "    pad_mode: constant", "    pad_mode: constant   # zeros"))


def test_missing_key_and_file_fail(tmp_path):
    with pytest.raises(pt.PocketTTSError, match="missing mimi.quantizer.dimension"):
        pt.Engine.check_config(_variant(tmp_path, "    dimension: 32\n", ""))
    with pytest.raises(pt.PocketTTSError, match="cannot open"):
        pt.Engine.check_config(str(tmp_path / "absent.yaml"))


@pytest.mark.gpu
def test_gpu_engine_created_with_reference_config():
    eng = pt.Engine(device=0, max_slots=1, max_ctx=64, cfg_yaml=str(GOLDEN))
    eng.close()
    with pytest.raises(pt.PocketTTSError, match="num_heads"):
        pt.Engine(device=0, max_slots=1, max_ctx=64,
                  cfg_yaml=_variant(Path(__import__("tempfile").mkdtemp()), "    num_heads: 16", "    num_heads: 8"))
