"""MI355X-native Pocket TTS (variant b6369a24): HIP engine + host mirror of the reference API."""

from ._lib import (BACK_BF16, BACK_F32, BACK_F32X6, FRAME, LIB_PATH, QUANT_ALL, QUANT_FLOW_LM, QUANT_NONE, SAMPLE_RATE, PocketTTSError, build_id,
                   check_build_id, lib, source_build_id)
from .engine import Engine, GenerationParams, StepResult, Voice
from .quantize import QuantizeConfig, QuantizedTensor, calculate_snr, quantize_weights
from .text import (Tokenizer, estimate_frames_after_eos, load_tokenizer, max_gen_len, prepare_text_prompt,
                   split_into_best_sentences)
from .tts_model import TTSModel

__all__ = ["Engine", "GenerationParams", "StepResult", "Voice", "TTSModel", "PocketTTSError", "FRAME",
           "SAMPLE_RATE", "LIB_PATH", "lib", "build_id", "source_build_id", "check_build_id", "prepare_text_prompt", "estimate_frames_after_eos", "max_gen_len",
           "Tokenizer", "load_tokenizer", "split_into_best_sentences", "QuantizeConfig", "QuantizedTensor",
           "quantize_weights", "calculate_snr", "QUANT_NONE", "QUANT_FLOW_LM", "QUANT_ALL", "BACK_F32", "BACK_BF16",
           "BACK_F32X6"]
