/* pocket_tts.h - C ABI of the MI355X-native Pocket TTS engine (variant b6369a24).
 *
 * This is the drop-in boundary for the reference's generation hot path. The
 * reference (ykevinc/pocket-tts, Rust/Candle) has no operator registry; the
 * seams it exposes are the model-level API of `TTSModel`
 * (crates/pocket-tts/src/tts_model.rs) and the kernel-level forwards of
 * `FlowLMModel` / `MimiModel`. Each entry point below names the reference
 * interface it replaces. Plain pointers and sizes only; the engine owns all
 * device memory, the caller owns host buffers. Every function returns 0 on
 * success or a PTTS_ERR_* code; `ptts_last_error()` gives a thread-local
 * message (the reference maps its anyhow::Error the same way at the FFI edge:
 * crates/pocket-tts-bindings/src/lib.rs:17).
 *
 * Threading: calls on one engine are externally serialized, as in the
 * reference (tts_model.py:315-316; server state.rs:69). One engine per GPU.
 *
 * Measurement and test hooks with no reference counterpart (per-kernel timing, the step plan,
 * the overlap probe, the GEMM-core test entry) are declared in pocket_tts_probe.h, not here:
 * this header is only the drop-in boundary a reference maintainer binds.
 */
#ifndef POCKET_TTS_H
#define POCKET_TTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTTS_OK 0
#define PTTS_ERR_INVALID 1 /* bad argument / shape */
#define PTTS_ERR_HIP 2     /* HIP runtime error (no GPU, OOM, launch failure) */
#define PTTS_ERR_STATE 3   /* call not valid in the current slot/engine state */
#define PTTS_ERR_IO 4      /* weights file missing or malformed */

/* ABI version of this header. Bumped whenever a struct below changes layout (3: cfg_yaml was
 * appended to ptts_engine_config; 4: back_frames; 5: back_bf16; 6: that field became back_mfma, with
 * the bf16x6 f32 mode). A caller checks ptts_abi_version() ==
 * PTTS_ABI_VERSION before passing any struct: a library built from another header reads a
 * different layout. */
#define PTTS_ABI_VERSION 6
int ptts_abi_version(void);
/* Build id of the loaded library: the first 16 hex digits of the sha256 over the sources it was
 * built from (pocket-tts_amd/Makefile, BUILD_ID), with "+probes" appended for a measurement build
 * (-DPTTS_PROBES). Lets a test harness refuse a stale prebuilt binary. */
const char* ptts_build_id(void);

#define PTTS_FRAME_SAMPLES 1920 /* 24 kHz / 12.5 Hz (config/b6369a24.yaml:24-27) */
#define PTTS_LATENT_DIM 32
#define PTTS_MODEL_DIM 1024
#define PTTS_SAMPLE_RATE 24000

typedef struct ptts_engine ptts_engine;
typedef struct ptts_voice ptts_voice;

typedef struct ptts_engine_config {
  int device;           /* HIP device ordinal (one engine per GPU) */
  int max_slots;        /* concurrent utterances (batch rows) */
  int max_ctx;          /* FlowLM KV capacity per slot, positions (voice + text + frames) */
  int lsd_decode_steps; /* TTSModel.lsd_decode_steps (tts_model.rs:22-49), engine-wide */
  uint64_t synth_seed;  /* synthetic weights (tests/golden/synth.py rule) if weights_path == NULL */
  const char* weights_path; /* local safetensors with TTSModel state-dict names, or NULL */
  void* weight_blob;        /* optional caller-owned device buffer of ptts_weight_blob_bytes() */
  int defer_weights;        /* 1: leave the blob unfilled; caller fills it (e.g. RCCL broadcast)
                               and then calls ptts_engine_finalize() */
  int pipeline;             /* 0: each ptts_step returns the frame it computed.
                               1: overlapped stepping - the Mimi decode of frame k runs on a
                               second stream concurrently with the FlowLM step of frame k+1, so a
                               call returns the frame computed by the PREVIOUS call (one extra
                               call drains the last frame; the first call after admission
                               returns no frame for the admitted rows). */
  int weight_quant;         /* PTTS_QUANT_*: the reference's weight quantization (quantize.rs,
                               QuantizeConfig::default(): symmetric per-tensor int8 levels) applied
                               when the weights are packed (TTSModel::load_quantized*,
                               tts_model.rs:108-171). The FlowLM step GEMMs then stream int8 codes
                               (float(q) * scale rebuilt in-kernel = the simulated f32 weight).
                               A deferred blob must have been packed with the same mode. */
  int fp8_gemm;             /* 1: the large FlowLM step GEMMs (qkv, linear1, linear2, adaLN) run
                               as fp8 W8A8 on v_mfma_f32_32x32x16_fp8_fp8: OCP e4m3 weight codes
                               with one scale per output row, activations quantized in-kernel per
                               (row, K slice). Not a reference numeric (the reference has no fp8;
                               BASELINE configs[4]): gated on accuracy vs the f32 path. Requires
                               weight_quant = PTTS_QUANT_NONE. 0 = f32 (default). */
  const char* cfg_yaml;     /* the reference's model config (config/b6369a24.yaml; TTSModel::load's
                               config, config.rs:111-115), or NULL. The kernels implement the
                               b6369a24 dimensions; when given, every hot-path key of the file must
                               be present and equal them, or creation fails (PTTS_ERR_INVALID,
                               naming the key): another variant is a rebuild. Checked, not read
                               for shapes. ptts_config_check() is the same check alone. */
  int back_frames;          /* pipelined engines only: frames per Mimi-decode pass, 1 (default;
                               0 means 1), 2, 4 or 8. With n > 1, frames n j .. n j + n - 1 of every
                               row are decoded by ONE back pass (the streaming codec state advances
                               as for n passes; PCM identical within float rounding), a call
                               returns the frame computed 2 n - 1 calls earlier, and rows admitted
                               inside a pass start at the next pass boundary (an utterance's frames
                               group into passes from its first). ptts_frame_lag() reports both
                               delays. 2 is the throughput setting (bench.py's default; 4 measured
                               in DESIGN.md section 14), 1 the low-latency one. */
  int back_mfma;            /* PTTS_BACK_*: how the Mimi decoder transformer GEMMs and the SEANet
                               decoder convs (the back part, at >= 16 rows) use the matrix cores.
                               PTTS_BACK_F32 (0): v_mfma_f32_32x32x2_f32, an exact f32 FMA chain.
                               PTTS_BACK_F32X6 (2): f32 products on the bf16 matrix pipe: each f32
                               operand as the exact sum of three bf16 pieces, the six piece products
                               of order <= 2 summed in f32 (dropped terms < 2^-24 |a b|): f32
                               accuracy (the GEMM-core tests hold it to the f32 tile's error against
                               fp64), 6 bf16 MFMAs per 16 k instead of 8 f32 ones.
                               PTTS_BACK_BF16 (1): operands rounded to bf16, f32 accumulation: NOT a
                               reference numeric (Candle runs f32), gated on PCM accuracy.
                               The latents, EOS logits and stop frames never depend on it (the back
                               part does not feed the FlowLM). */
} ptts_engine_config;

#define PTTS_BACK_F32 0
#define PTTS_BACK_BF16 1
#define PTTS_BACK_F32X6 2

#define PTTS_QUANT_NONE 0
#define PTTS_QUANT_FLOW_LM 1 /* quantize_weights() over the flow_lm.* tensors */
#define PTTS_QUANT_ALL 2     /* ... over the whole state dict (Mimi included) */

/* Per-utterance generation parameters: TTSModel's public fields temp / eos_threshold /
 * noise_clamp (tts_model.rs:22-49) plus what generate_stream_segment derives from the text
 * (max_gen_len = (words+2)*13, frames_after_eos: tts_model.rs:968-969,1230-1237). */
typedef struct ptts_gen_params {
  float temp;            /* noise std = sqrt(temp); 0 = deterministic (flow_lm.rs:39-65) */
  float eos_threshold;   /* EOS when out_eos logit > threshold (flow_lm.rs:139-145) */
  float noise_clamp;     /* <= 0: None; else truncated normal |x| <= clamp */
  int frames_after_eos;  /* frames yielded after the EOS step (5 if <=4 words else 3) */
  int max_frames;        /* max_gen_len */
  uint64_t seed;         /* noise stream seed for this utterance */
} ptts_gen_params;

/* Size of the packed device weight blob (all tensors, engine layout). */
size_t ptts_weight_blob_bytes(void);
/* Pack the weights (synthetic from synth_seed when weights_path is NULL/empty, else a local
 * safetensors file with TTSModel state-dict names) into a host buffer of at least
 * ptts_weight_blob_bytes(), in the engine's device layout. Host only: no GPU needed. A
 * multi-GPU launcher packs once, broadcasts the blob (RCCL) into every rank's engine buffer
 * (cfg.weight_blob + defer_weights) and calls ptts_engine_finalize(). Replaces the per-process
 * VarBuilder load of TTSModel::load_with_params_device (tts_model.rs:86-106). */
int ptts_pack_weights(uint64_t synth_seed, const char* weights_path, float* host_out, size_t n_bytes);
/* The checkpoint tensors the packer reads, one line each: "name\tdim0,dim1,...\n" (TTSModel
 * state-dict keys: flow_lm.* and mimi.*, the VarBuilder prefixes of tts_model.rs:279-426, with the
 * checkpoint's own shapes). A weights file needs exactly these (extra tensors, e.g. the dropped
 * VQ codebooks, are ignored; F32, BF16 or F16). *needed = bytes incl. the terminating 0. Host only. */
int ptts_weight_manifest(char* buf, size_t cap, size_t* needed);
/* Same with the reference's weight quantization applied (weight_quant = PTTS_QUANT_*;
 * quantize.rs:126-150 quantize_weights with QuantizeConfig::default()). */
int ptts_pack_weights_ex(uint64_t synth_seed, const char* weights_path, int weight_quant, float* host_out,
                         size_t n_bytes);
/* The quantizer alone (QuantizedTensor::quantize, quantize.rs:66-90): out = simulated values,
 * *scale = the per-tensor scale. Host only. */
int ptts_quantize_tensor(const float* x, size_t n, int num_levels, float* out, float* scale);
/* 1 if quantize_weights() with QuantizeConfig::default() quantizes tensor `name` of `numel`
 * elements in scope `weight_quant` (should_skip_layer + min_size, quantize.rs:120-150). */
int ptts_quant_applies(const char* name, size_t numel, int weight_quant);
/* Number of FlowLM GEMM weight matrices the engine streams as int8 codes (0 when not quantized). */
int ptts_engine_int8_matrices(ptts_engine* e);
/* Number of FlowLM GEMM weight matrices running on the fp8 path (fp8_gemm = 1), else 0. */
int ptts_engine_fp8_matrices(ptts_engine* e);

/* TTSModel::load / load_with_params_device (tts_model.rs:59-106,182-236). */
int ptts_engine_create(const ptts_engine_config* cfg, ptts_engine** out);
/* The cfg_yaml check of ptts_engine_create without an engine (no GPU needed): 0 if the model
 * config at `cfg_yaml` states the dimensions this build implements (config.rs:1-124 keys). */
int ptts_config_check(const char* cfg_yaml);
/* Second half of create when cfg->defer_weights = 1 (derived tables, time embeddings). */
int ptts_engine_finalize(ptts_engine* e);
void ptts_engine_destroy(ptts_engine* e);
/* Copy a host blob from ptts_pack_weights[_ex] into a deferred engine's weight buffer (the
 * single-process alternative to a device-side fill); call ptts_engine_finalize() after it. */
int ptts_engine_load_blob(ptts_engine* e, const float* host_blob, size_t n_bytes);
/* Device pointer of the packed weight blob (for the caller's RCCL broadcast). */
void* ptts_engine_weight_blob(ptts_engine* e);

/* TTSModel::get_voice_state_from_prompt_tensor (tts_model.rs:490-501): prefill an
 * `audio_prompt` [n_frames x 1024] (row-major, host) into an immutable voice KV prefix. */
int ptts_voice_from_prompt(ptts_engine* e, const float* prompt, int n_frames, ptts_voice** out);
/* TTSModel::get_voice_state_from_tensor (tts_model.rs:504-560): 24 kHz mono PCM ->
 * Mimi encoder -> speaker projection -> FlowLM prefill. n_samples is zero-padded to a
 * multiple of 1920. */
int ptts_voice_from_pcm(ptts_engine* e, const float* pcm, int n_samples, ptts_voice** out);
/* The voice-cloning front end of TTSModel::get_voice_state / get_voice_state_from_bytes
 * (tts_model.rs:428-463) after the WAV decode, then get_voice_state_from_tensor (:504-577):
 * `n_samples` mono samples at `sample_rate` Hz are resampled to 24 kHz on the GPU by the
 * resample_poly rule of the Python reference's convert_audio (audio_utils.py:8-28: the rule the
 * reference's own ref.wav -> ref_mimi_input pair was made with), zero-padded to whole frames and
 * encoded. The Rust driver resamples with rubato's FastFixedIn instead (audio.rs:210-231), a
 * deliberate divergence: its parity with this path is unpinned.
 * chunk_frames = TTSModel.voice_prompt_chunk_frames: the encoder chunk length in frames; 0 = the
 * reference's adaptive rule (adaptive_voice_prompt_chunk_frames, tts_model.rs:562-577: whole
 * prompt up to 120 frames, then 120/180/240), < 0 = one pass (the Python reference,
 * tts_model.py:258-262). Each chunk re-applies the downsample conv's replicate padding, as the
 * Rust driver's step=0 per chunk does (tts_model.rs:536-541, conv.rs:116-123).
 * ptts_voice_from_pcm(e, pcm, n, out) == ptts_voice_from_audio(e, pcm, n, 24000, 0, out). */
int ptts_voice_from_audio(ptts_engine* e, const float* samples, int n_samples, int sample_rate, int chunk_frames,
                          ptts_voice** out);
/* The GPU resampler alone (audio.rs:197-255 `resample` for one channel): y receives
 * ptts_resample_len(n_samples, sr_from, sr_to) samples = ceil(n * up / down) with up/down the
 * rates divided by their gcd. */
int ptts_resample_len(int n_samples, int sr_from, int sr_to);
int ptts_resample(ptts_engine* e, const float* x, int n_samples, int sr_from, int sr_to, float* y);
/* Resampler choice of the _ex entry points below. PTTS_RESAMPLE_POLY is the rule above (the
 * default everywhere). PTTS_RESAMPLE_RUBATO_SEPTIC is the Rust driver's own resample()
 * (audio.rs:197-255): rubato 0.14.1 FastFixedIn, PolynomialDegree::Septic, ratio sr_to / sr_from,
 * one process() call over the whole input, output kept as rubato returns it (no delay
 * compensation, no trim). Its source is not in the reference: the restated algorithm (kernels.h
 * septic_schedule, oracle/ptts_oracle.c orc_resample_septic) is parity-unpinned. Equal rates
 * return the input unchanged for both, as audio.rs:198-200 does. */
#define PTTS_RESAMPLE_POLY 0
#define PTTS_RESAMPLE_RUBATO_SEPTIC 1
/* Output length of the chosen resampler (0 if the arguments are invalid); for the rubato rule the
 * count of its position walk, about (n - 5) * sr_to / sr_from. */
int ptts_resample_len_ex(int n_samples, int sr_from, int sr_to, int resampler);
int ptts_resample_ex(ptts_engine* e, const float* x, int n_samples, int sr_from, int sr_to, int resampler, float* y);
/* ptts_voice_from_audio with the resampler chosen; ptts_voice_from_audio(...) ==
 * ptts_voice_from_audio_ex(..., PTTS_RESAMPLE_POLY, out). */
int ptts_voice_from_audio_ex(ptts_engine* e, const float* samples, int n_samples, int sample_rate, int chunk_frames,
                             int resampler, ptts_voice** out);
/* Conditioning rows the voice holds (frames). */
int ptts_voice_len(const ptts_voice* v);
/* The [n_frames x 1024] conditioning a PCM voice was built from (host copy); for tests. */
int ptts_voice_conditioning(const ptts_voice* v, float* out, int max_rows);
void ptts_voice_destroy(ptts_voice* v);

/* Admission of one utterance into batch row `slot` = the per-segment prologue of
 * generate_stream_segment (tts_model.rs:938-1004): copy the voice KV prefix, embed and
 * prefill `n_ids` text tokens (text.rs:289-303), reset the Mimi state, backbone = bos_emb. */
int ptts_slot_open(ptts_engine* e, int slot, const ptts_voice* v, const int32_t* ids, int n_ids,
                   const ptts_gen_params* p);
/* Batched admission of n utterances (distinct slots) in one call: voices[i], params[i] and
 * n_ids[i] tokens taken in order from the concatenated `ids`. Same per-row result as n
 * ptts_slot_open calls; the text prefills of all rows share one pass (the server admitting a
 * burst of requests, or a batch job starting). */
int ptts_slots_open(ptts_engine* e, int n, const int* slots, const ptts_voice* const* voices, const int32_t* ids,
                    const int* n_ids, const ptts_gen_params* params);
int ptts_slot_close(ptts_engine* e, int slot);

/* THE batched hot path: one iteration of the loop body of generate_stream_segment
 * (tts_model.rs:1006-1070) for rows [0, n_rows): FlowLM step -> EOS -> flow sampling ->
 * denorm/quantize -> Mimi decode -> 1920 PCM samples per active row.
 * Host outputs (each may be NULL):
 *   pcm [n_rows x 1920], frame_valid [n_rows] (row was active this step),
 *   last [n_rows] (this was the row's final frame: EOS tail reached or max_frames),
 *   eos_logits [n_rows], latents [n_rows x 32] (the sampled latent of this step). */
int ptts_step(ptts_engine* e, int n_rows, float* pcm, uint8_t* frame_valid, uint8_t* last,
              float* eos_logits, float* latents);
/* Same step, enqueued only (outputs stay in HBM); use ptts_sync() + ptts_fetch(). */
int ptts_step_async(ptts_engine* e, int n_rows);
/* Pipelined engines: a call that starts no frame. The frames already computed advance through
 * the back part and are returned as by ptts_step_async (fetch after it as usual), but no row
 * computes a new frame: every row pauses for this call, as rows past n_rows do. A caller whose
 * rows have all finished drains the pipeline with it (ptts_frame_lag() calls) without running
 * front parts whose frames would be discarded. Not valid right after an admission
 * (PTTS_ERR_INVALID: the admitted rows' first frame must fall on a step call). No reference
 * counterpart (the reference does not pipeline). */
int ptts_flush_async(ptts_engine* e, int n_rows);
int ptts_sync(ptts_engine* e);
int ptts_fetch(ptts_engine* e, int n_rows, float* pcm, uint8_t* frame_valid, uint8_t* last,
               float* eos_logits, float* latents);
/* Calls by which a frame trails the call that computed its FlowLM step: 0 (sequential), 1
 * (pipelined), 2 n - 1 (pipelined, back_frames = n > 1). *admit_delay (may be NULL): the calls by
 * which the rows of the latest admission start late (back_frames = n > 1, admitted at a call k with
 * k % n != 0: n - k % n), else 0. A row admitted before call k returns its first frame from call
 * k + lag + admit_delay. */
int ptts_frame_lag(const ptts_engine* e, int* admit_delay);
/* ptts_fetch of an earlier call: calls_back = 0 is the latest call (= ptts_fetch), 1 the call
 * before it. Lets a driver keep one call in flight (issue call k+1, then fetch call k) so that the
 * GPU always has the next step queued while the host hands out frames. calls_back <= 1. */
int ptts_fetch_prev(ptts_engine* e, int calls_back, int n_rows, float* pcm, uint8_t* frame_valid, uint8_t* last,
                    float* eos_logits, float* latents);
/* *ready = 1 if ptts_fetch_prev(e, calls_back, ..) would return without waiting (the call's frame
 * is complete), else 0; never blocks. A driver that also serves previews polls this and
 * ptts_preview_fetch instead of blocking in the fetch. */
int ptts_fetch_ready(ptts_engine* e, int calls_back, int* ready);
/* *done = 1 once the FlowLM step (front part) of the call calls_back (0..3) calls before the latest
 * has run on the GPU; wait = 1 blocks until it has. Pipelined engines let the host run calls ahead
 * of the GPU; a driver that admits new rows waits here (calls_back = 1) before its next call, so an
 * admission queues behind one FlowLM step at most (first-chunk latency), while the GPU still has
 * the next step queued. Calls are tracked from an engine's first ptts_front_done on (each later
 * call records an event after its front part; a driver that never asks pays no marker per call):
 * a call issued before that is answered from the front stream as a whole (done once everything
 * queued on it has run), which can only be later, never earlier, than its own front part. */
int ptts_front_done(ptts_engine* e, int calls_back, int wait, int* done);
/* First-frame previews (pipelined engines; no reference counterpart: the reference decodes each
 * frame right after its FlowLM step, tts_model.rs:1040-1047, and does not pipeline). With
 * max_rows > 0 (at most 8), the first frame of up to max_rows rows that start in one call is also
 * decoded right after that call's FlowLM step, alone, from the fresh Mimi state every utterance
 * starts from, so the first chunk of a new stream does not wait ptts_frame_lag() calls. The rows'
 * regular first frame still arrives through ptts_fetch (within float rounding of the preview); a
 * caller delivers whichever comes first. 0 disables. PTTS_ERR_INVALID on a sequential engine. */
int ptts_preview_enable(ptts_engine* e, int max_rows);
/* Completed previews, oldest first: *n_out frames, slot slots[i] and pcm [i][1920] (at most
 * max_n; a preview's rows are returned together). wait = 0: only those already complete (never
 * blocks); 1: blocks until the launched previews complete (as many as fit in max_n). A slot
 * re-admitted or closed before its preview is fetched drops that preview. */
int ptts_preview_fetch(ptts_engine* e, int wait, int max_n, int* slots, float* pcm, int* n_out);
/* Test hook (teacher forcing): overwrite the backbone input latent of `slot`. */
int ptts_slot_set_latent(ptts_engine* e, int slot, const float* latent32);
/* MimiModel::decode_from_latent (mimi.rs:143-157) after the denorm + DummyQuantizer of
 * tts_model.rs:1033-1038 (the kernel-level seam of SURVEY §8(b)): n_frames FlowLM latents
 * [n][32] decoded in sequence on `slot`'s streaming state, which is reset first; every pending
 * frame of the engine is dropped (call on an idle engine). Outputs (each optional, NULL = skip):
 * pcm [n][1920]; quantized [n][512]; after_upsample and after_transformer [n][16][512]
 * (time-major; the reference's tensors are [1][512][16]). */
int ptts_decode_latents(ptts_engine* e, int slot, const float* latents, int n_frames, float* pcm, float* quantized,
                        float* after_upsample, float* after_transformer);

/* TTSModel::generate for one segment (tts_model.rs:687-703) on row `slot`: loops ptts_step
 * until the row's last frame. pcm_out receives up to max_samples samples. */
int ptts_generate(ptts_engine* e, int slot, const ptts_voice* v, const int32_t* ids, int n_ids,
                  const ptts_gen_params* p, float* pcm_out, int max_samples, int* n_samples);

const char* ptts_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
