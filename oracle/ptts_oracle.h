/* TEST INFRASTRUCTURE ONLY - CPU oracle for the Pocket TTS hot path.
 *
 * A plain-C fp32 restatement of the reference's algorithm
 * (ykevinc/pocket-tts, variant b6369a24), used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker.
 * Nothing in the product (pocket-tts_amd/) links, loads or calls it.
 *
 * Parity pinning: checked against the fixtures in tests/golden/, which were
 * produced by the reference's own Python modules (tests/golden/gen_golden.py)
 * with the Candle-semantics GELU switch.
 */
#ifndef PTTS_ORACLE_H
#define PTTS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_model orc_model;
typedef struct orc_state orc_state;

/* Build the b6369a24 model with synthetic weights (tests/golden/synth.py rule). */
orc_model* orc_model_create(uint64_t seed);
/* Same, with the reference's weight quantization applied to the synthetic weights
 * (quantize.rs quantize_weights + QuantizeConfig::default()): quant 0 none, 1 the flow_lm.*
 * tensors, 2 every tensor. */
orc_model* orc_model_create_ex(uint64_t seed, int quant);
/* quantize.rs restatements: QuantizedTensor::quantize (returns the scale; out may alias x) and
 * the quantize_weights selection rule. */
float orc_quantize(const float* x, int64_t n, int num_levels, float* out);
int orc_quant_applies(const char* name, int64_t numel, int mode);
void orc_model_destroy(orc_model* m);
/* First n elements of a synthetic tensor (PRNG pinning). Returns 0 on success. */
int orc_synth_head(uint64_t seed, const char* name, const int64_t* shape, int ndim, float* out, int64_t n);

/* Per-utterance streaming state: FlowLM KV (linear, cap max_ctx) + Mimi decoder state. */
orc_state* orc_state_create(const orc_model* m, int max_ctx);
void orc_state_destroy(orc_state* s);
int orc_state_pos(const orc_state* s);

/* FlowLM transformer over T conditioning rows [T x 1024] (voice prompt / text embeddings);
 * tts_model.rs:580-599 and :958-964. */
void orc_prefill(const orc_model* m, orc_state* s, const float* x, int T);
void orc_prefill_tokens(const orc_model* m, orc_state* s, const int32_t* ids, int S);
/* Embedding gather only (text.rs:289-303). out: [S x 1024]. */
void orc_embed_tokens(const orc_model* m, const int32_t* ids, int S, float* out);

/* One step of generate_stream_segment's loop (tts_model.rs:1006-1070).
 * latent_in: [32] previous latent, NULL = bos_emb.
 * noise: [32] initial flow sample x_0 (NULL = zeros, i.e. temperature 0).
 * Outputs (any may be NULL): tout [1024], eos_logit [1], latent [32], pcm [1920],
 * quantized [512], after_upsample [16 x 512], after_tr [16 x 512] (time-major). */
void orc_step(const orc_model* m, orc_state* s, const float* latent_in, const float* noise,
              int lsd_steps, float* tout, float* eos_logit, float* latent, float* pcm,
              float* quantized, float* after_upsample, float* after_tr);

/* Mimi decode of one latent frame only (mimi.rs:143-157 + tts_model.rs:1033-1038). */
void orc_mimi_decode(const orc_model* m, orc_state* s, const float* latent, float* pcm);

/* Voice cloning front half: PCM (24 kHz, n multiple of 1920) -> conditioning [n/1920 x 1024]
 * (tts_model.py:258-262; mimi.py:88-111). Intermediates optional (time-major). */
void orc_encode(const orc_model* m, const float* pcm, int n, float* cond,
                float* after_encoder, float* after_encoder_tr, float* latent);

/* Same, with the Rust driver's chunking (tts_model.rs:520-541): chunk_frames frames per
 * encode_to_latent call, each with step=0 (replicate padding re-applied per chunk);
 * chunk_frames <= 0: one pass. */
void orc_encode_ex(const orc_model* m, const float* pcm, int n, int chunk_frames, float* cond,
                   float* after_encoder, float* after_encoder_tr, float* latent);

/* scipy resample_poly rule (audio_utils.py:8-28): output length, and the resampled signal
 * (returns its length). */
int orc_resample_len(int n, int sr_from, int sr_to);
int orc_resample(const float* x, int n, int sr_from, int sr_to, float* y);
/* The Rust driver's resampler instead (audio.rs:197-255: rubato 0.14.1 FastFixedIn, Septic, one
 * process() call over the whole input), restated from rubato's published algorithm (its source is
 * not in the reference: parity unpinned). Equal rates copy. Returns the output length. */
int orc_resample_septic_len(int n, int sr_from, int sr_to);
int orc_resample_septic(const float* x, int n, int sr_from, int sr_to, float* y);

/* Time-embedding table for lsd_steps (mlp.rs:296-319): out [lsd_steps x 512]. */
void orc_time_embeddings(const orc_model* m, int lsd_steps, float* out);

/* CPU baseline: n_utt independent utterances (prompt F rows, S ids), n_frames forced steps each,
 * parallel over utterances with `threads` OpenMP threads. Returns wall seconds of the step loop. */
double orc_bench(const orc_model* m, int n_utt, int F, int S, int n_frames, int threads);

#ifdef __cplusplus
}
#endif
#endif
