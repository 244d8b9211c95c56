/* TEST INFRASTRUCTURE ONLY - CPU oracle (checker) for the Pocket TTS hot path.
 * See ptts_oracle.h. Plain C99 + OpenMP, fp32 everywhere (the reference
 * computes in fp32: tts_model.rs:190,202-203).
 *
 * Citations are to /root/reference (ykevinc/pocket-tts):
 *   crates/pocket-tts/src/... (Rust/Candle, the behaviour we follow) and
 *   python-reference/pocket_tts/... (the fixture generator's code path).
 */
#include "ptts_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---- configuration: config/b6369a24.yaml:6-56, tts_model.rs:291-293,389-390 ---- */
enum {
  D = 1024, NH = 16, HD = 64, NL = 6, FF = 4096, LDIM = 32, VOCAB = 4001,
  FD = 512, FDEPTH = 6, FREQ = 256,
  MD = 512, MNH = 8, MNL = 2, MFF = 2048, MCTX = 250, UP = 16, FRAME = 1920,
  RING = 512 /* >= MCTX + UP */
};

/* ---------------- synthetic weights (tests/golden/synth.py) ---------------- */
static uint64_t fnv1a64(const char* s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (; *s; ++s) { h ^= (unsigned char)*s; h *= 0x100000001B3ull; }
  return h;
}
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static int contains(const char* s, const char* t) { return strstr(s, t) != NULL; }
static int ends_with(const char* s, const char* t) {
  size_t a = strlen(s), b = strlen(t);
  return a >= b && strcmp(s + a - b, t) == 0;
}
/* init_rule() of synth.py: returns 0 if the tensor is not random (computed buffer). */
static int init_rule(const char* name, const int64_t* shape, int nd, double* c, double* hw) {
  const char* leaf = strrchr(name, '.');
  leaf = leaf ? leaf + 1 : name;
  if (!strcmp(leaf, "freqs")) return 0;
  if (ends_with(name, "emb_std")) { *c = 1.0; *hw = 0.1; return 1; }
  if (ends_with(name, "emb_mean")) { *c = 0.0; *hw = 0.1; return 1; }
  if (ends_with(name, "bos_emb")) { *c = 0.0; *hw = sqrt(3.0); return 1; }
  if (ends_with(name, "conditioner.embed.weight")) { *c = 0.0; *hw = 1.0; return 1; }
  if (!strcmp(leaf, "alpha")) { *c = 1.0; *hw = 0.1; return 1; }
  if (!strcmp(leaf, "scale") && contains(name, "layer_scale")) { *c = 0.01; *hw = 0.005; return 1; }
  int is_norm = contains(name, "norm1.") || contains(name, "norm2.") || contains(name, "out_norm.") ||
                contains(name, "in_ln.");
  if (is_norm && !strcmp(leaf, "weight")) { *c = 1.0; *hw = 0.1; return 1; }
  if (is_norm && !strcmp(leaf, "bias")) { *c = 0.0; *hw = 0.1; return 1; }
  if (!strcmp(leaf, "bias")) { *c = 0.0; *hw = 0.05; return 1; }
  if (nd >= 2) {
    int64_t fan = 1;
    for (int i = 1; i < nd; ++i) fan *= shape[i];
    *c = 0.0; *hw = 1.0 / sqrt((double)fan);
    return 1;
  }
  return -1;
}
static void synth_fill(uint64_t seed, const char* name, const int64_t* shape, int nd, float* out,
                       int64_t n) {
  double c = 0, hw = 0;
  int r = init_rule(name, shape, nd, &c, &hw);
  if (r <= 0) { fprintf(stderr, "oracle: no init rule for %s\n", name); abort(); }
  uint64_t base = seed * 0x9E3779B97F4A7C15ull + fnv1a64(name);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t z = mix64(base + (uint64_t)i * 0xD1B54A32D192ED03ull);
    double u = (double)(z >> 40) * (1.0 / 16777216.0);
    out[i] = (float)(c + (2.0 * u - 1.0) * hw);
  }
}
int orc_synth_head(uint64_t seed, const char* name, const int64_t* shape, int ndim, float* out,
                   int64_t n) {
  double c, hw;
  if (init_rule(name, shape, ndim, &c, &hw) <= 0) return -1;
  synth_fill(seed, name, shape, ndim, out, n);
  return 0;
}

/* ---------------- model ---------------- */
typedef struct { float *in_proj, *out_proj, *n1w, *n1b, *n2w, *n2b, *l1, *l2, *ls1, *ls2; } Layer;
typedef struct { float *w, *b; int cin, cout, k, stride; } Conv; /* w repacked [cout][k][cin] */
typedef struct { float *w, *b; int cin, cout, r; float* wp; } ConvTr; /* w as torch [cin][cout][2r];
                                                                     ORC_FAST: wp = [cout][2r][cin] */

struct orc_model {
  uint64_t seed;
  int quant; /* weight quantization scope: 0 none, 1 flow_lm.*, 2 all (quantize.rs) */
  /* FlowLM (flow_lm.rs:24-37) */
  float *embed, *bos, *emb_mean, *emb_std, *input_linear, *out_norm_w, *out_norm_b, *eos_w, *eos_b;
  Layer fl[NL];
  /* flow head SimpleMLPAdaLN (mlp.rs:215-223) */
  float *te_l1w[2], *te_l1b[2], *te_l2w[2], *te_l2b[2], *te_alpha[2];
  float *cond_w, *cond_b, *inproj_w, *inproj_b;
  float *rb_lnw[FDEPTH], *rb_lnb[FDEPTH], *rb_w0[FDEPTH], *rb_b0[FDEPTH], *rb_w2[FDEPTH], *rb_b2[FDEPTH],
      *rb_aw[FDEPTH], *rb_ab[FDEPTH];
  float *fin_w, *fin_b, *fin_aw, *fin_ab;
  /* Mimi (mimi.rs:39-53) */
  float *quant_w, *up_w, *down_w, *speaker_proj;
  Layer mdec[MNL], menc[MNL];
  Conv dconv0, dres_a[3], dres_b[3], dfinal;
  ConvTr dtr[3];
  Conv econv0, eres_a[3], eres_b[3], edown[3], efinal;
};

/* ---------------- weight quantization (crates/pocket-tts/src/quantize.rs) ----------------
 * QuantizeConfig::default() (quantize.rs:27-40): skip names containing embed/lut/out_proj/
 * eos_head, keep tensors under min_size = 1024 elements, 256 levels. should_skip_layer is a
 * substring test (quantize.rs:120-123); quantize_weights applies it per tensor (:126-150). */
int orc_quant_applies(const char* name, int64_t numel, int mode) {
  static const char* skip[] = {"embed", "lut", "out_proj", "eos_head"};
  if (mode == 0 || numel < 1024) return 0;
  for (int i = 0; i < 4; ++i)
    if (contains(name, skip[i])) return 0;
  return mode == 2 || strncmp(name, "flow_lm.", 8) == 0;
}
/* QuantizedTensor::quantize (quantize.rs:66-90), f32 throughout as Candle computes it:
 * scale = max|x| / (levels/2 - 1) (1 if all zero); data = clamp(round(x / scale)) * scale,
 * round half away from zero (f32::round). Returns the scale. */
float orc_quantize(const float* x, int64_t n, int num_levels, float* out) {
  float amax = 0.f;
  for (int64_t i = 0; i < n; ++i) amax = fmaxf(amax, fabsf(x[i]));
  const float half = (float)(num_levels / 2);
  const float scale = amax > 0.f ? amax / (half - 1.0f) : 1.0f;
  const float lim = half - 1.0f;
  for (int64_t i = 0; i < n; ++i) {
    float q = roundf(x[i] / scale);
    q = fminf(fmaxf(q, -lim), lim);
    out[i] = q * scale;
  }
  return scale;
}

static float* orc_getw(const orc_model* m, const char* name, int64_t s0, int64_t s1, int64_t s2) {
  int64_t shape[3] = {s0, s1, s2};
  int nd = s2 ? 3 : (s1 ? 2 : 1);
  int64_t n = s0 * (s1 ? s1 : 1) * (s2 ? s2 : 1);
  float* p = (float*)malloc(sizeof(float) * (size_t)n);
  synth_fill(m->seed, name, shape, nd, p, n);
  if (orc_quant_applies(name, n, m->quant)) orc_quantize(p, n, 256, p);
  return p;
}
/* torch Conv1d weight [cout][cin][k] -> [cout][k][cin] */
static Conv mkconv(const orc_model* m, const char* pfx, int cin, int cout, int k, int stride, int bias) {
  char nm[256];
  Conv c = {0};
  c.cin = cin; c.cout = cout; c.k = k; c.stride = stride;
  snprintf(nm, sizeof nm, "%s.weight", pfx);
  float* w = orc_getw(m, nm, cout, cin, k);
  c.w = (float*)malloc(sizeof(float) * (size_t)cout * cin * k);
  for (int o = 0; o < cout; ++o)
    for (int i = 0; i < cin; ++i)
      for (int j = 0; j < k; ++j) c.w[((size_t)o * k + j) * cin + i] = w[((size_t)o * cin + i) * k + j];
  free(w);
  if (bias) { snprintf(nm, sizeof nm, "%s.bias", pfx); c.b = orc_getw(m, nm, cout, 0, 0); }
  return c;
}
static ConvTr mkconvtr(const orc_model* m, const char* pfx, int cin, int cout, int r) {
  char nm[256];
  ConvTr c = {0};
  c.cin = cin; c.cout = cout; c.r = r;
  snprintf(nm, sizeof nm, "%s.weight", pfx);
  c.w = orc_getw(m, nm, cin, cout, 2 * r);
  snprintf(nm, sizeof nm, "%s.bias", pfx);
  c.b = orc_getw(m, nm, cout, 0, 0);
#ifdef ORC_FAST
  c.wp = (float*)malloc(sizeof(float) * (size_t)cin * cout * 2 * r);
  for (int i = 0; i < cin; ++i)
    for (int o = 0; o < cout; ++o)
      for (int j = 0; j < 2 * r; ++j) c.wp[((size_t)o * 2 * r + j) * cin + i] = c.w[((size_t)i * cout + o) * 2 * r + j];
#endif
  return c;
}
static void mklayer(const orc_model* m, Layer* L, const char* pfx, int d, int ff, int ls) {
  char nm[256];
#define W_(field, suffix, a, b)                     \
  snprintf(nm, sizeof nm, "%s.%s", pfx, suffix);    \
  L->field = orc_getw(m, nm, a, b, 0);
  W_(in_proj, "self_attn.in_proj.weight", 3 * d, d);
  W_(out_proj, "self_attn.out_proj.weight", d, d);
  W_(n1w, "norm1.weight", d, 0);
  W_(n1b, "norm1.bias", d, 0);
  W_(n2w, "norm2.weight", d, 0);
  W_(n2b, "norm2.bias", d, 0);
  W_(l1, "linear1.weight", ff, d);
  W_(l2, "linear2.weight", d, ff);
  if (ls) {
    W_(ls1, "layer_scale_1.scale", d, 0);
    W_(ls2, "layer_scale_2.scale", d, 0);
  } else {
    L->ls1 = L->ls2 = NULL;
  }
#undef W_
}

orc_model* orc_model_create(uint64_t seed) { return orc_model_create_ex(seed, 0); }

orc_model* orc_model_create_ex(uint64_t seed, int quant) {
  orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
  char nm[256];
  m->seed = seed;
  m->quant = quant;
  m->embed = orc_getw(m, "flow_lm.conditioner.embed.weight", VOCAB, D, 0);
  m->bos = orc_getw(m, "flow_lm.bos_emb", LDIM, 0, 0);
  m->emb_mean = orc_getw(m, "flow_lm.emb_mean", LDIM, 0, 0);
  m->emb_std = orc_getw(m, "flow_lm.emb_std", LDIM, 0, 0);
  m->input_linear = orc_getw(m, "flow_lm.input_linear.weight", D, LDIM, 0);
  m->out_norm_w = orc_getw(m, "flow_lm.out_norm.weight", D, 0, 0);
  m->out_norm_b = orc_getw(m, "flow_lm.out_norm.bias", D, 0, 0);
  m->eos_w = orc_getw(m, "flow_lm.out_eos.weight", 1, D, 0);
  m->eos_b = orc_getw(m, "flow_lm.out_eos.bias", 1, 0, 0);
  for (int l = 0; l < NL; ++l) {
    snprintf(nm, sizeof nm, "flow_lm.transformer.layers.%d", l);
    mklayer(m, &m->fl[l], nm, D, FF, 0);
  }
  for (int i = 0; i < 2; ++i) {
    snprintf(nm, sizeof nm, "flow_lm.flow_net.time_embed.%d.mlp.0.weight", i);
    m->te_l1w[i] = orc_getw(m, nm, FD, FREQ, 0);
    snprintf(nm, sizeof nm, "flow_lm.flow_net.time_embed.%d.mlp.0.bias", i);
    m->te_l1b[i] = orc_getw(m, nm, FD, 0, 0);
    snprintf(nm, sizeof nm, "flow_lm.flow_net.time_embed.%d.mlp.2.weight", i);
    m->te_l2w[i] = orc_getw(m, nm, FD, FD, 0);
    snprintf(nm, sizeof nm, "flow_lm.flow_net.time_embed.%d.mlp.2.bias", i);
    m->te_l2b[i] = orc_getw(m, nm, FD, 0, 0);
    snprintf(nm, sizeof nm, "flow_lm.flow_net.time_embed.%d.mlp.3.alpha", i);
    m->te_alpha[i] = orc_getw(m, nm, FD, 0, 0);
  }
  m->cond_w = orc_getw(m, "flow_lm.flow_net.cond_embed.weight", FD, D, 0);
  m->cond_b = orc_getw(m, "flow_lm.flow_net.cond_embed.bias", FD, 0, 0);
  m->inproj_w = orc_getw(m, "flow_lm.flow_net.input_proj.weight", FD, LDIM, 0);
  m->inproj_b = orc_getw(m, "flow_lm.flow_net.input_proj.bias", FD, 0, 0);
  for (int i = 0; i < FDEPTH; ++i) {
#define RB(field, suffix, a, b)                                                   \
  snprintf(nm, sizeof nm, "flow_lm.flow_net.res_blocks.%d.%s", i, suffix);     \
  m->field[i] = orc_getw(m, nm, a, b, 0);
    RB(rb_lnw, "in_ln.weight", FD, 0);
    RB(rb_lnb, "in_ln.bias", FD, 0);
    RB(rb_w0, "mlp.0.weight", FD, FD);
    RB(rb_b0, "mlp.0.bias", FD, 0);
    RB(rb_w2, "mlp.2.weight", FD, FD);
    RB(rb_b2, "mlp.2.bias", FD, 0);
    RB(rb_aw, "adaLN_modulation.1.weight", 3 * FD, FD);
    RB(rb_ab, "adaLN_modulation.1.bias", 3 * FD, 0);
#undef RB
  }
  m->fin_w = orc_getw(m, "flow_lm.flow_net.final_layer.linear.weight", LDIM, FD, 0);
  m->fin_b = orc_getw(m, "flow_lm.flow_net.final_layer.linear.bias", LDIM, 0, 0);
  m->fin_aw = orc_getw(m, "flow_lm.flow_net.final_layer.adaLN_modulation.1.weight", 2 * FD, FD, 0);
  m->fin_ab = orc_getw(m, "flow_lm.flow_net.final_layer.adaLN_modulation.1.bias", 2 * FD, 0, 0);
  m->speaker_proj = orc_getw(m, "flow_lm.speaker_proj_weight", D, MD, 0);

  m->quant_w = orc_getw(m, "mimi.quantizer.output_proj.weight", MD, LDIM, 1);
  m->up_w = orc_getw(m, "mimi.upsample.convtr.convtr.weight", MD, 1, 2 * UP);
  for (int l = 0; l < MNL; ++l) {
    snprintf(nm, sizeof nm, "mimi.decoder_transformer.transformer.layers.%d", l);
    mklayer(m, &m->mdec[l], nm, MD, MFF, 1);
    snprintf(nm, sizeof nm, "mimi.encoder_transformer.transformer.layers.%d", l);
    mklayer(m, &m->menc[l], nm, MD, MFF, 1);
  }
  /* SEANetDecoder (seanet.rs:307-402; seanet.py:115-180) */
  m->dconv0 = mkconv(m, "mimi.decoder.model.0.conv", 512, 512, 7, 1, 1);
  static const int ratios[3] = {6, 5, 4};
  int ch = 512;
  for (int i = 0; i < 3; ++i) {
    int li = 2 + 3 * i;
    snprintf(nm, sizeof nm, "mimi.decoder.model.%d.convtr", li);
    m->dtr[i] = mkconvtr(m, nm, ch, ch / 2, ratios[i]);
    ch /= 2;
    snprintf(nm, sizeof nm, "mimi.decoder.model.%d.block.1.conv", li + 1);
    m->dres_a[i] = mkconv(m, nm, ch, ch / 2, 3, 1, 1);
    snprintf(nm, sizeof nm, "mimi.decoder.model.%d.block.3.conv", li + 1);
    m->dres_b[i] = mkconv(m, nm, ch / 2, ch, 1, 1, 1);
  }
  m->dfinal = mkconv(m, "mimi.decoder.model.11.conv", 64, 1, 3, 1, 1);
  /* SEANetEncoder (seanet.rs:148-247; seanet.py:55-112), ratios reversed [4,5,6] */
  m->econv0 = mkconv(m, "mimi.encoder.model.0.conv", 1, 64, 7, 1, 1);
  static const int eratios[3] = {4, 5, 6};
  ch = 64;
  for (int i = 0; i < 3; ++i) {
    int li = 1 + 3 * i;
    snprintf(nm, sizeof nm, "mimi.encoder.model.%d.block.1.conv", li);
    m->eres_a[i] = mkconv(m, nm, ch, ch / 2, 3, 1, 1);
    snprintf(nm, sizeof nm, "mimi.encoder.model.%d.block.3.conv", li);
    m->eres_b[i] = mkconv(m, nm, ch / 2, ch, 1, 1, 1);
    snprintf(nm, sizeof nm, "mimi.encoder.model.%d.conv", li + 2);
    m->edown[i] = mkconv(m, nm, ch, ch * 2, 2 * eratios[i], eratios[i], 1);
    ch *= 2;
  }
  m->efinal = mkconv(m, "mimi.encoder.model.11.conv", 512, 512, 3, 1, 1);
  /* ConvDownsample1d: k=32 s=16 no bias (conv.rs:279-312) */
  m->down_w = NULL;
  {
    Conv dc = mkconv(m, "mimi.downsample.conv.conv", 512, 512, 32, 16, 0);
    m->down_w = dc.w;
  }
  return m;
}

static void free_layer(Layer* L) {
  free(L->in_proj); free(L->out_proj); free(L->n1w); free(L->n1b); free(L->n2w); free(L->n2b);
  free(L->l1); free(L->l2); free(L->ls1); free(L->ls2);
}
static void free_conv(Conv* c) { free(c->w); free(c->b); }
void orc_model_destroy(orc_model* m) {
  if (!m) return;
  free(m->embed); free(m->bos); free(m->emb_mean); free(m->emb_std); free(m->input_linear);
  free(m->out_norm_w); free(m->out_norm_b); free(m->eos_w); free(m->eos_b);
  for (int l = 0; l < NL; ++l) free_layer(&m->fl[l]);
  for (int i = 0; i < 2; ++i) {
    free(m->te_l1w[i]); free(m->te_l1b[i]); free(m->te_l2w[i]); free(m->te_l2b[i]); free(m->te_alpha[i]);
  }
  free(m->cond_w); free(m->cond_b); free(m->inproj_w); free(m->inproj_b);
  for (int i = 0; i < FDEPTH; ++i) {
    free(m->rb_lnw[i]); free(m->rb_lnb[i]); free(m->rb_w0[i]); free(m->rb_b0[i]); free(m->rb_w2[i]);
    free(m->rb_b2[i]); free(m->rb_aw[i]); free(m->rb_ab[i]);
  }
  free(m->fin_w); free(m->fin_b); free(m->fin_aw); free(m->fin_ab); free(m->speaker_proj);
  free(m->quant_w); free(m->up_w); free(m->down_w);
  for (int l = 0; l < MNL; ++l) { free_layer(&m->mdec[l]); free_layer(&m->menc[l]); }
  free_conv(&m->dconv0); free_conv(&m->dfinal); free_conv(&m->econv0); free_conv(&m->efinal);
  for (int i = 0; i < 3; ++i) {
    free_conv(&m->dres_a[i]); free_conv(&m->dres_b[i]); free(m->dtr[i].w); free(m->dtr[i].b); free(m->dtr[i].wp);
    free_conv(&m->eres_a[i]); free_conv(&m->eres_b[i]); free_conv(&m->edown[i]);
  }
  free(m);
}

/* ---------------- primitive ops ---------------- */
#ifdef ORC_FAST
/* CPU-BASELINE BUILD ONLY (libptts_cpu_fast.so, oracle/Makefile): never the checker. A cache-
 * blocked AVX2/FMA GEMM, y[i][n] = x[i].W[n] over K-contiguous rows (x row stride ldx), the form
 * candle's gemm-crate matmuls and im2col convs take on a CPU: a 3-row x 4-column register tile of
 * 8-wide FMA accumulators (12 ymm), columns in blocks of 64 so a block of W stays in L2 while the
 * rows stream. M = 1 (the B = 1 GEMV) uses an 8-column tile sharing each x load. K % 8 tails
 * are handled scalar. Differs from the oracle's rounding (FMA, 8-way partial sums). */
#include <immintrin.h>
static inline float hsum8(__m256 v) {
  __m128 a = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
  a = _mm_add_ps(a, _mm_movehl_ps(a, a));
  a = _mm_add_ss(a, _mm_movehdup_ps(a));
  return _mm_cvtss_f32(a);
}
static void gemm_nt(float* y, int ldy, const float* x, long ldx, const float* W, int M, int N, int K,
                    const float* b) {
  const int K8 = K & ~7;
  if (M == 1) {
#pragma omp parallel for schedule(static) if ((long)N * K > 200000)
    for (int n0 = 0; n0 < N; n0 += 8) {
      const int nn = N - n0 < 8 ? N - n0 : 8;
      __m256 acc[8];
      for (int c = 0; c < 8; ++c) acc[c] = _mm256_setzero_ps();
      for (int k = 0; k < K8; k += 8) {
        const __m256 xv = _mm256_loadu_ps(x + k);
        for (int c = 0; c < nn; ++c) acc[c] = _mm256_fmadd_ps(xv, _mm256_loadu_ps(W + (size_t)(n0 + c) * K + k), acc[c]);
      }
      for (int c = 0; c < nn; ++c) {
        float v = hsum8(acc[c]);
        for (int k = K8; k < K; ++k) v += x[k] * W[(size_t)(n0 + c) * K + k];
        y[n0 + c] = b ? v + b[n0 + c] : v;
      }
    }
    return;
  }
  const int nblk = (N + 63) / 64, mblk = (M + 2) / 3;
#pragma omp parallel for collapse(2) schedule(static) if ((long)M * N * K > 200000)
  for (int nb = 0; nb < nblk; ++nb)
    for (int mb = 0; mb < mblk; ++mb) {
      const int i0 = 3 * mb, ni = M - i0 < 3 ? M - i0 : 3;
      const int ne = (nb + 1) * 64 < N ? (nb + 1) * 64 : N;
      const float* xr[3];
      for (int r = 0; r < 3; ++r) xr[r] = x + (size_t)(i0 + (r < ni ? r : 0)) * ldx;
      for (int n0 = nb * 64; n0 < ne; n0 += 4) {
        const int nn = ne - n0 < 4 ? ne - n0 : 4;
        const float* wr[4];
        for (int c = 0; c < 4; ++c) wr[c] = W + (size_t)(n0 + (c < nn ? c : 0)) * K;
        __m256 acc[3][4];
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 4; ++c) acc[r][c] = _mm256_setzero_ps();
        for (int k = 0; k < K8; k += 8) {
          const __m256 x0 = _mm256_loadu_ps(xr[0] + k), x1 = _mm256_loadu_ps(xr[1] + k), x2 = _mm256_loadu_ps(xr[2] + k);
          for (int c = 0; c < 4; ++c) {
            const __m256 wv = _mm256_loadu_ps(wr[c] + k);
            acc[0][c] = _mm256_fmadd_ps(x0, wv, acc[0][c]);
            acc[1][c] = _mm256_fmadd_ps(x1, wv, acc[1][c]);
            acc[2][c] = _mm256_fmadd_ps(x2, wv, acc[2][c]);
          }
        }
        for (int r = 0; r < ni; ++r)
          for (int c = 0; c < nn; ++c) {
            float v = hsum8(acc[r][c]);
            for (int k = K8; k < K; ++k) v += xr[r][k] * wr[c][k];
            y[(size_t)(i0 + r) * ldy + n0 + c] = b ? v + b[n0 + c] : v;
          }
      }
    }
}
#endif

/* y[M][N] = x[M][K] . W[N][K]^T (+ b)   (candle Linear: y = x W^T + b) */
static void linear(float* y, const float* x, const float* W, const float* b, int M, int N, int K) {
#ifdef ORC_FAST
  gemm_nt(y, N, x, K, W, M, N, K, b);
  return;
#endif
#pragma omp parallel for collapse(2) schedule(static) if ((long)M * N * K > 200000)
  for (int i = 0; i < M; ++i)
    for (int n = 0; n < N; ++n) {
      const float* xr = x + (size_t)i * K;
      const float* wr = W + (size_t)n * K;
      float acc = 0.f;
#pragma omp simd reduction(+ : acc)
      for (int k = 0; k < K; ++k) acc += xr[k] * wr[k];
      y[(size_t)i * N + n] = b ? acc + b[n] : acc;
    }
}
/* LayerNorm, biased variance (mlp.rs:29-58 -> candle_nn::LayerNorm; mlp.py:31-48) */
static void layernorm(float* y, const float* x, const float* w, const float* b, int M, int N, float eps) {
  for (int i = 0; i < M; ++i) {
    const float* xr = x + (size_t)i * N;
    float mean = 0.f, var = 0.f;
    for (int n = 0; n < N; ++n) mean += xr[n];
    mean /= (float)N;
    for (int n = 0; n < N; ++n) { float d = xr[n] - mean; var += d * d; }
    var /= (float)N;
    float inv = 1.0f / sqrtf(var + eps);
    for (int n = 0; n < N; ++n) {
      float v = (xr[n] - mean) * inv;
      y[(size_t)i * N + n] = w ? v * w[n] + b[n] : v;
    }
  }
}
/* Candle Tensor::gelu = tanh approximation (transformer.rs:85) */
static float gelu_tanh(float x) {
  return 0.5f * x * (1.0f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}
static float silu(float x) { return x / (1.0f + expf(-x)); }
static float elu(float x) { return x >= 0.f ? x : expf(x) - 1.0f; } /* seanet.rs:298-305, alpha 1 */

/* RoPE, interleaved pairs (rope.rs:18-60; rope.py:7-55) on rows [T][nh*64], positions p0+t */
static void rope(float* q, float* k, int T, int nh, int p0) {
  for (int t = 0; t < T; ++t) {
    float ts = (float)(p0 + t);
    for (int h = 0; h < nh; ++h)
      for (int i = 0; i < HD / 2; ++i) {
        float freq = expf((float)i * (-logf(10000.0f) * 2.0f / (float)HD));
        float ang = freq * ts;
        float c = cosf(ang), s = sinf(ang);
        float* qp = q + (size_t)t * nh * HD * 3 + h * HD + 2 * i; /* rows are packed qkv */
        float* kp = k + (size_t)t * nh * HD * 3 + h * HD + 2 * i;
        float qr = qp[0], qi = qp[1], kr = kp[0], ki = kp[1];
        qp[0] = qr * c - qi * s; qp[1] = qr * s + qi * c;
        kp[0] = kr * c - ki * s; kp[1] = kr * s + ki * c;
      }
  }
}

/* ---------------- state ---------------- */
struct orc_state {
  int max_ctx, pos;
  float* kv; /* [NL][2][NH][max_ctx][HD] */
  int mpos;
  float* ring;          /* [MNL][2][MNH][RING][HD] absolute position p stored at p % RING */
  float up_partial[MD * UP];         /* upsample convtr partial [512][16] (conv.rs:202-267) */
  float hist0[6 * 512];              /* decoder.model.0 previous [6][512] (time-major) */
  float tr_partial[3][256 * 6];      /* decoder convtr partials [cout][r] */
  float res_hist[3][2 * 256];        /* resblock conv3 previous [2][C] */
  float fin_hist[2 * 64];            /* decoder.model.11 previous [2][64] */
};

orc_state* orc_state_create(const orc_model* m, int max_ctx) {
  (void)m;
  orc_state* s = (orc_state*)calloc(1, sizeof(orc_state));
  s->max_ctx = max_ctx;
  s->kv = (float*)calloc((size_t)NL * 2 * NH * max_ctx * HD, sizeof(float));
  s->ring = (float*)calloc((size_t)MNL * 2 * MNH * RING * HD, sizeof(float));
  return s;
}
void orc_state_destroy(orc_state* s) {
  if (!s) return;
  free(s->kv); free(s->ring); free(s);
}
int orc_state_pos(const orc_state* s) { return s->pos; }

/* softmax attention of one query against keys K[j], j in [j0, j1] (absolute), key j at kbase + (j % cap)*HD */
static void attend(float* out, const float* q, const float* kb, const float* vb, int j0, int j1, int cap) {
  int n = j1 - j0 + 1;
  float* sc = (float*)malloc(sizeof(float) * (size_t)n);
  float mx = -INFINITY;
  for (int j = j0; j <= j1; ++j) {
    const float* kr = kb + (size_t)(j % cap) * HD;
    float acc = 0.f;
#pragma omp simd reduction(+ : acc)
    for (int d = 0; d < HD; ++d) acc += q[d] * kr[d];
    acc *= 0.125f; /* 1/sqrt(64): attention.rs:191,229 */
    sc[j - j0] = acc;
    if (acc > mx) mx = acc;
  }
  float sum = 0.f;
  for (int i = 0; i < n; ++i) { sc[i] = expf(sc[i] - mx); sum += sc[i]; }
  for (int d = 0; d < HD; ++d) out[d] = 0.f;
  for (int j = j0; j <= j1; ++j) {
    const float* vr = vb + (size_t)(j % cap) * HD;
    float p = sc[j - j0] / sum;
    for (int d = 0; d < HD; ++d) out[d] += p * vr[d];
  }
  free(sc);
}

/* One pre-LN transformer layer over T rows (transformer.rs:66-90; mimi_transformer.py:188-206).
 * kv: per-layer cache base [2][nh][cap][HD]; positions p0..p0+T-1; window (0 = none). */
static void tlayer(const Layer* L, float* x, int T, int d, int nh, int ff, float* kvl, int cap, int p0,
                   int window) {
  float* h = (float*)malloc(sizeof(float) * (size_t)T * d);
  float* qkv = (float*)malloc(sizeof(float) * (size_t)T * 3 * d);
  float* o = (float*)malloc(sizeof(float) * (size_t)T * d);
  float* u = (float*)malloc(sizeof(float) * (size_t)T * ff);
  layernorm(h, x, L->n1w, L->n1b, T, d, 1e-5f);
  linear(qkv, h, L->in_proj, NULL, T, 3 * d, d);
  rope(qkv, qkv + d, T, nh, p0);
  /* KV append (attention.rs:211-264) */
  for (int t = 0; t < T; ++t)
    for (int hh = 0; hh < nh; ++hh) {
      int slot = (p0 + t) % cap;
      memcpy(kvl + ((size_t)(0 * nh + hh) * cap + slot) * HD, qkv + (size_t)t * 3 * d + d + hh * HD,
             sizeof(float) * HD);
      memcpy(kvl + ((size_t)(1 * nh + hh) * cap + slot) * HD, qkv + (size_t)t * 3 * d + 2 * d + hh * HD,
             sizeof(float) * HD);
    }
  /* causal (+ context window) mask: sdpa.rs:128-171 */
#pragma omp parallel for collapse(2) schedule(static) if (T * nh > 8)
  for (int t = 0; t < T; ++t)
    for (int hh = 0; hh < nh; ++hh) {
      int p = p0 + t;
      int j0 = window ? (p - window + 1 > 0 ? p - window + 1 : 0) : 0;
      attend(o + (size_t)t * d + hh * HD, qkv + (size_t)t * 3 * d + hh * HD,
             kvl + (size_t)(0 * nh + hh) * cap * HD, kvl + (size_t)(1 * nh + hh) * cap * HD, j0, p, cap);
    }
  linear(h, o, L->out_proj, NULL, T, d, d);
  for (int i = 0; i < T * d; ++i) x[i] += L->ls1 ? L->ls1[i % d] * h[i] : h[i];
  layernorm(h, x, L->n2w, L->n2b, T, d, 1e-5f);
  linear(u, h, L->l1, NULL, T, ff, d);
  for (int i = 0; i < T * ff; ++i) u[i] = gelu_tanh(u[i]);
  linear(h, u, L->l2, NULL, T, d, ff);
  for (int i = 0; i < T * d; ++i) x[i] += L->ls2 ? L->ls2[i % d] * h[i] : h[i];
  free(h); free(qkv); free(o); free(u);
}

static void flow_transformer(const orc_model* m, orc_state* s, float* x, int T) {
  if (s->pos + T > s->max_ctx) { fprintf(stderr, "oracle: context overflow\n"); abort(); }
  for (int l = 0; l < NL; ++l)
    tlayer(&m->fl[l], x, T, D, NH, FF, s->kv + (size_t)l * 2 * NH * s->max_ctx * HD, s->max_ctx, s->pos, 0);
  s->pos += T;
}

void orc_prefill(const orc_model* m, orc_state* s, const float* x, int T) {
  float* buf = (float*)malloc(sizeof(float) * (size_t)T * D);
  memcpy(buf, x, sizeof(float) * (size_t)T * D);
  flow_transformer(m, s, buf, T);
  free(buf);
}
void orc_embed_tokens(const orc_model* m, const int32_t* ids, int S, float* out) {
  for (int i = 0; i < S; ++i) memcpy(out + (size_t)i * D, m->embed + (size_t)ids[i] * D, sizeof(float) * D);
}
void orc_prefill_tokens(const orc_model* m, orc_state* s, const int32_t* ids, int S) {
  float* buf = (float*)malloc(sizeof(float) * (size_t)S * D);
  orc_embed_tokens(m, ids, S, buf);
  flow_transformer(m, s, buf, S);
  free(buf);
}

/* TimestepEmbedder (mlp.rs:76-133; mlp.py:51-79); RMSNorm uses unbiased variance (mlp.rs:18-26) */
static void timestep_embed(const orc_model* m, int which, float tau, float* out) {
  float emb[FREQ], h[FD];
  for (int k = 0; k < FREQ / 2; ++k) {
    float f = expf(-logf(10000.0f) * (float)k / (float)(FREQ / 2));
    float a = tau * f;
    emb[k] = cosf(a);
    emb[FREQ / 2 + k] = sinf(a);
  }
  linear(h, emb, m->te_l1w[which], m->te_l1b[which], 1, FD, FREQ);
  for (int i = 0; i < FD; ++i) h[i] = silu(h[i]);
  linear(out, h, m->te_l2w[which], m->te_l2b[which], 1, FD, FD);
  float mean = 0.f, var = 0.f;
  for (int i = 0; i < FD; ++i) mean += out[i];
  mean /= FD;
  for (int i = 0; i < FD; ++i) { float dd = out[i] - mean; var += dd * dd; }
  var /= (float)(FD - 1);
  float inv = 1.0f / sqrtf(var + 1e-5f);
  for (int i = 0; i < FD; ++i) out[i] = out[i] * inv * m->te_alpha[which][i];
}
void orc_time_embeddings(const orc_model* m, int n, float* out) {
  for (int i = 0; i < n; ++i) {
    float a[FD], b[FD];
    timestep_embed(m, 0, (float)((double)i / n), a);
    timestep_embed(m, 1, (float)((double)(i + 1) / n), b);
    for (int k = 0; k < FD; ++k) out[(size_t)i * FD + k] = (a[k] + b[k]) / 2.0f;
  }
}

/* SimpleMLPAdaLN.forward_step_cached (mlp.rs:370-383) + ResBlock/FinalLayer */
static void flow_head(const orc_model* m, const float* c_emb, const float* tvec, const float* xin, float* out) {
  float y[FD], mod[3 * FD], x[FD], h[FD], u[FD];
  for (int i = 0; i < FD; ++i) y[i] = silu(tvec[i] + c_emb[i]); /* mlp.rs:329-330 */
  linear(x, xin, m->inproj_w, m->inproj_b, 1, FD, LDIM);
  for (int b = 0; b < FDEPTH; ++b) {
    linear(mod, y, m->rb_aw[b], m->rb_ab[b], 1, 3 * FD, FD);
    layernorm(h, x, m->rb_lnw[b], m->rb_lnb[b], 1, FD, 1e-6f);
    for (int i = 0; i < FD; ++i) h[i] = h[i] * (1.0f + mod[FD + i]) + mod[i]; /* modulate mlp.rs:135 */
    linear(u, h, m->rb_w0[b], m->rb_b0[b], 1, FD, FD);
    for (int i = 0; i < FD; ++i) u[i] = silu(u[i]);
    linear(h, u, m->rb_w2[b], m->rb_b2[b], 1, FD, FD);
    for (int i = 0; i < FD; ++i) x[i] = x[i] + h[i] * mod[2 * FD + i];
  }
  linear(mod, y, m->fin_aw, m->fin_ab, 1, 2 * FD, FD);
  layernorm(h, x, NULL, NULL, 1, FD, 1e-6f);
  for (int i = 0; i < FD; ++i) h[i] = h[i] * (1.0f + mod[FD + i]) + mod[i];
  linear(out, h, m->fin_w, m->fin_b, 1, LDIM, FD);
}

/* streaming conv, channels-last: x [T][cin], hist [P][cin] (P = k - stride) updated in place.
 * StreamingConv1d::forward (conv.rs:90-136) */
static void sconv(const Conv* c, const float* x, int T, float* hist, float* y, int apply_elu) {
  int P = c->k - c->stride;
  int Tp = P + T;
  float* xp = (float*)malloc(sizeof(float) * (size_t)Tp * c->cin);
  if (P) memcpy(xp, hist, sizeof(float) * (size_t)P * c->cin);
  for (int i = 0; i < T * c->cin; ++i) xp[(size_t)P * c->cin + i] = apply_elu ? elu(x[i]) : x[i];
  int To = T / c->stride;
#ifdef ORC_FAST /* output row t's taps are the contiguous k*cin floats at row t*stride of xp */
  gemm_nt(y, c->cout, xp, (long)c->stride * c->cin, c->w, To, c->cout, c->k * c->cin, c->b);
  if (P) memcpy(hist, xp + (size_t)T * c->cin, sizeof(float) * (size_t)P * c->cin);
  free(xp);
  return;
#endif
#pragma omp parallel for collapse(2) schedule(static) if ((long)To * c->cout * c->k * c->cin > 200000)
  for (int t = 0; t < To; ++t)
    for (int o = 0; o < c->cout; ++o) {
      float acc = 0.f;
      for (int j = 0; j < c->k; ++j) {
        const float* xr = xp + (size_t)(t * c->stride + j) * c->cin;
        const float* wr = c->w + ((size_t)o * c->k + j) * c->cin;
#pragma omp simd reduction(+ : acc)
        for (int i = 0; i < c->cin; ++i) acc += xr[i] * wr[i];
      }
      y[(size_t)t * c->cout + o] = c->b ? acc + c->b[o] : acc;
    }
  if (P) memcpy(hist, xp + (size_t)T * c->cin, sizeof(float) * (size_t)P * c->cin);
  free(xp);
}
/* streaming transposed conv with overlap-add partial (conv.rs:219-267), input ELU'd.
 * x [T][cin] -> y [T*r][cout]; partial [cout][r] */
static void sconvtr(const ConvTr* c, const float* x, int T, float* partial, float* y) {
  int r = c->r, K = 2 * r, To = T * r + r;
  float* full = (float*)calloc((size_t)To * c->cout, sizeof(float));
  float* e = (float*)malloc(sizeof(float) * (size_t)T * c->cin);
  for (int i = 0; i < T * c->cin; ++i) e[i] = elu(x[i]);
#ifdef ORC_FAST /* one GEMM [T][cin] x [cout*2r][cin]^T, then the overlap-add of the 2r taps */
  float* g = (float*)malloc(sizeof(float) * (size_t)T * c->cout * K);
  gemm_nt(g, c->cout * K, e, c->cin, c->wp, T, c->cout * K, c->cin, NULL);
  for (int t = 0; t < T; ++t)
    for (int o = 0; o < c->cout; ++o)
      for (int j = 0; j < K; ++j) full[(size_t)(t * r + j) * c->cout + o] += g[((size_t)t * c->cout + o) * K + j];
  free(g);
  if (0)
#else
#pragma omp parallel for schedule(static) if ((long)T * c->cout * c->cin * K > 200000)
#endif
  for (int o = 0; o < c->cout; ++o)
    for (int t = 0; t < T; ++t)
      for (int j = 0; j < K; ++j) {
        float acc = 0.f;
        for (int i = 0; i < c->cin; ++i) acc += e[(size_t)t * c->cin + i] * c->w[((size_t)i * c->cout + o) * K + j];
        full[(size_t)(t * r + j) * c->cout + o] += acc;
      }
  for (int t = 0; t < To; ++t)
    for (int o = 0; o < c->cout; ++o) full[(size_t)t * c->cout + o] += c->b[o];
  for (int j = 0; j < r; ++j)
    for (int o = 0; o < c->cout; ++o) full[(size_t)j * c->cout + o] += partial[o * r + j];
  for (int j = 0; j < r; ++j)
    for (int o = 0; o < c->cout; ++o) partial[o * r + j] = full[(size_t)(T * r + j) * c->cout + o] - c->b[o];
  memcpy(y, full, sizeof(float) * (size_t)T * r * c->cout);
  free(full); free(e);
}

void orc_mimi_decode_ex(const orc_model* m, orc_state* s, const float* latent, float* pcm, float* quantized,
                        float* after_up, float* after_tr) {
  float z[LDIM], q[MD];
  /* denorm + DummyQuantizer 1x1 conv (tts_model.rs:1033-1038; mimi.rs:8-37) */
  for (int k = 0; k < LDIM; ++k) z[k] = latent[k] * m->emb_std[k] + m->emb_mean[k];
  linear(q, z, m->quant_w, NULL, 1, MD, LDIM);
  if (quantized) memcpy(quantized, q, sizeof q);
  /* ConvTrUpsample1d depthwise k32 s16, partial overlap-add (conv.rs:315-346) */
  float* x = (float*)malloc(sizeof(float) * UP * MD);
  for (int c = 0; c < MD; ++c) {
    for (int r = 0; r < UP; ++r) x[r * MD + c] = q[c] * m->up_w[c * 2 * UP + r] + s->up_partial[c * UP + r];
    for (int r = 0; r < UP; ++r) s->up_partial[c * UP + r] = q[c] * m->up_w[c * 2 * UP + UP + r];
  }
  if (after_up) memcpy(after_up, x, sizeof(float) * UP * MD);
  /* decoder transformer, ring context 250 (transformer.rs:227-251, attention.rs:167-264) */
  for (int l = 0; l < MNL; ++l)
    tlayer(&m->mdec[l], x, UP, MD, MNH, MFF, s->ring + (size_t)l * 2 * MNH * RING * HD, RING, s->mpos, MCTX);
  s->mpos += UP;
  if (after_tr) memcpy(after_tr, x, sizeof(float) * UP * MD);
  /* SEANetDecoder (seanet.rs:396-402) */
  float* a = (float*)malloc(sizeof(float) * FRAME * 64);
  float* b = (float*)malloc(sizeof(float) * FRAME * 64);
  float* v = (float*)malloc(sizeof(float) * FRAME * 64);
  sconv(&m->dconv0, x, UP, s->hist0, a, 0);
  int T = UP, ch = 512;
  for (int i = 0; i < 3; ++i) {
    sconvtr(&m->dtr[i], a, T, s->tr_partial[i], b);
    T *= m->dtr[i].r;
    ch /= 2;
    sconv(&m->dres_a[i], b, T, s->res_hist[i], v, 1);
    sconv(&m->dres_b[i], v, T, NULL, a, 1);
    for (int k = 0; k < T * ch; ++k) a[k] += b[k]; /* SEANetResnetBlock skip (seanet.py:35) */
  }
  sconv(&m->dfinal, a, T, s->fin_hist, pcm, 1);
  free(x); free(a); free(b); free(v);
}
void orc_mimi_decode(const orc_model* m, orc_state* s, const float* latent, float* pcm) {
  orc_mimi_decode_ex(m, s, latent, pcm, NULL, NULL, NULL);
}

void orc_step(const orc_model* m, orc_state* s, const float* latent_in, const float* noise, int lsd_steps,
              float* tout_o, float* eos_o, float* latent_o, float* pcm_o, float* quant_o, float* up_o,
              float* tr_o) {
  float x[D], tout[D], cemb[FD], cur[LDIM], flow[LDIM], eos;
  /* FlowLMModel::forward (flow_lm.rs:98-164) */
  linear(x, latent_in ? latent_in : m->bos, m->input_linear, NULL, 1, D, LDIM);
  flow_transformer(m, s, x, 1);
  layernorm(tout, x, m->out_norm_w, m->out_norm_b, 1, D, 1e-5f);
  linear(&eos, tout, m->eos_w, m->eos_b, 1, 1, D);
  linear(cemb, tout, m->cond_w, m->cond_b, 1, FD, D);
  float* te = (float*)malloc(sizeof(float) * (size_t)lsd_steps * FD);
  orc_time_embeddings(m, lsd_steps, te);
  for (int k = 0; k < LDIM; ++k) cur[k] = noise ? noise[k] : 0.f;
  /* lsd_decode (flow_lm.rs:7-22) */
  for (int i = 0; i < lsd_steps; ++i) {
    flow_head(m, cemb, te + (size_t)i * FD, cur, flow);
    for (int k = 0; k < LDIM; ++k) cur[k] += flow[k] * (1.0f / (float)lsd_steps);
  }
  free(te);
  if (tout_o) memcpy(tout_o, tout, sizeof tout);
  if (eos_o) *eos_o = eos;
  if (latent_o) memcpy(latent_o, cur, sizeof cur);
  float pcm[FRAME];
  orc_mimi_decode_ex(m, s, cur, pcm, quant_o, up_o, tr_o);
  if (pcm_o) memcpy(pcm_o, pcm, sizeof pcm);
}

/* ---------------- encoder (voice cloning) ---------------- */
void orc_encode(const orc_model* m, const float* pcm, int n, float* cond, float* after_enc, float* after_tr,
                float* latent_o) {
  orc_encode_ex(m, pcm, n, -1, cond, after_enc, after_tr, latent_o);
}

void orc_encode_ex(const orc_model* m, const float* pcm, int n, int chunk_frames, float* cond, float* after_enc,
                   float* after_tr, float* latent_o) {
  int T = n;
  float* a = (float*)malloc(sizeof(float) * (size_t)T * 64);
  float* b = (float*)malloc(sizeof(float) * (size_t)T * 64);
  float* v = (float*)malloc(sizeof(float) * (size_t)T * 64);
  float hist[32 * 512];
  memset(hist, 0, sizeof hist);
  sconv(&m->econv0, pcm, T, hist, a, 0); /* fresh zero state: model_state=None (mimi.py:106) */
  int ch = 64;
  for (int i = 0; i < 3; ++i) {
    memset(hist, 0, sizeof hist);
    sconv(&m->eres_a[i], a, T, hist, v, 1);
    sconv(&m->eres_b[i], v, T, NULL, b, 1);
    for (int k = 0; k < T * ch; ++k) b[k] += a[k];
    memset(hist, 0, sizeof hist);
    sconv(&m->edown[i], b, T, hist, a, 1);
    T /= m->edown[i].stride;
    ch *= 2;
  }
  memset(hist, 0, sizeof hist);
  sconv(&m->efinal, a, T, hist, b, 1);
  if (after_enc) memcpy(after_enc, b, sizeof(float) * (size_t)T * 512);
  /* encoder transformer: whole sequence, positions 0..T-1, context 250 (mimi_transformer.py:30-38,107-118) */
  float* ring = (float*)calloc((size_t)2 * MNH * (size_t)T * HD, sizeof(float));
  for (int l = 0; l < MNL; ++l) tlayer(&m->menc[l], b, T, MD, MNH, MFF, ring, T, 0, MCTX);
  free(ring);
  if (after_tr) memcpy(after_tr, b, sizeof(float) * (size_t)T * 512);
  /* ConvDownsample1d, replicate padding on the first frame (conv.rs:116-123; conv.py:103-108).
   * The Rust driver encodes chunk by chunk with step=0 every time (tts_model.rs:536-541), so the
   * replicate padding is re-applied at each chunk's first frame; the streaming convs and the
   * transformer before it carry their state across chunks, which equals the one pass above. */
  Conv dc = {m->down_w, NULL, 512, 512, 32, 16};
  int F = T / 16;
  const int cf = chunk_frames <= 0 ? F : chunk_frames;
  for (int c0 = 0; c0 < F; c0 += cf) {
    const int nf = F - c0 < cf ? F - c0 : cf;
    const float* xc = b + (size_t)c0 * 16 * 512;
    for (int t = 0; t < 16; ++t) memcpy(hist + t * 512, xc, sizeof(float) * 512);
    sconv(&dc, xc, nf * 16, hist, a + (size_t)c0 * 512, 0);
  }
  if (latent_o) memcpy(latent_o, a, sizeof(float) * (size_t)F * 512);
  /* speaker projection (tts_model.rs:543-553) */
  linear(cond, a, m->speaker_proj, NULL, F, D, MD);
  free(a); free(b); free(v);
}

/* ---------------- resampler (voice-cloning front end) ----------------
 * scipy.signal.resample_poly(x, up, down) with its default Kaiser(5.0) FIR, as the Python reference
 * calls it in convert_audio (python-reference/pocket_tts/data/audio_utils.py:8-28); the Rust
 * reference's audio.rs:197-255 states it matches that function (it calls rubato 0.14.1
 * FastFixedIn/Septic, whose source is not in the reference: that drift stays unpinned, and the
 * reference's own test allows 0.3 for it, parity_tests.rs:379-433).
 * Filter: firwin(2*half+1, 1/max(up,down)), half = 10*max(up,down): h[i] = fc*sinc(fc*(i-half))
 * * kaiser(5.0)[i], normalised to unit DC gain, cast to f32 and scaled by `up` in f32 (scipy casts
 * the taps to the f32 input dtype). Output m = sum_j x[j] * h[m*down + half - j*up]; the f32
 * products are accumulated in double. */
static double bessel_i0(double x) {
  double s = 1.0, t = 1.0, q = 0.25 * x * x;
  for (int k = 1; k < 500; ++k) {
    t *= q / ((double)k * k);
    s += t;
    if (t < 1e-17 * s) break;
  }
  return s;
}
static int gcd_int(int a, int b) {
  while (b) { int t = a % b; a = b; b = t; }
  return a;
}
int orc_resample_len(int n, int sr_from, int sr_to) {
  if (n <= 0 || sr_from <= 0 || sr_to <= 0) return 0;
  const int g = gcd_int(sr_from, sr_to);
  const long up = sr_to / g, down = sr_from / g, t = (long)n * up;
  return (int)(t / down + (t % down != 0));
}
int orc_resample(const float* x, int n, int sr_from, int sr_to, float* y) {
  const int n_out = orc_resample_len(n, sr_from, sr_to);
  if (n_out <= 0) return 0;
  const int g = gcd_int(sr_from, sr_to), up = sr_to / g, down = sr_from / g;
  if (up == 1 && down == 1) { memcpy(y, x, sizeof(float) * (size_t)n); return n; }
  const int mr = up > down ? up : down, half = 10 * mr, L = 2 * half + 1;
  double* hd = (double*)malloc(sizeof(double) * (size_t)L);
  float* h = (float*)malloc(sizeof(float) * (size_t)L);
  const double fc = 1.0 / mr, alpha = 0.5 * (L - 1), i0b = bessel_i0(5.0);
  double s = 0.0;
  for (int i = 0; i < L; ++i) {
    const double mm = i - alpha, v = fc * mm, r = (i - alpha) / alpha;
    const double sinc = v == 0.0 ? 1.0 : sin(M_PI * v) / (M_PI * v);
    hd[i] = fc * sinc * (bessel_i0(5.0 * sqrt(fmax(0.0, 1.0 - r * r))) / i0b);
    s += hd[i];
  }
  for (int i = 0; i < L; ++i) h[i] = (float)(hd[i] / s) * (float)up;
  for (int m = 0; m < n_out; ++m) {
    const long a = (long)m * down + half;
    long jhi = a / up;
    if (jhi > n - 1) jhi = n - 1;
    const long lo = a - (L - 1);
    const long jlo = lo <= 0 ? 0 : (lo + up - 1) / up;
    double acc = 0.0;
    for (long j = jlo; j <= jhi; ++j) acc += (double)x[j] * (double)h[a - j * up];
    y[m] = (float)acc;
  }
  free(hd);
  free(h);
  return n_out;
}

/* rubato 0.14.1 FastFixedIn with PolynomialDegree::Septic, as the Rust driver calls it
 * (audio.rs:216-225: FastFixedIn::new(to/from, 1.0, Septic, n, channels), then one process()):
 * rubato keeps an 8-point polynomial window (POLYNOMIAL_LEN = 8) behind a zero history of 2 x 8
 * samples; its read position starts at last_index = -(8 / 2), and each output first advances it
 * by t_ratio = 1 / ratio (the ratio is fixed, so the ramp dt_ratio is 0) in f64, then evaluates
 * the septic through the samples at floor(idx) - 3 .. floor(idx) + 4 at frac = idx - floor(idx)
 * (coerced to f32); outputs continue while the position before the step is below
 * chunk - (8 + 1). The septic is the Lagrange polynomial of nodes -3..4 (rubato writes it in power
 * form: the same polynomial, f32 rounding apart), evaluated here as prefix x suffix products of
 * (frac - node) times 1 / prod_{m != j} (j - m), summed in tap order; the HIP kernel
 * (kernels.hip k_resample_septic) performs the same f32 operations in the same order. */
static long septic_walk(long n, int sr_from, int sr_to, int* start, float* frac) {
  const double ratio = (double)sr_to / (double)sr_from, t = 1.0 / ratio, end = (double)(n - 9);
  double idx = -4.0;
  long cnt = 0;
  while (idx < end) {
    idx += t;
    const double fl = floor(idx);
    if (start) start[cnt] = (int)fl;
    if (frac) frac[cnt] = (float)(idx - fl);
    ++cnt;
  }
  return cnt;
}
int orc_resample_septic_len(int n, int sr_from, int sr_to) {
  if (n <= 0 || sr_from <= 0 || sr_to <= 0) return 0;
  if (sr_from == sr_to) return n;
  return (int)septic_walk(n, sr_from, sr_to, NULL, NULL);
}
int orc_resample_septic(const float* x, int n, int sr_from, int sr_to, float* y) {
  const int n_out = orc_resample_septic_len(n, sr_from, sr_to);
  if (n_out <= 0) return 0;
  if (sr_from == sr_to) { memcpy(y, x, sizeof(float) * (size_t)n); return n; }
  int* st = (int*)malloc(sizeof(int) * (size_t)n_out);
  float* fr = (float*)malloc(sizeof(float) * (size_t)n_out);
  septic_walk(n, sr_from, sr_to, st, fr);
  static const float inv_den[8] = {-1.f / 5040.f, 1.f / 720.f, -1.f / 240.f, 1.f / 144.f,
                                   -1.f / 144.f,  1.f / 240.f, -1.f / 720.f, 1.f / 5040.f};
  for (int o = 0; o < n_out; ++o) {
    const float f = fr[o];
    float d[8], pre[8], suf[8];
    for (int m = 0; m < 8; ++m) d[m] = f - (float)(m - 3);
    pre[0] = 1.f;
    for (int m = 1; m < 8; ++m) pre[m] = pre[m - 1] * d[m - 1];
    suf[7] = 1.f;
    for (int m = 6; m >= 0; --m) suf[m] = suf[m + 1] * d[m + 1];
    float acc = 0.f;
    for (int j = 0; j < 8; ++j) {
      const int i = st[o] - 3 + j;
      const float v = (i >= 0 && i < n) ? x[i] : 0.f;
      acc = acc + v * ((pre[j] * suf[j]) * inv_den[j]);
    }
    y[o] = acc;
  }
  free(st);
  free(fr);
  return n_out;
}

/* ---------------- CPU baseline driver ---------------- */
double orc_bench(const orc_model* m, int n_utt, int F, int S, int n_frames, int threads) {
  orc_state** st = (orc_state**)malloc(sizeof(orc_state*) * (size_t)n_utt);
  float* prompt = (float*)malloc(sizeof(float) * (size_t)F * D);
  for (int i = 0; i < F * D; ++i) prompt[i] = 0.11f * (float)sin(0.37 * i);
  int32_t* ids = (int32_t*)malloc(sizeof(int32_t) * (size_t)S);
  for (int i = 0; i < S; ++i) ids[i] = (i * 97 + 13) % 4000;
  omp_set_num_threads(threads);
  for (int u = 0; u < n_utt; ++u) {
    st[u] = orc_state_create(m, F + S + n_frames + 8);
    if (u == 0) { orc_prefill(m, st[0], prompt, F); orc_prefill_tokens(m, st[0], ids, S); }
    else {
      memcpy(st[u]->kv, st[0]->kv, sizeof(float) * (size_t)NL * 2 * NH * st[0]->max_ctx * HD);
      st[u]->pos = st[0]->pos;
    }
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  /* one utterance per thread; nested parallel regions inside the ops stay serial */
  omp_set_max_active_levels(1);
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
  for (int u = 0; u < n_utt; ++u) {
    float lat[LDIM], pcm[FRAME];
    for (int f = 0; f < n_frames; ++f) orc_step(m, st[u], f ? lat : NULL, NULL, 1, NULL, NULL, lat, pcm, NULL, NULL, NULL);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  for (int u = 0; u < n_utt; ++u) orc_state_destroy(st[u]);
  free(st); free(prompt); free(ids);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
