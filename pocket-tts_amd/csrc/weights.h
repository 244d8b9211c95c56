// Weight sources (synthetic PRNG or local safetensors) and the packed device layout.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace ptts {

// Model dimensions of variant b6369a24 (config/b6369a24.yaml:6-56).
constexpr int D = 1024, NH = 16, HD = 64, NL = 6, FF = 4096, LDIM = 32, VOCAB = 4001;
constexpr int FD = 512, FDEPTH = 6, NCOND = 513, NCOND_PAD = 544, NADA = FDEPTH * 3 * FD + 2 * FD;
constexpr int MD = 512, MNH = 8, MNL = 2, MFF = 2048, MCTX = 250, UP = 16, FRAME = 1920;
constexpr int RING = 512;  // Mimi KV ring capacity >= context 250 + 16 new rows
constexpr int RATIOS[3] = {6, 5, 4};

class TensorSource {
 public:
  virtual ~TensorSource() = default;
  // Tensor `name` (TTSModel state-dict key) as fp32, checked against `shape`.
  virtual std::vector<float> get(const std::string& name, const std::vector<int64_t>& shape) = 0;
  // Quantization scope applied by this source (QuantMode) and the per-tensor scale it used for
  // `name` (0 = tensor kept in full precision). Plain sources quantize nothing.
  virtual int quant_mode() const { return 0; }
  virtual float quant_scale(const std::string&) const { return 0.f; }
};

// ---------------------------------------------------------------------------------------------
// Weight quantization of the reference (crates/pocket-tts/src/quantize.rs), restated:
// symmetric per-tensor int8 levels with QuantizeConfig::default() (skip names containing
// "embed", "lut", "out_proj", "eos_head"; tensors under 1024 elements stay f32; 256 levels).
// QUANT_FLOW_LM applies quantize_weights() to the flow_lm.* tensors (BASELINE configs[4],
// "int8-quantised FlowLM"), QUANT_ALL to the whole state dict.
enum QuantMode : int { QUANT_NONE = 0, QUANT_FLOW_LM = 1, QUANT_ALL = 2 };
// should_skip_layer / min_size test of quantize_weights (quantize.rs:120-150) plus the scope
bool quant_applies(const std::string& name, size_t numel, int mode);
// QuantizedTensor::quantize (quantize.rs:66-90) in place: v <- clamp(round(v/s), +-127) * s,
// s = max|v| / 127 (1 for an all-zero tensor). Returns s.
float quantize_inplace(std::vector<float>& v, int num_levels = 256);
// `base` with quantize_inplace applied to every tensor quant_applies() selects.
std::unique_ptr<TensorSource> make_quant_source(std::unique_ptr<TensorSource> base, int mode);

// Counter-based synthetic weights, bit-identical to tests/golden/synth.py.
std::unique_ptr<TensorSource> make_synth_source(uint64_t seed);
// Local safetensors file (F32 / BF16 / F16 tensors); throws on missing tensors.
std::unique_ptr<TensorSource> make_safetensors_source(const std::string& path);

// Offsets (in floats) of every packed tensor in the device weight blob.
struct Layout {
  struct TL {
    size_t in_proj, out_proj, n1w, n1b, n2w, n2b, l1, l2, ls1, ls2;
  };
  // FlowLM
  size_t embed, bos, emb_mean, emb_std, input_linear, out_norm_w, out_norm_b, cond_eos_w, cond_eos_b;
  TL fl[NL];
  size_t te_l1w[2], te_l1b[2], te_l2w[2], te_l2b[2], te_alpha[2];
  size_t inproj_w, inproj_b, ada_w, ada_b;
  size_t rb_lnw[FDEPTH], rb_lnb[FDEPTH], rb_w0[FDEPTH], rb_b0[FDEPTH], rb_w2[FDEPTH], rb_b2[FDEPTH];
  size_t fin_w, fin_b, speaker_proj;
  // Mimi
  size_t quant_w, up_w;
  TL mdec[MNL], menc[MNL];
  size_t dc0_w, dc0_b, dtr_w[3], dtr_b[3], dra_w[3], dra_b[3], drb_w[3], drb_b[3], dfin_w, dfin_b;
  size_t ec0_w, ec0_b, era_w[3], era_b[3], erb_w[3], erb_b[3], edn_w[3], edn_b[3], efin_w, efin_b, down_w;
  // Quantized storage. `qmode` is one float holding the QuantMode the blob was packed with.
  // Every FlowLM step GEMM weight whose source tensors were all quantized gets an int8 code
  // matrix at engine finalize: codes q[n][k] = W[n][k] / s[n] with the row scales s packed in
  // the blob (the per-tensor scale of the source tensor each row came from; 0 = not quantized).
  struct Q8 {
    size_t w, s;  // f32 weights [N][K], row scales [N]
    int N, K;
  };
  size_t qmode;
  std::vector<Q8> q8;
  size_t total;
};

// Compute the layout (dst == nullptr) or also pack every tensor from `src` into host memory `dst`.
Layout pack_weights(TensorSource* src, float* dst);

}  // namespace ptts
