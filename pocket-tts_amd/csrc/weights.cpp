// Weight sources and packing into the engine's device layout.
//
// Packed layouts (all fp32, row-major, rows padded to multiples of 32 where a GEMM reads them):
//   Linear W [N][K]                     (PyTorch layout, unchanged)
//   Conv1d W [Cout][k][Cin]             (from torch [Cout][Cin][k]; one K index = (tap, ci))
//   ConvTranspose1d (stride r, k = 2r)  polyphase [phase p][Cout][2][Cin] with
//       tap 0 (input frame q-1) = W[ci][co][p + r], tap 1 (frame q) = W[ci][co][p]
//   cond_embed | out_eos                one [544][1024] matrix (rows 513.. zero)
//   the 6 ResBlock adaLN + FinalLayer adaLN projections: one [10240][512] matrix
#include "weights.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <stdexcept>

#include "common.h"

namespace ptts {

// ------------------------------------------------------------------ synthetic source
namespace {
uint64_t fnv1a64(const std::string& s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x100000001B3ull;
  }
  return h;
}
uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
bool has(const std::string& s, const char* t) { return s.find(t) != std::string::npos; }
bool ends(const std::string& s, const char* t) {
  size_t n = strlen(t);
  return s.size() >= n && s.compare(s.size() - n, n, t) == 0;
}

// init_rule() of tests/golden/synth.py
bool init_rule(const std::string& name, const std::vector<int64_t>& shape, double& c, double& hw) {
  size_t dot = name.rfind('.');
  std::string leaf = dot == std::string::npos ? name : name.substr(dot + 1);
  if (leaf == "freqs") return false;
  if (ends(name, "emb_std")) { c = 1.0; hw = 0.1; return true; }
  if (ends(name, "emb_mean")) { c = 0.0; hw = 0.1; return true; }
  if (ends(name, "bos_emb")) { c = 0.0; hw = std::sqrt(3.0); return true; }
  if (ends(name, "conditioner.embed.weight")) { c = 0.0; hw = 1.0; return true; }
  if (leaf == "alpha") { c = 1.0; hw = 0.1; return true; }
  if (leaf == "scale" && has(name, "layer_scale")) { c = 0.01; hw = 0.005; return true; }
  bool is_norm = has(name, "norm1.") || has(name, "norm2.") || has(name, "out_norm.") || has(name, "in_ln.");
  if (is_norm && leaf == "weight") { c = 1.0; hw = 0.1; return true; }
  if (is_norm && leaf == "bias") { c = 0.0; hw = 0.1; return true; }
  if (leaf == "bias") { c = 0.0; hw = 0.05; return true; }
  if (shape.size() >= 2) {
    int64_t fan = 1;
    for (size_t i = 1; i < shape.size(); ++i) fan *= shape[i];
    c = 0.0;
    hw = 1.0 / std::sqrt((double)fan);
    return true;
  }
  throw Error(PTTS_ERR_INVALID, "no synthetic init rule for " + name);
}

class SynthSource : public TensorSource {
 public:
  explicit SynthSource(uint64_t seed) : seed_(seed) {}
  std::vector<float> get(const std::string& name, const std::vector<int64_t>& shape) override {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    double c = 0, hw = 0;
    if (!init_rule(name, shape, c, hw)) throw Error(PTTS_ERR_INVALID, "tensor is not synthetic: " + name);
    std::vector<float> out((size_t)n);
    const uint64_t base = seed_ * 0x9E3779B97F4A7C15ull + fnv1a64(name);
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t z = mix64(base + (uint64_t)i * 0xD1B54A32D192ED03ull);
      const double u = (double)(z >> 40) * (1.0 / 16777216.0);
      out[(size_t)i] = (float)(c + (2.0 * u - 1.0) * hw);
    }
    return out;
  }

 private:
  uint64_t seed_;
};

// ------------------------------------------------------------------ safetensors source
float bf16_to_f32(uint16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
float f16_to_f32(uint16_t h) {
  const uint32_t s = (h >> 15) & 1, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? NAN : INFINITY;
  else v = std::ldexp((float)(m | 0x400), (int)e - 25);
  return s ? -v : v;
}

class SafetensorsSource : public TensorSource {
 public:
  explicit SafetensorsSource(const std::string& path) {
    fd_ = open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw Error(PTTS_ERR_IO, "cannot open weights file " + path);
    struct stat st;
    fstat(fd_, &st);
    size_ = (size_t)st.st_size;
    map_ = (const uint8_t*)mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (map_ == MAP_FAILED) throw Error(PTTS_ERR_IO, "mmap failed for " + path);
    uint64_t hlen = 0;
    if (size_ < 8) throw Error(PTTS_ERR_IO, "truncated safetensors file");
    memcpy(&hlen, map_, 8);
    if (8 + hlen > size_) throw Error(PTTS_ERR_IO, "bad safetensors header length");
    parse(std::string((const char*)map_ + 8, hlen));
    data_ = map_ + 8 + hlen;
  }
  ~SafetensorsSource() override {
    if (map_ && map_ != MAP_FAILED) munmap((void*)map_, size_);
    if (fd_ >= 0) close(fd_);
  }
  std::vector<float> get(const std::string& name, const std::vector<int64_t>& shape) override {
    auto it = entries_.find(name);
    if (it == entries_.end()) throw Error(PTTS_ERR_IO, "tensor missing in weights file: " + name);
    const Entry& e = it->second;
    int64_t n = 1, ne = 1;
    for (auto d : shape) n *= d;
    for (auto d : e.shape) ne *= d;
    if (n != ne || e.shape != shape) throw Error(PTTS_ERR_IO, "shape mismatch for " + name);
    if (e.end - e.begin != (size_t)n * (e.dtype == "F32" ? 4 : 2) || data_ + e.end > map_ + size_)
      throw Error(PTTS_ERR_IO, "data_offsets out of range for " + name);
    std::vector<float> out((size_t)n);
    const uint8_t* p = data_ + e.begin;
    if (e.dtype == "F32") {
      memcpy(out.data(), p, (size_t)n * 4);
    } else if (e.dtype == "BF16" || e.dtype == "F16") {
      for (int64_t i = 0; i < n; ++i) {
        uint16_t v;
        memcpy(&v, p + 2 * i, 2);
        out[(size_t)i] = e.dtype == "BF16" ? bf16_to_f32(v) : f16_to_f32(v);
      }
    } else {
      throw Error(PTTS_ERR_IO, "unsupported dtype " + e.dtype + " for " + name);
    }
    return out;
  }

 private:
  struct Entry {
    std::string dtype;
    std::vector<int64_t> shape;
    size_t begin = 0, end = 0;
  };
  // Minimal parser for the safetensors header: {"name": {"dtype": "...", "shape": [...],
  // "data_offsets": [a, b]}, "__metadata__": {...}}
  void parse(const std::string& j) {
    size_t i = 0;
    auto ws = [&] { while (i < j.size() && isspace((unsigned char)j[i])) ++i; };
    auto str = [&]() -> std::string {
      ws();
      if (j[i] != '"') throw Error(PTTS_ERR_IO, "safetensors header: expected string");
      ++i;
      std::string s;
      while (i < j.size() && j[i] != '"') {
        if (j[i] == '\\') ++i;
        s += j[i++];
      }
      ++i;
      return s;
    };
    auto num = [&]() -> int64_t {
      ws();
      size_t k = i;
      while (i < j.size() && (isdigit((unsigned char)j[i]) || j[i] == '-')) ++i;
      return std::stoll(j.substr(k, i - k));
    };
    auto ints = [&]() -> std::vector<int64_t> {
      std::vector<int64_t> v;
      ws();
      ++i;  // [
      ws();
      if (j[i] == ']') { ++i; return v; }
      for (;;) {
        v.push_back(num());
        ws();
        if (j[i] == ',') { ++i; continue; }
        ++i;  // ]
        return v;
      }
    };
    std::function<void()> skip = [&]() {
      ws();
      if (j[i] == '"') { str(); return; }
      if (j[i] == '{' || j[i] == '[') {
        char open_c = j[i], close_c = open_c == '{' ? '}' : ']';
        int depth = 0;
        bool in_str = false;
        for (; i < j.size(); ++i) {
          char ch = j[i];
          if (in_str) {
            if (ch == '\\') ++i;
            else if (ch == '"') in_str = false;
            continue;
          }
          if (ch == '"') in_str = true;
          else if (ch == open_c) ++depth;
          else if (ch == close_c && --depth == 0) { ++i; return; }
        }
        return;
      }
      while (i < j.size() && j[i] != ',' && j[i] != '}') ++i;
    };
    ws();
    ++i;  // {
    for (;;) {
      ws();
      if (j[i] == '}') break;
      std::string key = str();
      ws();
      ++i;  // :
      if (key == "__metadata__") {
        skip();
      } else {
        Entry e;
        ws();
        ++i;  // {
        for (;;) {
          ws();
          if (j[i] == '}') { ++i; break; }
          std::string f = str();
          ws();
          ++i;  // :
          if (f == "dtype") e.dtype = str();
          else if (f == "shape") e.shape = ints();
          else if (f == "data_offsets") {
            auto v = ints();
            if (v.size() != 2) throw Error(PTTS_ERR_IO, "bad data_offsets");
            e.begin = (size_t)v[0];
            e.end = (size_t)v[1];
          } else skip();
          ws();
          if (j[i] == ',') ++i;
        }
        entries_[key] = e;
      }
      ws();
      if (j[i] == ',') ++i;
    }
  }
  int fd_ = -1;
  size_t size_ = 0;
  const uint8_t* map_ = nullptr;
  const uint8_t* data_ = nullptr;
  std::map<std::string, Entry> entries_;
};
}  // namespace

// ------------------------------------------------------------------ quantization (quantize.rs)
namespace {
class QuantSource : public TensorSource {
 public:
  QuantSource(std::unique_ptr<TensorSource> base, int mode) : base_(std::move(base)), mode_(mode) {}
  std::vector<float> get(const std::string& name, const std::vector<int64_t>& shape) override {
    std::vector<float> v = base_->get(name, shape);
    if (quant_applies(name, v.size(), mode_)) scales_[name] = quantize_inplace(v);
    return v;
  }
  int quant_mode() const override { return mode_; }
  float quant_scale(const std::string& name) const override {
    auto it = scales_.find(name);
    return it == scales_.end() ? 0.f : it->second;
  }

 private:
  std::unique_ptr<TensorSource> base_;
  int mode_;
  std::map<std::string, float> scales_;
};
}  // namespace

bool quant_applies(const std::string& name, size_t numel, int mode) {
  // QuantizeConfig::default() (quantize.rs:27-40): skip_layers, min_size 1024
  static const char* const kSkip[] = {"embed", "lut", "out_proj", "eos_head"};
  if (mode == QUANT_NONE || numel < 1024) return false;
  for (const char* k : kSkip)
    if (has(name, k)) return false;  // should_skip_layer (quantize.rs:120-123): substring match
  return mode == QUANT_ALL || name.compare(0, 8, "flow_lm.") == 0;
}

float quantize_inplace(std::vector<float>& v, int num_levels) {
  // QuantizedTensor::quantize (quantize.rs:66-90), all in f32 as Candle computes it:
  // abs_max = max|x|; scale = abs_max / (half - 1); q = clamp(round(x / scale), +-(half - 1));
  // data = q * scale. round() is half away from zero (Rust f32::round).
  float amax = 0.f;
  for (float x : v) amax = std::max(amax, std::fabs(x));
  const float half = (float)(num_levels / 2);
  const float scale = amax > 0.f ? amax / (half - 1.0f) : 1.0f;
  const float lim = half - 1.0f;
  for (float& x : v) {
    float q = std::round(x / scale);
    q = std::min(std::max(q, -lim), lim);
    x = q * scale;
  }
  return scale;
}

std::unique_ptr<TensorSource> make_quant_source(std::unique_ptr<TensorSource> base, int mode) {
  if (mode < QUANT_NONE || mode > QUANT_ALL) throw Error(PTTS_ERR_INVALID, "unknown weight_quant mode");
  if (mode == QUANT_NONE) return base;
  return std::make_unique<QuantSource>(std::move(base), mode);
}

std::unique_ptr<TensorSource> make_synth_source(uint64_t seed) { return std::make_unique<SynthSource>(seed); }
std::unique_ptr<TensorSource> make_safetensors_source(const std::string& path) {
  return std::make_unique<SafetensorsSource>(path);
}

// ------------------------------------------------------------------ packing
Layout pack_weights(TensorSource* src, float* dst) {
  Layout L{};
  size_t cur = 0;
  auto alloc = [&](size_t n) {
    size_t off = cur;
    cur += (n + 63) / 64 * 64;  // 256-byte aligned tensors
    return off;
  };
  auto fetch = [&](const std::string& name, std::vector<int64_t> shape) { return src->get(name, shape); };
  // plain copy of a tensor
  auto put = [&](const std::string& name, std::vector<int64_t> shape) {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    size_t off = alloc((size_t)n);
    if (dst) {
      auto v = fetch(name, shape);
      memcpy(dst + off, v.data(), v.size() * sizeof(float));
    }
    return off;
  };
  // Conv1d [cout][cin][k] -> [cout_pad][k][cin]
  auto put_conv = [&](const std::string& name, int cout, int cin, int k, int cout_pad) {
    size_t off = alloc((size_t)cout_pad * k * cin);
    if (dst) {
      auto v = fetch(name, {cout, cin, k});
      float* o = dst + off;
      memset(o, 0, sizeof(float) * (size_t)cout_pad * k * cin);
      for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < cin; ++ci)
          for (int j = 0; j < k; ++j) o[((size_t)co * k + j) * cin + ci] = v[((size_t)co * cin + ci) * k + j];
    }
    return off;
  };
  // ConvTranspose1d [cin][cout][2r] -> polyphase [r][cout][2][cin]
  auto put_convtr = [&](const std::string& name, int cin, int cout, int r) {
    size_t off = alloc((size_t)r * cout * 2 * cin);
    if (dst) {
      auto v = fetch(name, {cin, cout, 2 * r});
      float* o = dst + off;
      for (int p = 0; p < r; ++p)
        for (int co = 0; co < cout; ++co)
          for (int ci = 0; ci < cin; ++ci) {
            o[(((size_t)p * cout + co) * 2 + 0) * cin + ci] = v[((size_t)ci * cout + co) * 2 * r + p + r];
            o[(((size_t)p * cout + co) * 2 + 1) * cin + ci] = v[((size_t)ci * cout + co) * 2 * r + p];
          }
    }
    return off;
  };
  auto layer = [&](Layout::TL& t, const std::string& p, int d, int ff, bool ls) {
    t.in_proj = put(p + ".self_attn.in_proj.weight", {3 * d, d});
    t.out_proj = put(p + ".self_attn.out_proj.weight", {d, d});
    t.n1w = put(p + ".norm1.weight", {d});
    t.n1b = put(p + ".norm1.bias", {d});
    t.n2w = put(p + ".norm2.weight", {d});
    t.n2b = put(p + ".norm2.bias", {d});
    t.l1 = put(p + ".linear1.weight", {ff, d});
    t.l2 = put(p + ".linear2.weight", {d, ff});
    t.ls1 = ls ? put(p + ".layer_scale_1.scale", {d}) : 0;
    t.ls2 = ls ? put(p + ".layer_scale_2.scale", {d}) : 0;
  };
  const std::string F = "flow_lm.", FN = "flow_lm.flow_net.";
  // ---------------- FlowLM (flow_lm.rs:67-95)
  L.embed = put(F + "conditioner.embed.weight", {VOCAB, D});
  L.bos = put(F + "bos_emb", {LDIM});
  L.emb_mean = put(F + "emb_mean", {LDIM});
  L.emb_std = put(F + "emb_std", {LDIM});
  L.input_linear = put(F + "input_linear.weight", {D, LDIM});
  for (int l = 0; l < NL; ++l) layer(L.fl[l], F + "transformer.layers." + std::to_string(l), D, FF, false);
  L.out_norm_w = put(F + "out_norm.weight", {D});
  L.out_norm_b = put(F + "out_norm.bias", {D});
  L.cond_eos_w = alloc((size_t)NCOND_PAD * D);
  L.cond_eos_b = alloc(NCOND_PAD);
  if (dst) {
    auto cw = fetch(FN + "cond_embed.weight", {FD, D});
    auto cb = fetch(FN + "cond_embed.bias", {FD});
    auto ew = fetch(F + "out_eos.weight", {1, D});
    auto eb = fetch(F + "out_eos.bias", {1});
    memset(dst + L.cond_eos_w, 0, sizeof(float) * NCOND_PAD * D);
    memset(dst + L.cond_eos_b, 0, sizeof(float) * NCOND_PAD);
    memcpy(dst + L.cond_eos_w, cw.data(), cw.size() * 4);
    memcpy(dst + L.cond_eos_w + (size_t)FD * D, ew.data(), ew.size() * 4);
    memcpy(dst + L.cond_eos_b, cb.data(), cb.size() * 4);
    dst[L.cond_eos_b + FD] = eb[0];
  }
  for (int i = 0; i < 2; ++i) {
    const std::string p = FN + "time_embed." + std::to_string(i) + ".mlp.";
    L.te_l1w[i] = put(p + "0.weight", {FD, 256});
    L.te_l1b[i] = put(p + "0.bias", {FD});
    L.te_l2w[i] = put(p + "2.weight", {FD, FD});
    L.te_l2b[i] = put(p + "2.bias", {FD});
    L.te_alpha[i] = put(p + "3.alpha", {FD});
  }
  L.inproj_w = put(FN + "input_proj.weight", {FD, LDIM});
  L.inproj_b = put(FN + "input_proj.bias", {FD});
  L.ada_w = alloc((size_t)NADA * FD);
  L.ada_b = alloc(NADA);
  if (dst) {
    for (int b = 0; b < FDEPTH; ++b) {
      const std::string p = FN + "res_blocks." + std::to_string(b) + ".adaLN_modulation.1.";
      auto w = fetch(p + "weight", {3 * FD, FD});
      auto bb = fetch(p + "bias", {3 * FD});
      memcpy(dst + L.ada_w + (size_t)b * 3 * FD * FD, w.data(), w.size() * 4);
      memcpy(dst + L.ada_b + (size_t)b * 3 * FD, bb.data(), bb.size() * 4);
    }
    auto w = fetch(FN + "final_layer.adaLN_modulation.1.weight", {2 * FD, FD});
    auto bb = fetch(FN + "final_layer.adaLN_modulation.1.bias", {2 * FD});
    memcpy(dst + L.ada_w + (size_t)FDEPTH * 3 * FD * FD, w.data(), w.size() * 4);
    memcpy(dst + L.ada_b + (size_t)FDEPTH * 3 * FD, bb.data(), bb.size() * 4);
  }
  for (int b = 0; b < FDEPTH; ++b) {
    const std::string p = FN + "res_blocks." + std::to_string(b) + ".";
    L.rb_lnw[b] = put(p + "in_ln.weight", {FD});
    L.rb_lnb[b] = put(p + "in_ln.bias", {FD});
    L.rb_w0[b] = put(p + "mlp.0.weight", {FD, FD});
    L.rb_b0[b] = put(p + "mlp.0.bias", {FD});
    L.rb_w2[b] = put(p + "mlp.2.weight", {FD, FD});
    L.rb_b2[b] = put(p + "mlp.2.bias", {FD});
  }
  L.fin_w = put(FN + "final_layer.linear.weight", {LDIM, FD});
  L.fin_b = put(FN + "final_layer.linear.bias", {LDIM});
  L.speaker_proj = put(F + "speaker_proj_weight", {D, MD});
  // ---------------- Mimi (mimi.rs:55-107, seanet.rs)
  L.quant_w = put("mimi.quantizer.output_proj.weight", {MD, LDIM, 1});
  L.up_w = put("mimi.upsample.convtr.convtr.weight", {MD, 1, 2 * UP});
  for (int l = 0; l < MNL; ++l) {
    layer(L.mdec[l], "mimi.decoder_transformer.transformer.layers." + std::to_string(l), MD, MFF, true);
    layer(L.menc[l], "mimi.encoder_transformer.transformer.layers." + std::to_string(l), MD, MFF, true);
  }
  L.dc0_w = put_conv("mimi.decoder.model.0.conv.weight", 512, 512, 7, 512);
  L.dc0_b = put("mimi.decoder.model.0.conv.bias", {512});
  int ch = 512;
  for (int i = 0; i < 3; ++i) {
    const int li = 2 + 3 * i, r = RATIOS[i];
    const std::string p = "mimi.decoder.model.";
    L.dtr_w[i] = put_convtr(p + std::to_string(li) + ".convtr.weight", ch, ch / 2, r);
    L.dtr_b[i] = put(p + std::to_string(li) + ".convtr.bias", {ch / 2});
    ch /= 2;
    L.dra_w[i] = put_conv(p + std::to_string(li + 1) + ".block.1.conv.weight", ch / 2, ch, 3, ch / 2);
    L.dra_b[i] = put(p + std::to_string(li + 1) + ".block.1.conv.bias", {ch / 2});
    L.drb_w[i] = put_conv(p + std::to_string(li + 1) + ".block.3.conv.weight", ch, ch / 2, 1, ch);
    L.drb_b[i] = put(p + std::to_string(li + 1) + ".block.3.conv.bias", {ch});
  }
  L.dfin_w = put_conv("mimi.decoder.model.11.conv.weight", 1, 64, 3, 1);
  L.dfin_b = put("mimi.decoder.model.11.conv.bias", {1});
  // encoder (seanet.rs:148-247): ratios reversed [4, 5, 6]
  L.ec0_w = put("mimi.encoder.model.0.conv.weight", {64, 1, 7});
  L.ec0_b = put("mimi.encoder.model.0.conv.bias", {64});
  ch = 64;
  for (int i = 0; i < 3; ++i) {
    const int li = 1 + 3 * i, r = RATIOS[2 - i];
    const std::string p = "mimi.encoder.model.";
    L.era_w[i] = put_conv(p + std::to_string(li) + ".block.1.conv.weight", ch / 2, ch, 3, ch / 2);
    L.era_b[i] = put(p + std::to_string(li) + ".block.1.conv.bias", {ch / 2});
    L.erb_w[i] = put_conv(p + std::to_string(li) + ".block.3.conv.weight", ch, ch / 2, 1, ch);
    L.erb_b[i] = put(p + std::to_string(li) + ".block.3.conv.bias", {ch});
    L.edn_w[i] = put_conv(p + std::to_string(li + 2) + ".conv.weight", 2 * ch, ch, 2 * r, 2 * ch);
    L.edn_b[i] = put(p + std::to_string(li + 2) + ".conv.bias", {2 * ch});
    ch *= 2;
  }
  L.efin_w = put_conv("mimi.encoder.model.11.conv.weight", 512, 512, 3, 512);
  L.efin_b = put("mimi.encoder.model.11.conv.bias", {512});
  L.down_w = put_conv("mimi.downsample.conv.conv.weight", 512, 512, 32, 512);

  // ---------------- quantized storage: mode marker and int8-code row scales. Rows take the
  // scale of the tensor they were packed from; a matrix with any unquantized part is skipped
  // at finalize (its scale rows hold 0 there).
  L.qmode = alloc(1);
  if (dst) dst[L.qmode] = src ? (float)src->quant_mode() : 0.f;
  auto q8 = [&](size_t w, int N, int K, std::vector<std::pair<std::string, int>> parts) {
    Layout::Q8 q{w, alloc((size_t)N), N, K};
    if (dst) {
      int row = 0;
      for (auto& pr : parts) {
        const float sc = src ? src->quant_scale(pr.first) : 0.f;
        for (int i = 0; i < pr.second; ++i) dst[q.s + row++] = sc;
      }
      if (row != N) throw Error(PTTS_ERR_INVALID, "int8 scale rows do not cover the matrix");
    }
    L.q8.push_back(q);
  };
  for (int l = 0; l < NL; ++l) {
    const std::string p = F + "transformer.layers." + std::to_string(l);
    q8(L.fl[l].in_proj, 3 * D, D, {{p + ".self_attn.in_proj.weight", 3 * D}});
    q8(L.fl[l].l1, FF, D, {{p + ".linear1.weight", FF}});
    q8(L.fl[l].l2, D, FF, {{p + ".linear2.weight", D}});
  }
  q8(L.input_linear, D, LDIM, {{F + "input_linear.weight", D}});
  q8(L.inproj_w, FD, LDIM, {{FN + "input_proj.weight", FD}});
  {
    std::vector<std::pair<std::string, int>> parts;
    for (int b = 0; b < FDEPTH; ++b)
      parts.push_back({FN + "res_blocks." + std::to_string(b) + ".adaLN_modulation.1.weight", 3 * FD});
    parts.push_back({FN + "final_layer.adaLN_modulation.1.weight", 2 * FD});
    q8(L.ada_w, NADA, FD, parts);
  }
  for (int b = 0; b < FDEPTH; ++b) {
    const std::string p = FN + "res_blocks." + std::to_string(b) + ".";
    q8(L.rb_w0[b], FD, FD, {{p + "mlp.0.weight", FD}});
    q8(L.rb_w2[b], FD, FD, {{p + "mlp.2.weight", FD}});
  }
  q8(L.fin_w, LDIM, FD, {{FN + "final_layer.linear.weight", LDIM}});
  L.total = cur;
  return L;
}

}  // namespace ptts
