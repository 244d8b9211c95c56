// extern "C" boundary (include/pocket_tts.h): exceptions -> status codes + thread-local message.
#include <cstdlib>
#include <cstring>
#include <string>

#include "engine.h"
#include "pocket_tts.h"
#include "pocket_tts_probe.h"

struct ptts_engine {
  ptts::Engine* impl = nullptr;
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F&& f) {
  try {
    f();
    g_err.clear();
    return PTTS_OK;
  } catch (const ptts::Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "host out of memory";
    return PTTS_ERR_HIP;
  } catch (const std::exception& e) {
    g_err = e.what();
    return PTTS_ERR_INVALID;
  }
}
ptts::Engine& eng(ptts_engine* e) {
  if (!e || !e->impl) throw ptts::Error(PTTS_ERR_INVALID, "null engine");
  return *e->impl;
}

// HIP runtime setting read when the runtime initializes (the process's first HIP call, normally
// after this library is loaded): graphs launched as their kernel nodes instead of pre-captured AQL
// packets. The step graphs run 0.7 % faster that way (steady step 0.5027 -> 0.4991 ms, same-box
// A/B medians of 4, profiles/r06/ab_env2.txt). A value the caller set is kept; a process that
// initialized HIP before loading this library keeps the runtime's default.
__attribute__((constructor)) void ptts_runtime_env() { setenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0", 0); }
}  // namespace

extern "C" {

int ptts_abi_version(void) { return PTTS_ABI_VERSION; }

size_t ptts_weight_blob_bytes(void) { return ptts::pack_weights(nullptr, nullptr).total * sizeof(float); }

int ptts_pack_weights(uint64_t synth_seed, const char* weights_path, float* host_out, size_t n_bytes) {
  return ptts_pack_weights_ex(synth_seed, weights_path, PTTS_QUANT_NONE, host_out, n_bytes);
}

int ptts_pack_weights_ex(uint64_t synth_seed, const char* weights_path, int weight_quant, float* host_out,
                         size_t n_bytes) {
  return guard([&] {
    if (!host_out) throw ptts::Error(PTTS_ERR_INVALID, "null output buffer");
    const size_t need = ptts::pack_weights(nullptr, nullptr).total * sizeof(float);
    if (n_bytes < need) throw ptts::Error(PTTS_ERR_INVALID, "output buffer smaller than ptts_weight_blob_bytes()");
    std::unique_ptr<ptts::TensorSource> src = weights_path && weights_path[0]
                                                  ? ptts::make_safetensors_source(weights_path)
                                                  : ptts::make_synth_source(synth_seed);
    src = ptts::make_quant_source(std::move(src), weight_quant);
    std::memset(host_out, 0, need);
    ptts::pack_weights(src.get(), host_out);
  });
}

namespace {
// Records the (name, shape) of every tensor pack_weights() reads; returns zeros.
class ManifestSource : public ptts::TensorSource {
 public:
  std::string text;
  std::vector<float> get(const std::string& name, const std::vector<int64_t>& shape) override {
    int64_t n = 1;
    text += name + "\t";
    for (size_t i = 0; i < shape.size(); ++i) {
      text += (i ? "," : "") + std::to_string(shape[i]);
      n *= shape[i];
    }
    text += "\n";
    return std::vector<float>((size_t)n, 0.f);
  }
};
}  // namespace

int ptts_weight_manifest(char* buf, size_t cap, size_t* needed) {
  return guard([&] {
    ManifestSource ms;
    std::vector<float> scratch(ptts::pack_weights(nullptr, nullptr).total, 0.f);
    ptts::pack_weights(&ms, scratch.data());
    if (needed) *needed = ms.text.size() + 1;
    if (buf && cap) {
      const size_t n = std::min(cap - 1, ms.text.size());
      std::memcpy(buf, ms.text.data(), n);
      buf[n] = 0;
      if (n < ms.text.size()) throw ptts::Error(PTTS_ERR_INVALID, "manifest buffer too small");
    }
  });
}

int ptts_quantize_tensor(const float* x, size_t n, int num_levels, float* out, float* scale) {
  return guard([&] {
    if ((!x || !out) && n) throw ptts::Error(PTTS_ERR_INVALID, "null tensor");
    if (num_levels < 4) throw ptts::Error(PTTS_ERR_INVALID, "num_levels must be >= 4");
    std::vector<float> v(x, x + n);
    const float s = ptts::quantize_inplace(v, num_levels);
    if (n) std::memcpy(out, v.data(), n * sizeof(float));
    if (scale) *scale = s;
  });
}

int ptts_quant_applies(const char* name, size_t numel, int weight_quant) {
  return name && ptts::quant_applies(name, numel, weight_quant) ? 1 : 0;
}

int ptts_engine_int8_matrices(ptts_engine* e) { return (e && e->impl) ? e->impl->int8_matrices() : 0; }
int ptts_engine_fp8_matrices(ptts_engine* e) { return (e && e->impl) ? e->impl->fp8_matrices() : 0; }

int ptts_config_check(const char* cfg_yaml) {
  return guard([&] {
    if (!cfg_yaml || !*cfg_yaml) throw ptts::Error(PTTS_ERR_INVALID, "null model config path");
    ptts::check_model_config(cfg_yaml);
  });
}

int ptts_engine_create(const ptts_engine_config* cfg, ptts_engine** out) {
  return guard([&] {
    if (!cfg || !out) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    *out = nullptr;
    auto* h = new ptts_engine();
    try {
      h->impl = new ptts::Engine(*cfg);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int ptts_engine_load_blob(ptts_engine* e, const float* host_blob, size_t n_bytes) {
  return guard([&] {
    if (!host_blob) throw ptts::Error(PTTS_ERR_INVALID, "null blob");
    eng(e).load_blob(host_blob, n_bytes);
  });
}

int ptts_engine_finalize(ptts_engine* e) { return guard([&] { eng(e).finalize(); }); }

void ptts_engine_destroy(ptts_engine* e) {
  if (!e) return;
  delete e->impl;
  delete e;
}

void* ptts_engine_weight_blob(ptts_engine* e) { return (e && e->impl) ? e->impl->blob() : nullptr; }

int ptts_voice_from_prompt(ptts_engine* e, const float* prompt, int n_frames, ptts_voice** out) {
  return guard([&] {
    if (!out) throw ptts::Error(PTTS_ERR_INVALID, "null out");
    *out = eng(e).voice_from_prompt(prompt, n_frames);
  });
}

int ptts_voice_from_pcm(ptts_engine* e, const float* pcm, int n_samples, ptts_voice** out) {
  return guard([&] {
    if (!out) throw ptts::Error(PTTS_ERR_INVALID, "null out");
    *out = eng(e).voice_from_pcm(pcm, n_samples);
  });
}

int ptts_voice_from_audio(ptts_engine* e, const float* samples, int n_samples, int sample_rate, int chunk_frames,
                          ptts_voice** out) {
  return guard([&] {
    if (!out) throw ptts::Error(PTTS_ERR_INVALID, "null out");
    *out = eng(e).voice_from_audio(samples, n_samples, sample_rate, chunk_frames);
  });
}

int ptts_resample_len(int n_samples, int sr_from, int sr_to) {
  if (n_samples <= 0 || sr_from <= 0 || sr_to <= 0) return 0;
  const ptts::ResamplePlan p = ptts::resample_plan(sr_from, sr_to);
  const long n = p.out_len(n_samples);
  return n < (1L << 30) ? (int)n : 0;
}

int ptts_resample(ptts_engine* e, const float* x, int n_samples, int sr_from, int sr_to, float* y) {
  return guard([&] { eng(e).resample_host(x, n_samples, sr_from, sr_to, y); });
}

int ptts_resample_len_ex(int n_samples, int sr_from, int sr_to, int resampler) {
  if (resampler == PTTS_RESAMPLE_POLY) return ptts_resample_len(n_samples, sr_from, sr_to);
  if (resampler != PTTS_RESAMPLE_RUBATO_SEPTIC || n_samples <= 0 || sr_from <= 0 || sr_to <= 0) return 0;
  if (sr_from == sr_to) return n_samples;
  const long n = ptts::septic_schedule(n_samples, sr_from, sr_to, nullptr, nullptr);
  return n < (1L << 30) ? (int)n : 0;
}

int ptts_resample_ex(ptts_engine* e, const float* x, int n_samples, int sr_from, int sr_to, int resampler, float* y) {
  return guard([&] { eng(e).resample_host(x, n_samples, sr_from, sr_to, y, resampler); });
}

int ptts_voice_from_audio_ex(ptts_engine* e, const float* samples, int n_samples, int sample_rate, int chunk_frames,
                             int resampler, ptts_voice** out) {
  return guard([&] {
    if (!out) throw ptts::Error(PTTS_ERR_INVALID, "null out");
    *out = eng(e).voice_from_audio(samples, n_samples, sample_rate, chunk_frames, resampler);
  });
}

int ptts_test_gemm(ptts_engine* e, int layout, int m, int n, int k, int splits, int tail_slices, const float* x,
                   const float* w, float* y) {
  return guard([&] { eng(e).test_gemm(layout, m, n, k, splits, tail_slices, x, w, y); });
}

int ptts_voice_len(const ptts_voice* v) { return v ? v->F : 0; }

int ptts_voice_conditioning(const ptts_voice* v, float* out, int max_rows) {
  return guard([&] {
    if (!v || !out) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    if (v->cond.empty()) throw ptts::Error(PTTS_ERR_STATE, "voice was not built from PCM");
    const int rows = std::min(max_rows, v->F);
    memcpy(out, v->cond.data(), sizeof(float) * rows * ptts::D);
  });
}

void ptts_voice_destroy(ptts_voice* v) { ptts::voice_destroy(v); }

int ptts_slot_open(ptts_engine* e, int slot, const ptts_voice* v, const int32_t* ids, int n_ids,
                   const ptts_gen_params* p) {
  return guard([&] {
    if (!p) throw ptts::Error(PTTS_ERR_INVALID, "null params");
    eng(e).slot_open(slot, v, ids, n_ids, *p);
  });
}

int ptts_slots_open(ptts_engine* e, int n, const int* slots, const ptts_voice* const* voices, const int32_t* ids,
                    const int* n_ids, const ptts_gen_params* params) {
  return guard([&] { eng(e).slots_open(n, slots, voices, ids, n_ids, params); });
}

int ptts_probe_overlap(ptts_engine* e, int n_rows, int reps, double* us8) {
  return guard([&] {
    if (!us8) throw ptts::Error(PTTS_ERR_INVALID, "null output");
    for (int i = 0; i < 8; ++i) us8[i] = 0.0;
    eng(e).overlap_probe(n_rows, reps, us8);
  });
}

int ptts_slot_close(ptts_engine* e, int slot) { return guard([&] { eng(e).slot_close(slot); }); }

int ptts_decode_latents(ptts_engine* e, int slot, const float* latents, int n_frames, float* pcm, float* quantized,
                        float* after_upsample, float* after_transformer) {
  return guard([&] { eng(e).decode_latents(slot, latents, n_frames, pcm, quantized, after_upsample, after_transformer); });
}

int ptts_slot_set_latent(ptts_engine* e, int slot, const float* latent32) {
  return guard([&] { eng(e).set_latent(slot, latent32); });
}

int ptts_step(ptts_engine* e, int n_rows, float* pcm, uint8_t* frame_valid, uint8_t* last, float* eos_logits,
              float* latents) {
  return guard([&] {
    auto& E = eng(e);
    E.step_async(n_rows);
    E.fetch(n_rows, pcm, frame_valid, last, eos_logits, latents);
  });
}

int ptts_step_async(ptts_engine* e, int n_rows) { return guard([&] { eng(e).step_async(n_rows); }); }

int ptts_flush_async(ptts_engine* e, int n_rows) { return guard([&] { eng(e).flush_async(n_rows); }); }

int ptts_sync(ptts_engine* e) { return guard([&] { eng(e).sync(); }); }

int ptts_fetch(ptts_engine* e, int n_rows, float* pcm, uint8_t* frame_valid, uint8_t* last, float* eos_logits,
               float* latents) {
  return guard([&] { eng(e).fetch(n_rows, pcm, frame_valid, last, eos_logits, latents); });
}

int ptts_fetch_prev(ptts_engine* e, int calls_back, int n_rows, float* pcm, uint8_t* frame_valid, uint8_t* last,
                    float* eos_logits, float* latents) {
  return guard([&] { eng(e).fetch(n_rows, pcm, frame_valid, last, eos_logits, latents, calls_back); });
}

int ptts_fetch_ready(ptts_engine* e, int calls_back, int* ready) {
  return guard([&] {
    if (!ready) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    *ready = eng(e).fetch_ready(calls_back) ? 1 : 0;
  });
}

int ptts_front_done(ptts_engine* e, int calls_back, int wait, int* done) {
  return guard([&] {
    if (!done) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    *done = eng(e).front_done(calls_back, wait != 0) ? 1 : 0;
  });
}

int ptts_preview_enable(ptts_engine* e, int max_rows) { return guard([&] { eng(e).preview_enable(max_rows); }); }

int ptts_preview_fetch(ptts_engine* e, int wait, int max_n, int* slots, float* pcm, int* n_out) {
  return guard([&] {
    if (!n_out) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    *n_out = 0;
    *n_out = eng(e).preview_fetch(wait, max_n, slots, pcm);
  });
}

int ptts_frame_lag(const ptts_engine* e, int* admit_delay) {
  if (!e || !e->impl) return -1;
  const ptts::Engine& E = *e->impl;
  if (admit_delay) *admit_delay = E.admit_delay();
  return E.frame_lag();
}

int ptts_generate(ptts_engine* e, int slot, const ptts_voice* v, const int32_t* ids, int n_ids,
                  const ptts_gen_params* p, float* pcm_out, int max_samples, int* n_samples) {
  return guard([&] {
    if (!p || !n_samples) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    auto& E = eng(e);
    E.slot_open(slot, v, ids, n_ids, *p);
    const int B = slot + 1;
    std::vector<float> pcm((size_t)B * ptts::FRAME);
    std::vector<uint8_t> valid(B), last(B);
    int total = 0;
    // a frame arrives frame_lag() calls after its step (+1 when the admission started a call late):
    // that many extra calls drain the last one
    const int lead = E.frame_lag() + E.admit_delay();
    for (int it = 0; it < p->max_frames + lead; ++it) {
      E.step_async(B);
      E.fetch(B, pcm.data(), valid.data(), last.data(), nullptr, nullptr);
      if (!valid[slot]) {
        if (it < lead) continue;
        break;
      }
      const int take = std::max(0, std::min(ptts::FRAME, max_samples - total));
      if (pcm_out && take > 0) memcpy(pcm_out + total, pcm.data() + (size_t)slot * ptts::FRAME, sizeof(float) * take);
      total += ptts::FRAME;
      if (last[slot]) break;
    }
    *n_samples = total;
  });
}

int ptts_time_kernel(ptts_engine* e, int n_rows, const char* name, int reps, double* avg_us) {
  return guard([&] {
    if (!name || !avg_us) throw ptts::Error(PTTS_ERR_INVALID, "null argument");
    *avg_us = eng(e).time_op(n_rows, name, reps);
  });
}

int ptts_plan_ops(ptts_engine* e, int n_rows, char* buf, int buflen) {
  return guard([&] {
    std::string s;
    for (auto& n : eng(e).plan_names(n_rows)) s += n + "\n";
    if (!buf || buflen <= (int)s.size()) throw ptts::Error(PTTS_ERR_INVALID, "buffer too small");
    memcpy(buf, s.c_str(), s.size() + 1);
  });
}

const char* ptts_last_error(void) { return g_err.c_str(); }

}  // extern "C"
