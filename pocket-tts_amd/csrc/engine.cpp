// Engine: device memory, step plan, HIP graphs, voice and slot management.
//
// Data layout in HBM (fp32):
//   weight blob                packed by weights.cpp (one allocation; RCCL-broadcastable)
//   FlowLM KV                  [slot][layer][k|v][head][max_ctx][64]   (attention.rs:211-231, preallocated;
//                              positions < F of an admitted slot are read from its voice's own
//                              [layer][k|v][head][F][64] cache, shared by every slot of that voice)
//   Mimi KV ring               [slot][layer][k|v][head][512][64]       (attention.rs:167-264, ctx 250)
//   conv histories             [slot][P][C] per streaming conv          (conv.rs:71-136, time-major)
//   activations                row-major [rows][features]; Mimi/SEANet channels-last [slot][time][ch]
#include "engine.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>

namespace ptts {

namespace {
// voice reference counts (ptts_voice::refs / dead): engines and ptts_voice_destroy may run on
// different host threads
std::mutex& voice_mu() {
  static std::mutex m;
  return m;
}

int pick_splits(int M, int N, int K) {
  const int tiles = ((N + 31) / 32) * ((M + 31) / 32);
  const int chunks = K / 32;
  int s = std::max(1, 768 / std::max(1, tiles));
  s = std::min(s, std::max(1, chunks / 4));
  return std::min(s, 16);  // k_row_reduce sums at most 16 slabs
}
}  // namespace

// Tuning override of an op's tile layout / split-K count (tools/back_tune.py, probe builds only):
// PTTS_OVR="name=L[:S],...", read at every plan build.
static void tile_override(const std::string& name, int& layout, int& ksplit) {
  const char* e = probe_env("PTTS_OVR");
  if (!e) return;
  const std::string s(e);
  size_t p = 0;
  while (p < s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    const std::string item = s.substr(p, q - p);
    p = q + 1;
    const size_t eq = item.find('=');
    if (eq == std::string::npos || item.compare(0, eq, name) != 0 || eq != name.size()) continue;
    const std::string v = item.substr(eq + 1);
    const size_t c = v.find(':');
    layout = atoi(v.substr(0, c).c_str());
    if (c != std::string::npos) ksplit = atoi(v.substr(c + 1).c_str());
  }
}

// layouts served by k_gemm_glds (kernels.hip gemm_launch): the only ones that split a conv's K
static bool lds_dma_layout(int layout) {
  return (layout >= 6 && layout <= 8) || (layout >= 11 && layout <= 16) || (layout >= 21 && layout <= 27) ||
         (layout >= 30 && layout <= 42) || (layout >= 130 && layout <= 139) || (layout >= 230 && layout <= 239);
}

float* Engine::dalloc(size_t n) {
  void* p = nullptr;
  PTTS_HIP(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(float)));
  PTTS_HIP(hipMemset(p, 0, std::max<size_t>(n, 1) * sizeof(float)));
  // hipMemset runs on the null stream, which does not order against the engine's non-blocking
  // streams: wait for it, or a kernel that fills the buffer next on stream_ can be overwritten
  // by the zeroing (seen: the transposed input-projection weight zeroed under quantized engines)
  PTTS_HIP(hipDeviceSynchronize());
  allocs_.push_back(p);
  return (float*)p;
}

Engine::Engine(const ptts_engine_config& cfg) {
  check_model_config(cfg.cfg_yaml);  // before any device work
  PTTS_REQUIRE(cfg.max_slots >= 1 && cfg.max_slots <= 256, "max_slots must be in [1, 256]");
  PTTS_REQUIRE(cfg.max_ctx >= 16 && cfg.max_ctx <= 8192, "max_ctx must be in [16, 8192]");
  PTTS_REQUIRE(cfg.lsd_decode_steps >= 1 && cfg.lsd_decode_steps <= 64, "lsd_decode_steps must be in [1, 64]");
  dev_ = cfg.device;
  max_slots_ = cfg.max_slots;
  max_ctx_ = cfg.max_ctx;
  lsd_ = cfg.lsd_decode_steps;
  PTTS_REQUIRE(cfg.weight_quant >= QUANT_NONE && cfg.weight_quant <= QUANT_ALL, "unknown weight_quant mode");
  wq_ = cfg.weight_quant;
  PTTS_REQUIRE(cfg.fp8_gemm == 0 || cfg.fp8_gemm == 1, "fp8_gemm must be 0 or 1");
  PTTS_REQUIRE(!(cfg.fp8_gemm && cfg.weight_quant != QUANT_NONE), "fp8_gemm and weight_quant are exclusive");
  fp8_ = cfg.fp8_gemm;
  PTTS_REQUIRE(cfg.back_frames >= 0 && cfg.back_frames <= NFR_MAX && !(cfg.back_frames & (cfg.back_frames - 1)),
               "back_frames must be 0, 1, 2, 4 or 8");
  nfr_ = cfg.pipeline && cfg.back_frames >= 2 ? cfg.back_frames : 1;
  PTTS_REQUIRE(cfg.back_mfma >= PTTS_BACK_F32 && cfg.back_mfma <= PTTS_BACK_F32X6, "unknown back_mfma mode");
  back_mfma_ = cfg.back_mfma;
  nhb_ = nfr_ > 1 ? 3 * nfr_ : 3;
  int ndev = 0;
  PTTS_HIP(hipGetDeviceCount(&ndev));
  PTTS_REQUIRE(dev_ >= 0 && dev_ < ndev, "HIP device ordinal out of range");
  PTTS_HIP(hipSetDevice(dev_));
  PTTS_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));

  L_ = pack_weights(nullptr, nullptr);
  if (cfg.weight_blob) {
    blob_ = (float*)cfg.weight_blob;
    own_blob_ = false;
  } else {
    blob_ = dalloc(L_.total);
  }

  const int B = max_slots_;
  kv_layer_ = (long)2 * NH * max_ctx_ * 64;
  kv_slot_ = kv_layer_ * NL;
  kv_ = dalloc((size_t)kv_slot_ * (B + 1));
  ring_layer_ = (long)2 * MNH * RING * 64;
  ring_slot_ = ring_layer_ * MNL;
  ring_ = dalloc((size_t)ring_slot_ * B);
  fpos_ = (int*)dalloc(B + 1);
  mpos_ = (int*)dalloc(B + 1);
  st_ = (SlotState*)dalloc((sizeof(SlotState) * B + 3) / 4);
  lat_in_ = dalloc((size_t)B * LDIM);
  cur_ = dalloc((size_t)B * LDIM);
  // overlap-add history [slot][512] (the last committed frame's quantizer output) and the
  // pass's quantizer outputs [slot][NFR_MAX][512], copied into it by the commit (quant_upsample)
  qprev_ = dalloc((size_t)(1 + NFR_MAX) * B * MD);
  qcur_ = qprev_ + (size_t)B * MD;
  eos_ = dalloc(B);
  static_assert(sizeof(FrameFlags) == 2 * sizeof(float), "FrameFlags packs into two floats");
  meta_floats_ = (size_t)B * (LDIM + 1 + 2);
  // multi-frame passes: pass p's PCM [B][nfr][1920] and the meta blocks of its buffers nfr p ..
  // nfr p + nfr - 1 in ONE device block and ONE pinned host block, so the pass delivers its frames
  // with one copy node (a 128-B multiple per meta block keeps FrameFlags 8-B aligned)
  const size_t mstride = (meta_floats_ + 31) / 32 * 32;
  if (nfr_ > 1)
    for (int p = 0; p < nhb_ / nfr_; ++p) {
      const size_t n = (size_t)B * nfr_ * FRAME + nfr_ * mstride;
      pcmp_[p] = dalloc(n);
      PTTS_HIP(hipHostMalloc((void**)&h_pcmp_[p], sizeof(float) * n, hipHostMallocDefault));
    }
  for (int q = 0; q < NHB; ++q) {  // front -> back hand-off buffers
    meta_[q] = nfr_ > 1 && q < nhb_ ? pcmp_[q / nfr_] + (size_t)B * nfr_ * FRAME + (q % nfr_) * mstride
                                    : dalloc(meta_floats_);
    lat_out_[q] = meta_[q];                                  // 128-B aligned,
    flags_[q] = (FrameFlags*)(meta_[q] + (size_t)B * LDIM);  // so FrameFlags stay 8-B aligned
    eos_out_[q] = meta_[q] + (size_t)B * (LDIM + 2);
    pcm_[q] = dalloc((size_t)B * FRAME);
  }
  fin_side_ = dalloc((size_t)B * (nfr_ * FRAME / RESBLOCK_FIN_TT) * 2);  // fused final conv's boundary shares
  PTTS_HIP(hipHostMalloc((void**)&h_act_, sizeof(SlotState) * B, hipHostMallocDefault));
  // back part's own split-K slabs: up to 8 slices of the Mimi / conv0 rows (B * 16 x 512), 4 of the
  // stage-0 transposed conv (B * 16 x 6 * 256), per frame of a pass
  mpcap_ = (size_t)nfr_ * std::max({(size_t)8 * B * UP * MD, (size_t)4 * B * UP * RATIOS[0] * (MD / 2)});
  mpartial_ = dalloc(mpcap_);

  // streaming conv histories (SEANetDecoder, seanet.rs:307-402): source T, channels, rows kept
  const int hT[8] = {16, 16, 96, 96, 480, 480, 1920, 1920};
  const int hC[8] = {512, 512, 256, 256, 128, 128, 64, 64};
  const int hP[8] = {6, 1, 2, 1, 2, 1, 2, 2};
  for (int i = 0; i < 8; ++i) {
    hist_T_[i] = hT[i];
    hist_C_[i] = hC[i];
    hist_P_[i] = hP[i];
    hist_[i] = dalloc((size_t)B * hP[i] * hC[i]);
  }

  const int R = std::max(B, PREFILL);
  x_ = dalloc((size_t)R * D);
  h_ = dalloc((size_t)R * D);
  q_ = dalloc((size_t)R * D);
  o_ = dalloc((size_t)R * D);
  u_ = dalloc((size_t)R * FF);
  // split-K slabs: skinny FlowLM/head GEMMs, and the 2-way split Mimi QKV (B*16 rows x 1536)
  pcap_ = std::max({(size_t)4 << 20, (size_t)2 * B * UP * 3 * MD, (size_t)PREFILL * FF});
  partial_ = dalloc(pcap_);
  tslab_ = dalloc(TAIL_CAP);
  tickets_ = (int*)dalloc(TICKETS);  // zero; every split-tail launch leaves them zero
  ids_dev_ = (int*)dalloc(PREFILL);
  rowtab_dev_ = (int*)dalloc(PREFILL);
  ctab_dev_ = (int*)dalloc(PREFILL);
  qrow_dev_ = (int*)dalloc(PREFILL);
  orow_dev_ = (int*)dalloc(PREFILL);
  admit_slots_ = (int*)dalloc(B);
  admit_st_ = (SlotState*)dalloc((sizeof(SlotState) * B + 3) / 4);
  admit_fpos_ = (int*)dalloc(B);
  vpre_ = (const float**)dalloc((sizeof(float*) * (B + 1) + 3) / 4);  // zero: no slot has a prefix
  vlen_ = (int*)dalloc(B + 1);
  slot_voice_.assign(B, nullptr);
  drained_.assign(B, 1);
  admit_call_.assign(B, -1);
  share_voice_ = probe_env("PTTS_NO_SHARED_VOICE") == nullptr;
#ifdef PTTS_PROBES
  if (probe_env("PTTS_STAMPS")) {
    stamp_ring_ = (unsigned long long*)dalloc((size_t)STAMP_CAP * 4);
    stamp_ctr_ = (unsigned*)dalloc(1);
  }
#endif
  // pipelined stepping: the back part's kernels run at most one workgroup per CU, so the
  // latency-bound front part always finds room on every CU (measured 0.735 -> 0.688 ms per step
  // for the GEMMs alone; tools/sweep_env.sh)
  // three hand-off buffers: the front part may run two frames ahead of the back part. With the
  // back part now the longer of the two alone (498 vs 441 us), the front no longer idles behind
  // it: steady step 0.6370 -> 0.6321 ms (medians of 4; when the front was the longer part, 3
  // buffers measured 0.5% slower).
  if (probe_env("PTTS_BACK_WG_CAP")) back_cap_ = atoi(probe_env("PTTS_BACK_WG_CAP"));
  if (probe_env("PTTS_FRONT_PRIO")) set_front_prio(atoi(probe_env("PTTS_FRONT_PRIO")));
  if (probe_env("PTTS_BACK_PRIO")) set_back_prio(atoi(probe_env("PTTS_BACK_PRIO")));
  if (probe_env("PTTS_FRONT_SKIP")) set_front_skip(atoi(probe_env("PTTS_FRONT_SKIP")));
  ysilu_ = dalloc((size_t)lsd_ * B * FD);
  mods_ = dalloc((size_t)lsd_ * B * NADA);
  xf_ = dalloc((size_t)B * FD);
  hf_ = dalloc((size_t)B * FD);
  uf_ = dalloc((size_t)B * FD);
  PTTS_REQUIRE(hx_floats(B) * 4 < (1ull << 31), "flow-head hand-off regions exceed 2 GB (lsd_decode_steps too large)");
  hx_ = dalloc(hx_floats(B));
  // adaLN shift / scale in the chain's fragment order (written by the adaLN reduce), zeroed:
  // rows past B in the last row group read finite values and are never stored
  fhm_ = dalloc((size_t)lsd_ * ((B + 15) / 16) * (FDEPTH + 1) * 2 * 16 * FD);
  PTTS_HIP(hipMemset(hx_, 0xFF, hx_floats(B) * 4));  // empty (the launch ahead re-arms the used part)
  PTTS_HIP(hipDeviceSynchronize());                    // null-stream memset: see dalloc
  hctr_ = (int*)dalloc(4 * ((B + 15) / 16) + 4);
  herr_ = (int*)dalloc(4);
  const size_t BF = (size_t)B * nfr_;  // utterance frames of one back-part pass
  mx_ = dalloc(BF * UP * MD);
  mh_ = dalloc(BF * UP * MD);
  mq_ = dalloc(BF * UP * MD);
  mo_ = dalloc(BF * UP * MD);
  mqkv_ = dalloc(BF * UP * 3 * MD);
  mu_ = dalloc(BF * UP * MFF);
  a0_ = dalloc(BF * 16 * 512);
  int T = 16, ch = 512;
  for (int i = 0; i < 3; ++i) {
    T *= RATIOS[i];
    ch /= 2;
    cb_[i] = dalloc(BF * T * ch);
    ce_[i] = dalloc(BF * T * ch);
    cv_[i] = dalloc(BF * T * (ch / 2));
    ca_[i] = dalloc(BF * T * ch);
    trb_[i] = dalloc((size_t)RATIOS[i] * ch);
  }
  temb_ = dalloc((size_t)lsd_ * FD);
  rope_ = dalloc((size_t)max_ctx_ * 64);
  temb_tmp_ = dalloc((size_t)2 * lsd_ * FD);

  for (int q = 0; q < NHB; ++q) {
    PTTS_HIP(hipHostMalloc((void**)&h_pcm_[q], sizeof(float) * B * FRAME, hipHostMallocDefault));
    if (nfr_ > 1 && q < nhb_)  // inside the pass's pinned block (above)
      h_meta_[q] = h_pcmp_[q / nfr_] + (size_t)B * nfr_ * FRAME + (q % nfr_) * ((meta_floats_ + 31) / 32 * 32);
    else
      PTTS_HIP(hipHostMalloc((void**)&h_meta_[q], sizeof(float) * meta_floats_, hipHostMallocDefault));
    memset(h_meta_[q], 0, sizeof(float) * meta_floats_);
  }
  PTTS_HIP(hipHostMalloc((void**)&h_err_, sizeof(int), hipHostMallocDefault));
  *h_err_ = 0;
  PTTS_HIP(hipHostMalloc((void**)&h_slots_, sizeof(int) * B, hipHostMallocDefault));
  PTTS_HIP(hipHostMalloc((void**)&h_st_, sizeof(SlotState) * B, hipHostMallocDefault));
  PTTS_HIP(hipHostMalloc((void**)&h_fp_, sizeof(int) * B, hipHostMallocDefault));
  PTTS_HIP(hipHostMalloc((void**)&h_ids_, sizeof(int) * PREFILL, hipHostMallocDefault));
  PTTS_HIP(hipHostMalloc((void**)&h_tab_, sizeof(int) * 4 * PREFILL, hipHostMallocDefault));  // ptab | ctab | qrow | orow
  PTTS_HIP(hipHostMalloc((void**)&h_vpre_, sizeof(float*) * (B + 1), hipHostMallocDefault));
  PTTS_HIP(hipHostMalloc((void**)&h_vlen_, sizeof(int) * (B + 1), hipHostMallocDefault));
  memset(h_vpre_, 0, sizeof(float*) * (B + 1));
  memset(h_vlen_, 0, sizeof(int) * (B + 1));
  PTTS_HIP(hipStreamCreateWithFlags(&stream_be_, hipStreamNonBlocking));
  for (int q = 0; q < NHB; ++q) {
    PTTS_HIP(hipEventCreateWithFlags(&ev_front_[q], hipEventDisableTiming));
    PTTS_HIP(hipEventCreateWithFlags(&ev_back_[q], hipEventDisableTiming));
    PTTS_HIP(hipEventRecord(ev_front_[q], stream_));
    PTTS_HIP(hipEventRecord(ev_back_[q], stream_));
  }
  PTTS_HIP(hipEventCreateWithFlags(&ev_admit_, hipEventDisableTiming));
  PTTS_HIP(hipEventCreateWithFlags(&ev_be_tail_, hipEventDisableTiming));
  PTTS_HIP(hipEventCreateWithFlags(&ev_act_, hipEventDisableTiming));
  for (hipEvent_t& e : ev_call_) PTTS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  PTTS_HIP(hipEventRecord(ev_act_, stream_));
  PTTS_HIP(hipEventRecord(ev_admit_, stream_));
  pipeline_ = cfg.pipeline != 0;
  head_resident_ = flow_head_max_resident(dev_);

  if (!cfg.defer_weights) {
    std::unique_ptr<TensorSource> src = cfg.weights_path && cfg.weights_path[0]
                                            ? make_safetensors_source(cfg.weights_path)
                                            : make_synth_source(cfg.synth_seed);
    src = make_quant_source(std::move(src), wq_);
    upload_weights(src.get());
    finalize();
  }
}

Engine::~Engine() {
  (void)hipSetDevice(dev_);
  if (stream_) (void)hipStreamSynchronize(stream_);
  if (stream_be_) (void)hipStreamSynchronize(stream_be_);
  if (stream_pv_) (void)hipStreamSynchronize(stream_pv_);
#ifdef PTTS_PROBES
  if (stamp_ring_) {  // tag (part << 8 | buffer << 1 | end), then the 100-MHz realtime count
    unsigned n = 0;
    std::vector<unsigned long long> r((size_t)STAMP_CAP * 2);
    if (hipMemcpy(&n, stamp_ctr_, 4, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(r.data(), stamp_ring_, r.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
      if (FILE* f = fopen(probe_env("PTTS_STAMPS"), "w")) {
        for (int p = 0; p < 2; ++p)
          for (size_t i = 0; i < stamp_names_[p].size(); ++i) fprintf(f, "# %d %zu %s\n", p, i, stamp_names_[p][i].c_str());
        for (unsigned i = 0; i < std::min(n, STAMP_CAP); ++i) fprintf(f, "%llu %llu\n", r[2 * i], r[2 * i + 1]);
        fclose(f);
      }
  }
#endif
  for (int s = 0; s < (int)slot_voice_.size(); ++s) voice_release(s, true);
  for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : graph_defs_) (void)hipGraphDestroy(kv.second);
  for (auto& kv : pv_graphs_) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : pv_graph_defs_) (void)hipGraphDestroy(kv.second);
  for (PvEntry& q : pv_q_) {
    if (q.ev) (void)hipEventDestroy(q.ev);
    if (q.h_pcm) (void)hipHostFree(q.h_pcm);
  }
  for (int q = 0; q < NHB; ++q)
    if (ev_pv_read_[q]) (void)hipEventDestroy(ev_pv_read_[q]);
  if (ev_pv_front_) (void)hipEventDestroy(ev_pv_front_);
  if (stream_pv_) (void)hipStreamDestroy(stream_pv_);
  for (int q = 0; q < NHB; ++q) {
    if (ev_front_[q]) (void)hipEventDestroy(ev_front_[q]);
    if (ev_back_[q]) (void)hipEventDestroy(ev_back_[q]);
  }
  if (ev_admit_) (void)hipEventDestroy(ev_admit_);
  if (ev_be_tail_) (void)hipEventDestroy(ev_be_tail_);
  if (ev_act_) (void)hipEventDestroy(ev_act_);
  for (hipEvent_t e : ev_call_)
    if (e) (void)hipEventDestroy(e);
  if (stream_be_) (void)hipStreamDestroy(stream_be_);
  for (void* p : allocs_) (void)hipFree(p);
  for (int q = 0; q < NHB; ++q) {
    if (h_pcm_[q]) (void)hipHostFree(h_pcm_[q]);
    if (h_meta_[q] && !(nfr_ > 1 && q < nhb_)) (void)hipHostFree(h_meta_[q]);
  }
  for (int p = 0; p < NHB / 2; ++p)
    if (h_pcmp_[p]) (void)hipHostFree(h_pcmp_[p]);
  if (h_act_) (void)hipHostFree(h_act_);
  if (h_err_) (void)hipHostFree(h_err_);
  for (void* hp : {(void*)h_slots_, (void*)h_st_, (void*)h_fp_, (void*)h_ids_, (void*)h_tab_, (void*)h_vpre_,
                   (void*)h_vlen_})
    if (hp) (void)hipHostFree(hp);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void Engine::upload_weights(TensorSource* src) {
  std::vector<float> host(L_.total, 0.f);
  pack_weights(src, host.data());
  PTTS_HIP(hipMemcpy(blob_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
}

void Engine::load_blob(const float* host, size_t n_bytes) {
  PTTS_REQUIRE(n_bytes == L_.total * sizeof(float), "blob size differs from ptts_weight_blob_bytes()");
  PTTS_REQUIRE(!ready_, "engine already finalized");
  PTTS_HIP(hipSetDevice(dev_));
  PTTS_HIP(hipMemcpy(blob_, host, n_bytes, hipMemcpyHostToDevice));
}

// The FlowLM step matrices as fragment-packed copies for the register-resident split-K GEMM
// (bit mask of the matrices that use it: 1 qkv, 2 out, 4 linear1, 8 linear2, 16 the flow head's
// adaLN matrix, M = lsd * B rows): out on 32x32 tiles with 8 K slices of 128 (4 waves splitting
// each), linear2 on 32x32 tiles with 16 slices of 256. Alone on the chip every matrix is faster
// this way (qkv 8.1 -> 4.9 us, out 4.5 -> 3.2, linear1 8.1 -> 5.2, linear2 7.9 -> 5.3); in the
// pipelined step only out + linear2 + adaLN pay (steady step 0.6595 -> 0.6326 ms, medians of 3):
// the qkv / linear1 versions on any tile slow the concurrent back part more than they gain.
// The int8 codes of quantized weight W [N][K] (derive_int8) in pack_q8 order: the codes widened
// to f32 (temporary), fragment-packed by `pack` exactly as the f32 weight would be, then one byte
// per element with a lane's four fragment groups per 16-B load (nj: groups per lane and wave).
// fp8_gemm engines: the e4m3 codes of fp8_codes (f8map_) the same way.
const uint32_t* Engine::pack_codes(const float* W, int N, int K, int nj,
                                   const std::function<void(const float*, float*)>& pack) {
  auto it = q8map_.find(W);
  auto it8 = f8map_.find(W);
  if (it == q8map_.end() && it8 == f8map_.end()) return nullptr;
  const size_t n = (size_t)N * K;
  float* tmp = nullptr;
  PTTS_HIP(hipMalloc(&tmp, sizeof(float) * 2 * n));
  void* q = nullptr;
  PTTS_HIP(hipMalloc(&q, n));
  allocs_.push_back(q);
  if (it != q8map_.end()) codes_to_f32(it->second.first, (long)n, tmp, stream_);
  else codes_u8_to_f32(it8->second.first, (long)n, tmp, stream_);
  pack(tmp, tmp + n);
  pack_q8(tmp + n, (long)(n / 4), nj, (uint32_t*)q, stream_);
  PTTS_HIP(hipStreamSynchronize(stream_));
  PTTS_HIP(hipFree(tmp));
  return (const uint32_t*)q;
}

void Engine::derive_gemv() {
  // sequential stepping (the B = 1 first-chunk path, no concurrent back part) and frame-pair
  // pipelined stepping (the front part bounds the step): every matrix. Single-frame pipelined
  // stepping (the back part bounds it): qkv and linear1 stay on the LDS-DMA tile, whose smaller
  // register footprint crowds the concurrent back part less (same-box product bench, DESIGN.md §1:
  // pairs 4,093 -> 4,395x with every matrix register-resident, single frames 4,228 -> 4,170x)
  int mask = pipeline_ && nfr_ == 1 ? 2 | 8 | 16 : 31;
  if (probe_env("PTTS_GEMV_MASK")) mask = atoi(probe_env("PTTS_GEMV_MASK"));  // probe builds: A/B runs
  gemv_mask_ = mask;
  struct M {
    const float* w;
    int N, K, bit;
    GemvShape g;
  };
  std::vector<M> mats;
  const GemvShape wide{4, 128};  // qkv / linear1 tile
  const GemvShape outg{1, 32};   // out tile
  for (int l = 0; l < NL; ++l) {
    const Layout::TL& t = L_.fl[l];
    mats.push_back({W(t.in_proj), 3 * D, D, 1, wide});
    mats.push_back({W(t.out_proj), D, D, 2, outg});
    mats.push_back({W(t.l1), FF, D, 4, wide});
    mats.push_back({W(t.l2), D, FF, 8, GemvShape{1, 64}});
  }
  const GemvShape ada{4, 128};  // flow-head adaLN matrix: 0.6365 -> 0.6315 ms
  mats.push_back({W(L_.ada_w), NADA, FD, 16, ada});
  // Code-carrying matrices (weight_quant: int8, fp8_gemm: e4m3) are read from their codes only
  // (k_gemv / k_ffn_fused with WQ != 0 never touch an f32 packed copy), so they get no f32 copy.
  auto scale_of = [&](const float* w) { return fp8_ ? f8map_.at(w).second : q8map_.at(w).second; };
  // linear1 on the whole-K GEMM (gemv_fk: GELU in its epilogue, no split-K slabs, no reduce launch)
  // wherever the register-resident linear1 is used; PTTS_NO_FK (probe builds) keeps the split-K form
  if ((mask & 4) && !probe_env("PTTS_NO_FK") && gemv_fk_supported(1, FF, D)) {
    // linear1 + linear2 as ONE launch (ffn_fused) wherever the whole-K linear1 is used;
    // PTTS_NO_FFN (probe builds) keeps the two launches
    const bool ffn = !probe_env("PTTS_NO_FFN") && ffn_fused_supported(1, D, FF);
    if (ffn) ffn_groups_ = probe_env("PTTS_FFN16") ? 16 : 8;  // probe builds: the 16-group form, for A/B runs
    const int G = ffn_groups_;
    // weight_quant / fp8 engines: both matrices as codes (the fused launch then streams a quarter
    // of the bytes)
    std::vector<std::pair<const uint32_t*, const uint32_t*>> codes(NL, {nullptr, nullptr});
    bool all_codes = ffn;
    for (int l = 0; l < NL && ffn; ++l) {
      const float *w1 = W(L_.fl[l].l1), *w2 = W(L_.fl[l].l2);
      codes[l].first = pack_codes(w1, FF, D, 8, [&](const float* c, float* o) { pack_gemv_fk(c, FF, D, o, stream_); });
      codes[l].second = pack_codes(w2, D, FF, 8, [&](const float* c, float* o) { pack_ffn2(c, G, o, stream_); });
      if (codes[l].first && codes[l].second) ffn8map_[w2] = {{codes[l].first, scale_of(w1)}, {codes[l].second, scale_of(w2)}};
      else all_codes = false;
    }
    const bool f32_copies = !all_codes;
    void* q = nullptr;
    PTTS_HIP(hipMalloc(&q, sizeof(float) * ((f32_copies ? (size_t)NL * FF * D : 0) + FK_A_FLOATS)));  // all written before read
    allocs_.push_back(q);
    float* dst = (float*)q;
    for (int l = 0; l < NL; ++l) {
      if (f32_copies) pack_gemv_fk(W(L_.fl[l].l1), FF, D, dst, stream_);
      fkmap_[W(L_.fl[l].l1)] = f32_copies ? dst : nullptr;  // nullptr: the fused launch reads the codes
      if (f32_copies) dst += (size_t)FF * D;
    }
    hfrag_ = dst;
    if (ffn) {
      void* f = nullptr;
      PTTS_HIP(hipMalloc(&f, sizeof(float) * ((f32_copies ? (size_t)NL * D * FF : 0) + 2 * FFN_HAND_FLOATS)));
      allocs_.push_back(f);
      float* fd = (float*)f;
      for (int l = 0; l < NL; ++l) {
        if (f32_copies) pack_ffn2(W(L_.fl[l].l2), G, fd, stream_);
        ffnmap_[W(L_.fl[l].l2)] = f32_copies ? fd : nullptr;
        if (f32_copies) fd += (size_t)D * FF;
      }
      ffn_hand_ = fd;  // both sets empty (0xFFFFFFFF) before the first launch
      PTTS_HIP(hipMemsetD32Async(ffn_hand_, 0xFFFFFFFFu, 2 * FFN_HAND_FLOATS, stream_));
    }
  }
  std::vector<Gemv> sel;  // (matrix, codes) of every register-resident matrix
  std::vector<const M*> selm;
  size_t total = 0;
  for (const M& m : mats) {
    if (!(mask & m.bit) || !gemv_supported(m.g, m.N, m.K)) continue;
    Gemv gv{nullptr, m.g, m.bit, nullptr, nullptr};
    // weight_quant engines: the int8 codes of a quantized matrix in the same fragment order;
    // fp8_gemm engines: the e4m3 codes of the {4, 128} matrices (qkv, adaLN; W8A8 tiles). An e4m3
    // matrix on another tile (linear2's {1, 64}) gets no register-resident form at all: it stays on
    // k_gemm_fp8 (W8A8), so every fp8 matrix runs fp8 in every stepping mode
    const GemvShape g = m.g;
    const int N = m.N, K = m.K;
    if (!fp8_ || (g.wn == 4 && g.kw == 128)) {
      gv.q8 = pack_codes(m.w, N, K, g.kw / 8, [&](const float* c, float* o) { pack_gemv(c, N, K, g, o, stream_); });
      if (gv.q8) gv.scale = scale_of(m.w);
    } else if (f8map_.count(m.w)) {
      continue;
    }
    if (!gv.q8) total += (size_t)N * K;
    sel.push_back(gv);
    selm.push_back(&m);
  }
  float* dst = nullptr;
  if (total) {
    void* p = nullptr;
    PTTS_HIP(hipMalloc(&p, sizeof(float) * total));  // every element is written by the packing
    allocs_.push_back(p);
    dst = (float*)p;
  }
  for (size_t i = 0; i < sel.size(); ++i) {
    const M& m = *selm[i];
    Gemv gv = sel[i];
    if (!gv.q8) {
      pack_gemv(m.w, m.N, m.K, m.g, dst, stream_);
      gv.packed = dst;
      dst += (size_t)m.N * m.K;
    }
    gvmap_[m.w] = gv;
  }
  PTTS_HIP(hipGetLastError());
  PTTS_HIP(hipStreamSynchronize(stream_));
}

// bf16x6 back part (back_mfma = PTTS_BACK_F32X6): every back-part GEMM / conv weight matrix split
// into its exact three bf16 pieces (split3: hi | mid in W's f32 layout, lo as bf16), padded with
// zero rows to a multiple of 32 (the tiles read rows < Nw). Shapes as build_back multiplies them.
void Engine::derive_split() {
  auto add = [&](size_t off, int N, int K) {
    const int Nw = (N + 31) / 32 * 32;
    void *hm = nullptr, *lo = nullptr;
    PTTS_HIP(hipMalloc(&hm, sizeof(unsigned) * (size_t)Nw * K));
    allocs_.push_back(hm);
    PTTS_HIP(hipMalloc(&lo, sizeof(unsigned short) * (size_t)Nw * K));
    allocs_.push_back(lo);
    if (Nw > N) {
      PTTS_HIP(hipMemsetAsync((unsigned*)hm + (size_t)N * K, 0, sizeof(unsigned) * (size_t)(Nw - N) * K, stream_));
      PTTS_HIP(hipMemsetAsync((unsigned short*)lo + (size_t)N * K, 0, sizeof(unsigned short) * (size_t)(Nw - N) * K,
                              stream_));
    }
    split3(W(off), (long)N * K, (unsigned*)hm, (unsigned short*)lo, stream_);
    split_[W(off)] = {(const unsigned*)hm, (const unsigned short*)lo};
  };
  for (int l = 0; l < MNL; ++l) {
    const Layout::TL& t = L_.mdec[l];
    add(t.in_proj, 3 * MD, MD);
    add(t.out_proj, MD, MD);
    add(t.l1, MFF, MD);
    add(t.l2, MD, MFF);
  }
  add(L_.dc0_w, 512, 7 * 512);
  for (int i = 0, ch = 512; i < 3; ++i, ch /= 2) {
    add(L_.dtr_w[i], RATIOS[i] * (ch / 2), 2 * ch);
    add(L_.dra_w[i], ch / 4, 3 * (ch / 2));
    add(L_.drb_w[i], ch / 2, ch / 4);
  }
  PTTS_HIP(hipGetLastError());
  PTTS_HIP(hipStreamSynchronize(stream_));
}

// A bf16x6 tile (layout >= 200) reads the split copy of its weight matrix (derive_split)
void Engine::attach_split(GemmArgs& a) const {
  if (a.layout < 200) return;
  auto it = split_.find(a.W);
  PTTS_REQUIRE(it != split_.end(), "bf16x6 tile without a split weight copy");
  a.Whm = it->second.first;
  a.Wlo = it->second.second;
}

void Engine::finalize() {
  PTTS_HIP(hipSetDevice(dev_));
  if (wq_ != QUANT_NONE && q8map_.empty()) derive_int8();
  if (fp8_ && f8map_.empty()) derive_fp8();
  if (gvmap_.empty()) derive_gemv();
  if (back_mfma_ == PTTS_BACK_F32X6 && split_.empty()) derive_split();
  if (!inw_t_) {  // every element is written by the transpose below: no (null-stream) memset
    void* p = nullptr;
    PTTS_HIP(hipMalloc(&p, sizeof(float) * LDIM * D));
    allocs_.push_back(p);
    inw_t_ = (float*)p;
  }
  transpose(W(L_.input_linear), D, LDIM, inw_t_, stream_);
  if (!fh_inw_t_) {  // flow-head input projection transposed ([32][512], the x0 side job)
    void* p = nullptr;
    PTTS_HIP(hipMalloc(&p, sizeof(float) * LDIM * FD));
    allocs_.push_back(p);
    fh_inw_t_ = (float*)p;
  }
  transpose(W(L_.inproj_w), FD, LDIM, fh_inw_t_, stream_);
  if (!fhw_ && head_uniform_stride()) {  // every element is written by the packing below
    void* p = nullptr;
    PTTS_HIP(hipMalloc(&p, sizeof(float) * flow_head_packed_floats()));
    allocs_.push_back(p);
    fhw_ = (float*)p;
  }
  if (fhw_) pack_flow_head(W(L_.rb_w0[0]), W(L_.rb_w2[0]), (long)(L_.rb_w0[1] - L_.rb_w0[0]), W(L_.fin_w), fhw_, stream_);
  TimeEmbedWeights tw;
  for (int i = 0; i < 2; ++i) {
    tw.l1w[i] = W(L_.te_l1w[i]);
    tw.l1b[i] = W(L_.te_l1b[i]);
    tw.l2w[i] = W(L_.te_l2w[i]);
    tw.l2b[i] = W(L_.te_l2b[i]);
    tw.alpha[i] = W(L_.te_alpha[i]);
  }
  time_embeddings(tw, lsd_, temb_tmp_, temb_, stream_);
  rope_table(rope_, max_ctx_, stream_);
  for (int i = 0, ch = MD / 2; i < 3; ++i, ch /= 2)  // bias of the phase-merged transposed convs
    for (int p = 0; p < RATIOS[i]; ++p)
      PTTS_HIP(hipMemcpyAsync(trb_[i] + (size_t)p * ch, W(L_.dtr_b[i]), sizeof(float) * ch, hipMemcpyDeviceToDevice,
                              stream_));
  PTTS_HIP(hipGetLastError());
  PTTS_HIP(hipStreamSynchronize(stream_));
  ready_ = true;
}

void Engine::run_ops(const std::vector<Op>& ops) {
  xh_dirty_ = true;  // eager passes (prefills, encoder) use x_ / h_ as scratch
  for (const Op& op : ops) {
    op.fn(stream_);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw Error(PTTS_ERR_HIP, "launch of " + op.name + " failed: " + hipGetErrorString(e));
  }
}

// int8 code matrices of the quantized FlowLM GEMM weights, derived on the device from the
// blob (so a blob received over RCCL needs nothing else): every Layout::Q8 matrix whose rows
// all carry a scale gets codes; quant_codes checks float(q) * s == W bit for bit.
void Engine::derive_int8() {
  float mode = 0.f;
  PTTS_HIP(hipMemcpy(&mode, blob_ + L_.qmode, sizeof(float), hipMemcpyDeviceToHost));
  PTTS_REQUIRE((int)mode == wq_, "weight blob was packed with a different weight_quant mode");
  std::vector<const Layout::Q8*> use;
  size_t bytes = 0;
  for (const Layout::Q8& q : L_.q8) {
    std::vector<float> s((size_t)q.N);
    PTTS_HIP(hipMemcpy(s.data(), blob_ + q.s, s.size() * sizeof(float), hipMemcpyDeviceToHost));
    if (std::all_of(s.begin(), s.end(), [](float v) { return v > 0.f; })) {
      use.push_back(&q);
      bytes += ((size_t)q.N * q.K + 255) / 256 * 256;
    }
  }
  if (use.empty()) return;
  void* codes = nullptr;
  PTTS_HIP(hipMalloc(&codes, bytes));
  allocs_.push_back(codes);
  int* bad = (int*)dalloc(1);
  size_t off = 0;
  for (const Layout::Q8* q : use) {
    int8_t* c = (int8_t*)codes + off;
    quant_codes(W(q->w), W(q->s), q->N, q->K, c, bad, stream_);
    q8map_[W(q->w)] = {c, W(q->s)};
    off += ((size_t)q->N * q->K + 255) / 256 * 256;
  }
  PTTS_HIP(hipGetLastError());
  int nbad = 0;
  PTTS_HIP(hipMemcpyAsync(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost, stream_));
  PTTS_HIP(hipStreamSynchronize(stream_));
  if (nbad) {
    q8map_.clear();
    throw Error(PTTS_ERR_INVALID, "quantized weights are not on their int8 grid (" + std::to_string(nbad) +
                                      " elements): blob not packed by the quantizer");
  }
}

// e4m3 codes + row scales of the large FlowLM step GEMM weights (the int8 path's set: qkv,
// linear1, linear2, adaLN; >= 2M weights), derived on the device from the f32 blob.
void Engine::derive_fp8() {
  std::vector<const Layout::Q8*> use;
  size_t bytes = 0, nsc = 0;
  for (const Layout::Q8& q : L_.q8)
    if ((long)q.N * q.K >= (2L << 20)) {
      use.push_back(&q);
      bytes += ((size_t)q.N * q.K + 255) / 256 * 256;
      nsc += (size_t)q.N;
    }
  void* codes = nullptr;
  PTTS_HIP(hipMalloc(&codes, std::max<size_t>(bytes, 1)));
  allocs_.push_back(codes);
  float* scales = dalloc(nsc);
  size_t off = 0, so = 0;
  for (const Layout::Q8* q : use) {
    uint8_t* c = (uint8_t*)codes + off;
    fp8_codes(W(q->w), q->N, q->K, c, scales + so, stream_);
    f8map_[W(q->w)] = {c, scales + so};
    off += ((size_t)q->N * q->K + 255) / 256 * 256;
    so += (size_t)q->N;
  }
  PTTS_HIP(hipGetLastError());
  PTTS_HIP(hipStreamSynchronize(stream_));
}

// ------------------------------------------------------------------ op builders
void Engine::linear_split(std::vector<Op>& ops, const std::string& name, const float* X, long ldx, int M,
                          const float* Wt, int N, int K, int* S_out) {
  PTTS_REQUIRE(K % 32 == 0, "GEMM K must be a multiple of 32");
  int S = pick_splits(M, N, K);
  int layout = 0, tail = 0;
  // wide skinny GEMMs (FlowLM qkv/ff1, flow-head adaLN): 32x128 LDS-DMA tiles, 8-way split-K
  // (tools/gemm_bench.hip on MI355X: qkv 6.7 -> 6.3 us, ff1 7.9 -> 6.5 us, ada 10.1 -> 8.7 us)
  if (M <= 64 && N >= 3072) {
    layout = 7;  // 2-buffer LDS (40 KB) co-resides with the back part
    S = std::max(1, std::min(8, K / 64));
  } else if (M >= 256) {  // prefill passes (text admission, M = 48 rows per slot): MFMA-bound,
    // LDS-DMA tiles with the DMAs interleaved between the MFMAs and a split tail (the tiles past
    // whole rounds of the CUs' workgroup slots run as K slices; tools/mm_bench.hip at M = 1536,
    // against rocBLAS fp32 on the same box: qkv 108 / 111, out 88 / 98, ff1 112 / 125, ff2 117 /
    // 122 TF/s): 128x64, two per CU, 4 slices; linear1 128x64 one per CU, 2 slices
    layout = N >= 4096 && K <= 1024 ? 34 : 35;
    tail = N >= 4096 && K <= 1024 ? 2 : 4;
    S = 1;
  } else if (M <= 64 && K >= 4096) {  // FlowLM ff2: 8 slabs (tools/gemm_bench.hip flow.ff2: 8.5 -> 7.3 us)
    S = 8;
  } else if (M <= 64 && N <= 512 && K == 512) {  // flow-head MLPs: 8 waves, 8 slabs (head.mlp: 3.9 -> 3.4 us)
    layout = 9;
    S = 8;
  }
  // quantized FlowLM weights on the step path: stream int8 codes (k_gemm_w8, 32x64 tiles, the
  // smallest power-of-two split reaching 256 workgroups with >= 4 K chunks per slice). Only the
  // large matrices (qkv, ff1, ff2, adaLN; >= 2M weights): below that the launch is latency-bound
  // and the f32 copy of the same values is as fast (tools/w8_probe.py). Prefill passes
  // (M >= 256) keep the f32 copy too: they are MFMA-bound.
  auto gv = gvmap_.find(Wt);
  if (gv != gvmap_.end() && M <= 64 && (gemv_mask_ & gv->second.bit)) {  // register-resident weights (derive_gemv)
    const GemvShape g = gv->second.g;
    const float* P = gv->second.packed;
    const uint32_t* q8 = gv->second.q8;
    const float* sc = gv->second.scale;
    const int Sg = K / g.ks();
    PTTS_REQUIRE((size_t)Sg * M * N <= pcap_, "split-K partial buffer too small");
    float* part = partial_;
    const bool f8 = fp8_ && q8;
    ops.push_back({name, [=](hipStream_t s) { gemv_splitk(X, ldx, M, N, K, P, g, part, s, q8, sc, f8); }, 2.0 * M * N * K,
                   (q8 ? 1.0 * N * K + 4.0 * N : 4.0 * N * K) + 4.0 * ((double)M * K + (double)Sg * M * N)});
    *S_out = Sg;
    return;
  }
  auto f8 = f8map_.find(Wt);
  const bool wf8 = f8 != f8map_.end() && M <= 64;
  if (wf8) {  // fp8 W8A8 (k_gemm_fp8): 32x64 tiles, >= 256 workgroups, K slice <= FP8_KSLICE_MAX
    layout = 0;
    const int tiles = ((N + 63) / 64) * ((M + 31) / 32), nch = K / 32;
    S = 1;
    while (S < 16 && tiles * S < 256 && nch / (2 * S) >= 4) S *= 2;
    while ((nch + S - 1) / S > FP8_KSLICE_MAX / 32) ++S;
  }
  auto q8 = q8map_.find(Wt);
  const bool w8 = q8 != q8map_.end() && M <= 64 && (long)N * K >= (2L << 20);
  if (w8) {
    layout = 0;
    const int tiles = ((N + 63) / 64) * ((M + 31) / 32);
    S = 1;
    while (S < 16 && tiles * S < 256 && (K / 32) / (2 * S) >= 4) S *= 2;
  }
  if (!w8 && !wf8) tile_override(name, layout, S);
  while (S > 1 && (size_t)S * M * N > pcap_) --S;
  PTTS_REQUIRE((size_t)S * M * N <= pcap_, "split-K partial buffer too small");
  GemmArgs a{};
  if (w8) {
    a.Wq = q8->second.first;
    a.wscale = q8->second.second;
  }
  if (wf8) {
    PTTS_REQUIRE((K / 32 + S - 1) / S <= FP8_KSLICE_MAX / 32, "fp8 GEMM K slice too long");
    a.Wf8 = f8->second.first;
    a.wscale = f8->second.second;
  }
  a.mode = 0;
  a.layout = layout;
  a.M = M;
  a.N = N;
  a.K = K;
  a.Nw = (N + 31) / 32 * 32;
  a.X = X;
  a.ldx = ldx;
  a.W = Wt;
  a.S = S;
  a.partial = partial_;
  if (tail > 0 && S == 1 && !w8 && !wf8) {
    a.tail_S = tail;
    a.tail_slab = tslab_;
    a.tail_cap = (long)TAIL_CAP;
    a.tickets = tickets_;
    a.tickets_cap = TICKETS;
  }
  // FlowLM / flow-head step weights are read once per step: non-temporal loads on the LDS-DMA
  // tiles (step -1.1 %; the 32x32 register tile keeps default-policy loads)
  a.w_nt = M <= 64 && layout != 0;
  a.front = 1;  // FlowLM / flow-head GEMMs (and the prefill passes, on the same stream)
  ops.push_back({name, [a, S](hipStream_t s) { gemm(a, S, s); }, 2.0 * M * N * K,
                 (w8 || wf8 ? (double)N * K + 4.0 * N : 4.0 * N * K) + 4.0 * ((double)M * K + (double)S * M * N)});
  *S_out = S;
}

// Algorithmic cost of a row-reduce launch (HBM-bound): the S slabs, the operands it reads per row
// (bias, gate, residual, LayerNorm affine, modulation) and every row it stores, plus the side jobs.
static Op rr_op(const std::string& name, const RowReduceArgs& a) {
  const double mn = (double)a.M * a.N;
  double f = mn * (a.S + 1 + (a.act ? 8 : 0) + (a.ln ? 8 : 0));
  double b = mn * a.S + (a.bias ? a.N : 0) + (a.gate ? (a.ldg ? mn : a.N) : 0) + (a.R ? mn : 0) + (a.Y ? mn : 0) +
             (a.Y2 ? mn : 0) + (a.euler ? 2.0 * a.M * 32 : 0);
  if (a.ln) b += mn + (a.ln_w ? 2.0 * a.N : 0) + (a.mshift ? 2.0 * mn : 0);
  if (a.fhm) b += mn * 2.0 / 3.0;  // the fragment-order copy of the shift / scale columns
  if (a.fill) b += 4.0 * a.fill_n4;
  if (a.x0_hx) {  // x0 = cur W_in^T + b_in for x0_B rows
    b += (double)a.x0_B * (32 + 512) + 32.0 * 512;
    f += 2.0 * a.x0_B * 32 * 512;
  }
  return Op{name, [a](hipStream_t s) { row_reduce(a, s); }, f, 4.0 * b};
}

// The row-reduce epilogue of the split GEMM just emitted, as its own launch (an in-launch split-K
// combine by the last-arriving workgroup measured slower on every front GEMM: ff2 43 vs 13 us with
// the LayerNorm row finisher, ff1 15.6 vs 11.4 us tile-local).
void Engine::push_rr(std::vector<Op>& ops, const std::string& name, const RowReduceArgs& r) {
  RowReduceArgs a = r;
  a.front = 1;  // the FlowLM / flow-head reduces (the back part's go through rr_op directly)
  ops.push_back(rr_op(name, a));
}

void Engine::dense_op(std::vector<Op>& ops, const std::string& name, const float* X, int M, const float* Wt, int N,
                      int K, const float* bias, int act, const float* rscale, const float* R, float* Y, int layout) {
  PTTS_REQUIRE(K % 32 == 0, "GEMM K must be a multiple of 32");
  int ks = 1;
  tile_override(name, layout, ks);
  PTTS_REQUIRE(!(layout == 8 || layout == 15 || layout == 16) || K % 64 == 0, "BK 64 tiles need K % 64 == 0");
  GemmArgs a{};
  a.mode = 0;
  a.layout = layout;
  a.M = M;
  a.N = N;
  a.K = K;
  a.Nw = (N + 31) / 32 * 32;
  a.X = X;
  a.ldx = K;
  a.W = Wt;
  a.S = 1;
  a.bias = bias;
  a.act = act;
  a.rscale = rscale;
  a.R = R;
  a.ldr = N;
  a.Y = Y;
  a.ldy = N;
  attach_split(a);
  ops.push_back({name, [a](hipStream_t s) { gemm(a, 1, s); }, 2.0 * M * N * K,
                 4.0 * ((double)N * K + (double)M * K + (double)M * N * (R ? 2 : 1))});
}

void Engine::conv_op(std::vector<Op>& ops, const std::string& name, const float* X, int B, int T_in, int cin,
                     const float* H, int P, int stride, int elu, const float* Wt, int cout, int ktaps, int phases,
                     const float* bias, const float* R, float* Y, int T_out, int tstride, int layout, int elu_out,
                     float* Y2, int ksplit) {
  PTTS_REQUIRE(cin % 32 == 0, "conv cin must be a multiple of 32");
  tile_override(name, layout, ksplit);
  PTTS_REQUIRE(!(layout == 8 || layout == 15 || layout == 16) || cin % 64 == 0, "BK 64 tiles need cin % 64 == 0");
  // ksplit > 1: single-phase conv on an LDS-DMA tile, K split into ksplit partial slabs in the
  // back part's slab buffer; the caller adds the row-reduce epilogue
  PTTS_REQUIRE(ksplit == 1 || (phases == 1 && lds_dma_layout(layout)), "K-split convs need a single-phase LDS-DMA tile");
  GemmArgs a{};
  a.mode = 1;
  a.layout = layout;
  a.Tq = T_in / stride;
  a.M = B * a.Tq;
  a.N = cout;
  a.K = ktaps * cin;
  a.Nw = (cout + 31) / 32 * 32;
  a.X = X;
  a.ldx = cin;
  a.H = H;
  a.P = P;
  a.T_in = T_in;
  a.stride_in = stride;
  a.cin = cin;
  a.elu_in = elu;
  a.W = Wt;
  a.w_phase_stride = (long)cout * ktaps * cin;
  a.S = 1;
  a.bias = bias;
  a.R = R;
  a.ldr = cout;
  a.Y = Y;
  a.ldy = cout;
  a.T_out = T_out;
  a.out_tstride = tstride;
  a.elu_out = elu_out;
  a.Y2 = Y2;
  const int nph = phases;
  attach_split(a);
  if (ksplit > 1) {
    PTTS_REQUIRE((size_t)ksplit * a.M * a.N <= mpcap_, "back split-K slab buffer too small");
    a.S = ksplit;
    a.partial = mpartial_;
    phases = ksplit;  // grid z
  }
  ops.push_back({name, [a, phases](hipStream_t s) { gemm(a, phases, s); }, 2.0 * a.M * a.N * a.K * nph,
                 4.0 * ((double)nph * a.N * a.K + (double)B * T_in * cin +
                        (double)B * T_out * cout * ((R ? 2 : 1) + (Y2 ? 1 : 0)))});
}

// FlowLM transformer layers over M rows (x_ holds the residual stream, h_ = norm1_0(x_)).
// StreamingTransformerLayer::forward (transformer.rs:66-90).
void Engine::flow_layers(std::vector<Op>& ops, int M, RowMap map, int qg, bool out_norm, const std::string& tag) {
  for (int l = 0; l < NL; ++l) {
    const Layout::TL& t = L_.fl[l];
    const std::string p = tag + ".l" + std::to_string(l);
    KvStore kv{kv_ + (long)l * kv_layer_, kv_slot_, max_ctx_};
    if (share_voice_) {  // positions below a slot's voice length read the voice's own cache
      kv.pre = vpre_;
      kv.pre_len = vlen_;
      kv.layer = l;
    }
    int S = 1;
    linear_split(ops, p + ".qkv_gemm", h_, D, M, W(t.in_proj), 3 * D, D, &S);
    if (qg == 1) {  // step: slab sum + RoPE + KV append fused into the attention kernel
      const float* P = partial_;
      float* O = o_;
      const float* rope = rope_;
      // K and V of every head over the cached positions the launch reads (8,192 B per position):
      // each row's own positions, plus ONE copy of every distinct shared voice prefix (the rows of
      // a voice read its cache, KvStore::pre: plan_kvu_), the QKV slabs, the appended K/V and the
      // output row; QK^T + PV = 4,096 flops per position and row
      const double L = plan_ctx_ > 0 ? plan_ctx_ : max_ctx_ / 2.0;
      const double kvu = plan_kvu_ > 0 ? plan_kvu_ : M * L;
      ops.push_back({p + ".attention", [=](hipStream_t s) { attention_step_qkv(P, S, M, NH, map, kv, rope, O, s); },
                     (double)M * 4096.0 * L,
                     8192.0 * kvu + (double)M * (4.0 * (S * 3.0 * D + 2.0 * D + D) + 64.0 * 4 * 2)});
    } else {
      {
        const float* P = partial_;
        float* Q = q_;
        ops.push_back({p + ".qkv_rope", [=](hipStream_t s) { qkv_rope_append(P, S, nullptr, M, NH, map, kv, Q, s); }});
      }
      const float* Q = q_;
      float* O = o_;
      RowMap am = map;  // compact admission: the attention runs on the padded 16-row groups
      int Ma = M;
      if (map.ptab) {
        am.tab = map.ptab;
        Ma = map.mpad;
      }
      ops.push_back({p + ".attention", [=](hipStream_t s) { attention(Q, Ma, NH, am, kv, 0, qg, O, s); }});
    }
    auto rr = [&](const std::string& name, int S2, int N, int act, bool resid, float* Y, const float* lnw,
                  const float* lnb, bool ln, float* Hout, float* Hfrag = nullptr) {
      RowReduceArgs a{};
      a.Hfrag = Hfrag;
      a.P = partial_;
      a.S = S2;
      a.M = M;
      a.N = N;
      a.act = act;
      if (resid) {
        a.R = x_;
        a.ldr = D;
      }
      a.Y = Y;
      a.ldy = N;
      a.ln = ln ? 1 : 0;
      a.ln_w = lnw;
      a.ln_b = lnb;
      a.eps = 1e-5f;
      a.Hout = Hout;
      a.ldh = N;
      push_rr(ops, name, a);
    };
    linear_split(ops, p + ".out_gemm", o_, D, M, W(t.out_proj), D, D, &S);
    // step passes with the whole-K linear1 (gemv_fk): the out reduce also stores norm2's output in
    // its A-fragment order, and linear1 applies GELU in its own epilogue (no slabs, no reduce)
    auto fk = qg == 1 && gemv_fk_supported(M, FF, D) ? fkmap_.find(W(t.l1)) : fkmap_.end();
    const bool use_fk = fk != fkmap_.end() && hfrag_;
    rr(p + ".out_reduce_ln2", S, D, ACT_NONE, true, x_, W(t.n2w), W(t.n2b), true, h_, use_fk ? hfrag_ : nullptr);
    auto ffn = use_fk && ffn_hand_ ? ffnmap_.find(W(t.l2)) : ffnmap_.end();
    if (ffn != ffnmap_.end()) {
      // linear1 + GELU + linear2 in one launch (16 K slices of linear2 into the slabs): layer l uses
      // hand-off set l % 2 and empties the other for layer l + 1 (the last layer's launch empties
      // set 0 for the next step's first, NL even)
      static_assert(NL % 2 == 0, "the fused FFN's hand-off sets alternate by layer");
      const float *A = hfrag_, *P1 = fk->second, *P2 = ffn->second;
      float *hand = ffn_hand_, *Pp = partial_;
      int* err = herr_;
      const int set = l & 1;
      const int groups = ffn_groups_;
      auto f8 = ffn8map_.find(W(t.l2));  // weight_quant engines: int8 codes of both matrices
      const uint32_t *Q1 = nullptr, *Q2 = nullptr;
      const float *s1 = nullptr, *s2 = nullptr;
      if (f8 != ffn8map_.end()) {
        Q1 = f8->second.first.first;
        s1 = f8->second.first.second;
        Q2 = f8->second.second.first;
        s2 = f8->second.second.second;
      }
      const bool e4m3 = fp8_ && Q1;
      Op op{p + ".ffn", [=](hipStream_t s) { ffn_fused(A, M, P1, P2, groups, hand, set, Pp, err, s, Q1, s1, Q2, s2, e4m3); },
            2.0 * M * FF * D * 2,
            (Q1 ? 2.0 * FF * D + 8.0 * (FF + D) : 8.0 * FF * D) + 4.0 * ((double)M * D + (double)groups * M * D)};
      // an isolated replay (time_op, overlap_probe) finds its set empty again
      op.prep = [hand](hipStream_t s) { PTTS_HIP(hipMemsetD32Async(hand, 0xFFFFFFFFu, 2 * FFN_HAND_FLOATS, s)); };
      ops.push_back(op);
      S = groups;
    } else {
      if (use_fk) {
        const float* Pk = fk->second;
        const float* A = hfrag_;
        float* U = u_;
        ops.push_back({p + ".ff1_gemm", [=](hipStream_t s) { gemv_fk(A, M, FF, Pk, nullptr, ACT_GELU, U, FF, s); },
                       2.0 * M * FF * D, 4.0 * ((double)FF * D + (double)M * D + (double)M * FF)});
      } else {
        linear_split(ops, p + ".ff1_gemm", h_, D, M, W(t.l1), FF, D, &S);
        rr(p + ".ff1_reduce_gelu", S, FF, ACT_GELU, false, u_, nullptr, nullptr, false, nullptr);
      }
      linear_split(ops, p + ".ff2_gemm", u_, FF, M, W(t.l2), D, FF, &S);
    }
    if (l + 1 < NL)
      rr(p + ".ff2_reduce_ln1", S, D, ACT_NONE, true, x_, W(L_.fl[l + 1].n1w), W(L_.fl[l + 1].n1b), true, h_);
    else
      rr(p + ".ff2_reduce_outnorm", S, D, ACT_NONE, true, x_, W(L_.out_norm_w), W(L_.out_norm_b), out_norm, h_);
  }
}

// Prefill T rows already in x_ into slot `slot` at positions p0.. (tts_model.rs:580-599, 958-964).
void Engine::prefill_rows(std::vector<Op>& ops, int slot, int T, int p0) {
  {
    float* x = x_;
    float* h = h_;
    const float* w = W(L_.fl[0].n1w);
    const float* b = W(L_.fl[0].n1b);
    ops.push_back({"prefill.ln1", [=](hipStream_t s) { layernorm(x, D, h, D, T, D, w, b, 1e-5f, s); }});
  }
  RowMap map{slot, T, p0, nullptr};
  flow_layers(ops, T, map, 16, false, "prefill");
}

// The persistent flow-head launch needs <= 128 rows and ResBlock tensors at one uniform stride
// in the packed blob (pack_weights lays the six blocks out identically).
bool Engine::use_head_chain(int B) const {
  if (!flow_head_fits(B)) return false;
  // every workgroup spins on counters the others bump: all of them must be resident at once
  if (flow_head_grid(B) > head_resident_) return false;
  return head_uniform_stride();
}

bool Engine::head_uniform_stride() const {
  const long s = (long)(L_.rb_w0[1] - L_.rb_w0[0]);
  for (int i = 1; i < FDEPTH; ++i)
    if ((long)(L_.rb_lnw[i] - L_.rb_lnw[i - 1]) != s || (long)(L_.rb_lnb[i] - L_.rb_lnb[i - 1]) != s ||
        (long)(L_.rb_w0[i] - L_.rb_w0[i - 1]) != s || (long)(L_.rb_b0[i] - L_.rb_b0[i - 1]) != s ||
        (long)(L_.rb_w2[i] - L_.rb_w2[i - 1]) != s || (long)(L_.rb_b2[i] - L_.rb_b2[i - 1]) != s)
      return false;
  return true;
}

// FRONT part of a step (FlowLM + flow head) for rows [0, B), handing its frame to buffer `hb`.
void Engine::build_front(std::vector<Op>& ops, int B, int hb) {
  int S = 1;
  // ---- FlowLM step (flow_lm.rs:98-164): input_linear -> transformer -> out_norm. The input
  // projection + norm1 of layer 0 (x_, h_) were computed by the previous step's front_commit, or
  // by refresh_xh() after anything else wrote x_, h_ or lat_in_.
  flow_layers(ops, B, RowMap{0, 1, 0, fpos_}, 1, true, "flow");
  // ---- flow head (mlp.rs:215-383): cond_embed | out_eos, EOS bookkeeping, noise
  linear_split(ops, "head.cond_eos_gemm", h_, D, B, W(L_.cond_eos_w), NCOND, D, &S);
  PTTS_REQUIRE(S <= FLOW_COND_MAX_SLABS, "head.flow_cond sums at most 16 split-K slabs");
  {
    const float* P = partial_;
    const float* bias = W(L_.cond_eos_b);
    const float* temb = temb_;
    const int lsd = lsd_;
    SlotState* st = st_;
    float *ys = ysilu_, *cur = cur_, *eos = eos_;
    ops.push_back({"head.flow_cond", [=](hipStream_t s) { flow_cond(P, S, B, bias, temb, lsd, st, ys, cur, eos, s); },
                   (double)B * NCOND * (S + 1) + 4.0 * lsd * B * FD,
                   4.0 * ((double)S * B * NCOND + NCOND + lsd * FD + lsd * (double)B * FD + B * (LDIM + 1.0))});
  }
  // all adaLN modulations of all lsd steps in one GEMM (mlp.rs:322-368)
  linear_split(ops, "head.ada_gemm", ysilu_, FD, lsd_ * B, W(L_.ada_w), NADA, FD, &S);
  {
    RowReduceArgs a{};
    a.P = partial_;
    a.S = S;
    a.M = lsd_ * B;
    a.N = NADA;
    a.bias = W(L_.ada_b);
    a.Y = mods_;
    a.ldy = NADA;
    if (use_head_chain(B)) {  // side jobs: x0 into hand-off region 0, empty the other regions
      const size_t r0 = (size_t)((B + 15) / 16 * 16) * FD;  // floats per hand-off region
      a.fill = hx_ + r0;
      a.fill_n4 = (long)((hx_floats(B) - r0) / 4);
      a.x0_cur = cur_;
      a.x0_w = fh_inw_t_;
      a.x0_b = W(L_.inproj_b);
      a.x0_hx = hx_;
      a.x0_B = B;
      a.fhm = fhm_;
      a.fhm_B = B;
    }
    push_rr(ops, "head.ada_reduce", a);
  }
  // lsd_decode Euler steps (flow_lm.rs:7-22) over ResBlocks (mlp.rs:146-213): one persistent
  // launch (k_flow_head) for the whole chain, or 28 GEMM + row-reduce launches per step
  if (use_head_chain(B)) {
    FlowHeadArgs f{};
    f.B = B;
    f.lsd = lsd_;
    f.euler_scale = 1.0f / (float)lsd_;
    f.cur = cur_;
    f.mods = mods_;
    f.ldm = NADA;
    f.in_w = W(L_.inproj_w);
    f.in_b = W(L_.inproj_b);
    f.lnw = W(L_.rb_lnw[0]);
    f.lnb = W(L_.rb_lnb[0]);
    f.w0 = W(L_.rb_w0[0]);
    f.b0 = W(L_.rb_b0[0]);
    f.w2 = W(L_.rb_w2[0]);
    f.b2 = W(L_.rb_b2[0]);
    f.blk = (long)(L_.rb_w0[1] - L_.rb_w0[0]);
    f.fin_w = W(L_.fin_w);
    f.fin_b = W(L_.fin_b);
    f.wp = fhw_;
    f.fhm = fhm_;
    f.hx = hx_;
    f.x0_ready = 1;
    f.ctr = hctr_;
    f.err = herr_;
    f.dbg = probe_env("PTTS_HEAD_DBG") ? (unsigned long long*)strtoull(probe_env("PTTS_HEAD_DBG"), nullptr, 0) : nullptr;
    const double fl = 2.0 * lsd_ * B * ((double)FD * LDIM + 2.0 * FDEPTH * FD * FD + (double)LDIM * FD);
    const double by = 4.0 * ((double)FD * LDIM + 2.0 * FDEPTH * FD * FD + (double)LDIM * FD) +
                      4.0 * lsd_ * B * ((double)FDEPTH * 3 * FD + 2 * FD);
    // isolated replays: re-empty the regions and recompute x0 (the adaLN reduce's side jobs)
    float* hx = hx_;
    const size_t nhx = hx_floats(B);
    const float *cur = cur_, *iw = fh_inw_t_, *ib = W(L_.inproj_b);
    Op op{"head.chain", [f](hipStream_t s) { flow_head(f, s); }, fl, by};
    op.prep = [hx, nhx, cur, iw, ib, B](hipStream_t s) {
      PTTS_HIP(hipMemsetD32Async(hx, 0xFFFFFFFFu, nhx, s));
      flow_head_x0(cur, iw, ib, hx, B, s);
    };
    ops.push_back(op);
  }
  for (int st = 0; st < lsd_ && !use_head_chain(B); ++st) {
    const float* mods = mods_ + (size_t)st * B * NADA;
    const std::string p = "head.s" + std::to_string(st);
    linear_split(ops, p + ".inproj_gemm", cur_, LDIM, B, W(L_.inproj_w), FD, LDIM, &S);
    {
      RowReduceArgs a{};
      a.P = partial_;
      a.S = S;
      a.M = B;
      a.N = FD;
      a.bias = W(L_.inproj_b);
      a.Y = xf_;
      a.ldy = FD;
      a.ln = 1;
      a.ln_w = W(L_.rb_lnw[0]);
      a.ln_b = W(L_.rb_lnb[0]);
      a.eps = 1e-6f;
      a.mshift = mods + 0;
      a.mscale = mods + FD;
      a.ldm = NADA;
      a.Hout = hf_;
      a.ldh = FD;
      push_rr(ops, p + ".inproj_reduce", a);
    }
    for (int i = 0; i < FDEPTH; ++i) {
      const std::string pb = p + ".rb" + std::to_string(i);
      {
        linear_split(ops, pb + ".mlp0_gemm", hf_, FD, B, W(L_.rb_w0[i]), FD, FD, &S);
        RowReduceArgs a{};
        a.P = partial_;
        a.S = S;
        a.M = B;
        a.N = FD;
        a.bias = W(L_.rb_b0[i]);
        a.act = ACT_SILU;
        a.Y = uf_;
        a.ldy = FD;
        push_rr(ops, pb + ".mlp0_reduce", a);
      }
      linear_split(ops, pb + ".mlp2_gemm", uf_, FD, B, W(L_.rb_w2[i]), FD, FD, &S);
      {
        RowReduceArgs a{};
        a.P = partial_;
        a.S = S;
        a.M = B;
        a.N = FD;
        a.bias = W(L_.rb_b2[i]);
        a.gate = mods + (size_t)i * 3 * FD + 2 * FD;
        a.ldg = NADA;
        a.R = xf_;
        a.ldr = FD;
        a.Y = xf_;
        a.ldy = FD;
        a.ln = 1;
        a.eps = 1e-6f;
        if (i + 1 < FDEPTH) {
          a.ln_w = W(L_.rb_lnw[i + 1]);
          a.ln_b = W(L_.rb_lnb[i + 1]);
          a.mshift = mods + (size_t)(i + 1) * 3 * FD;
          a.mscale = mods + (size_t)(i + 1) * 3 * FD + FD;
        } else {  // FinalLayer: non-affine LN + final adaLN (mlp.rs:182-213)
          a.mshift = mods + (size_t)FDEPTH * 3 * FD;
          a.mscale = mods + (size_t)FDEPTH * 3 * FD + FD;
        }
        a.ldm = NADA;
        a.Hout = hf_;
        a.ldh = FD;
        push_rr(ops, pb + ".mlp2_reduce", a);
      }
    }
    linear_split(ops, p + ".final_gemm", hf_, FD, B, W(L_.fin_w), LDIM, FD, &S);
    {
      RowReduceArgs a{};
      a.P = partial_;
      a.S = S;
      a.M = B;
      a.N = LDIM;
      a.bias = W(L_.fin_b);
      a.euler = cur_;
      a.euler_scale = 1.0f / (float)lsd_;
      push_rr(ops, p + ".euler", a);
    }
  }
  // ---- EOS rule, frame flags, hand-off of the frame to the back part, next backbone input
  {
    FrontCommitArgs c{};
    c.B = B;
    c.st = st_;
    c.eos = eos_;
    c.cur = cur_;
    c.lat_in = lat_in_;
    c.lat_out = lat_out_[hb];
    c.eos_out = eos_out_[hb];
    c.flags = flags_[hb];
    c.fpos = fpos_;
    c.Wt = inw_t_;
    c.lnw = W(L_.fl[0].n1w);
    c.lnb = W(L_.fl[0].n1b);
    c.x = x_;
    c.h = h_;
    c.err_dev = herr_;
    c.err_host = h_err_;
    c.n_zero = nfr_ > 1 ? max_slots_ - B : 0;
    ops.push_back({"front_commit", [c](hipStream_t s) { front_commit(c, s); }, 2.0 * B * D * LDIM,
                   (double)B * (sizeof(SlotState) * 2 + 4.0 * (1 + 3 * LDIM + 1 + 2 + 2 + 2 * D)) +
                       4.0 * ((double)D * LDIM + 2 * D)});
  }
}

// Tiles of the back part's GEMMs and convs at B >= 16 (the MFMA-bound shapes), one row per launch:
// LDS-DMA tile layout (kernels.hip gemm_launch) and split-K slices. Chosen from tools/mm_bench.hip
// (each launch alone on the chip, B = 32) and A/B runs of the pipelined step, where the back part
// shares every CU with the latency-bound front part. Pipelined split-K at most 2
// since round 5 (the front part bounds the step, and 4 slices' slab traffic slowed it: 0.549 ->
// 0.530 ms, profiles/r05/back_splits_ab.txt). Below B = 16 every GEMM runs on the 32x32 register
// tile (layout 0) with the split-K noted at the launch.
struct BackTile {
  int layout, splits;
};
static BackTile back_tile(const std::string& op, bool pipeline) {
  static const struct {
    const char* op;
    BackTile seq, pipe;
  } table[] = {
      {"mimi.qkv", {32, 1}, {32, 1}},
      {"mimi.out", {32, 4}, {32, 2}},
      {"mimi.ff1", {32, 1}, {32, 1}},
      {"mimi.ff2", {32, 4}, {32, 2}},
      {"seanet.conv0", {32, 4}, {32, 2}},
      {"seanet.up0.convtr", {32, 4}, {32, 2}},
      {"seanet.up1.convtr", {32, 1}, {32, 1}},
      {"seanet.up2.convtr", {32, 1}, {32, 1}},
      // the stage-0/1 residual convs when not fused (see resblock_fused)
      {"seanet.up0.res_conv3", {18, 1}, {18, 1}},
      {"seanet.up1.res_conv3", {20, 1}, {20, 1}},
      {"seanet.up0.res_conv1", {6, 1}, {6, 1}},
      {"seanet.up1.res_conv1", {6, 1}, {6, 1}},
      {"seanet.up2.res_conv3", {14, 1}, {14, 1}},
      {"seanet.up2.res_conv1", {6, 1}, {23, 1}},
  };
  for (const auto& t : table)
    if (op == t.op) return pipeline ? t.pipe : t.seq;
  throw Error(PTTS_ERR_INVALID, "no tile for " + op);
}

// BACK part of a step: Mimi decode of the frames the front part left in buffer `hb`; `qp` is the
// frame's parity for the quantizer history (the previous frame's quantizer output is in qp ^ 1).
void Engine::build_back(std::vector<Op>& ops, int B, int hb, int nfr, int qp, int pcm_frames) {
  PTTS_REQUIRE(nfr >= 1 && nfr <= nfr_, "frames per back pass out of range");
  PTTS_REQUIRE(pcm_frames >= nfr, "pass block smaller than the pass");
  int hbs[NFR_MAX];  // frame f's hand-off buffer (f < nfr)
  for (int f = 0; f < NFR_MAX; ++f) hbs[f] = (hb + std::min(f, nfr - 1)) % nhb_;
  const bool big = B >= 16;  // B * 16 >= 256 Mimi rows: the LDS-DMA tiles fill the chip
  auto tile = [&](const std::string& op, int small_splits) {
    BackTile t = big ? back_tile(op, pipeline_) : BackTile{0, small_splits};
    // four-frame passes: SEANet conv0 and the stage-0 transposed conv have twice a pair pass's rows
    // (B * 64: 256 / 1,024 64 x 64 tiles at B = 32), enough to fill the chip unsplit, so neither
    // writes slabs nor needs its reduce launch (steady step 0.5179 -> 0.5137 ms,
    // profiles/r06/ab_quad_splits.txt; unsplit in pair passes: +2.7 %, profiles/r06/ab1.txt)
    if (big && nfr >= 4 && (op == "seanet.conv0" || op == "seanet.up0.convtr")) t.splits = 1;
    // back_mfma bf16 / bf16x6: the bf16-operand / split-f32 twin of the ILV tile (kernels.hip
    // PTTS_GLB: layout + 100, PTTS_GLX6: + 200); the register-blocked and non-ILV tiles of the f32
    // table map to the 64 x 64 one
    if (big && back_mfma_ == PTTS_BACK_BF16) t.layout = 100 + (t.layout == 35 || t.layout == 31 ? t.layout : 32);
    if (big && back_mfma_ == PTTS_BACK_F32X6) t.layout = 200 + (t.layout == 35 ? t.layout : 32);
    tile_override(op, t.layout, t.splits);  // probe builds only (tools/back_tune.py)
    return t;
  };
  // ---- Mimi decode (mimi.rs:143-157): quantize + upsample, decoder transformer, SEANet decoder
  {
    const float *sd = W(L_.emb_std), *mn = W(L_.emb_mean), *wq = W(L_.quant_w), *wu = W(L_.up_w);
    const float *lw = W(L_.mdec[0].n1w), *lb = W(L_.mdec[0].n1b);
    const float* qin = qprev_;
    float* qout = qcur_;
    float *x = mx_, *h = mh_;
    std::array<const float*, NFR_MAX> lat;
    std::array<const FrameFlags*, NFR_MAX> fl;
    for (int f = 0; f < NFR_MAX; ++f) {
      lat[f] = lat_out_[hbs[f]];
      fl[f] = flags_[hbs[f]];
    }
    ops.push_back({"mimi.quant_upsample",
                   [=](hipStream_t s) { quant_upsample(lat.data(), fl.data(), nfr, B, sd, mn, wq, wu, qin, qout, x, h, lw, lb, s); },
                   (double)B * nfr * (2.0 * MD * LDIM + 2.0 * MD * 2 * UP + 8.0 * UP * MD),
                   4.0 * ((double)B * nfr * (LDIM + 2 * MD + 2.0 * UP * MD) + 2.0 * MD * LDIM + MD * 2.0 * UP + 2.0 * MD)});
  }
  const int MR = B * UP * nfr;  // Mimi rows of the pass: 16 per frame per utterance
  RowMap mmap{0, UP * nfr, 0, mpos_};
  // a split-K GEMM into the back part's own slab buffer, its epilogue in a row reduce
  auto split_gemm = [&](const std::string& name, const float* X, int M, const float* Wt, int N, int K, BackTile t) {
    PTTS_REQUIRE(t.splits >= 1 && t.splits <= 16, name + ": split-K 1..16");
    PTTS_REQUIRE((size_t)t.splits * M * N <= mpcap_, "back split-K slab buffer too small");
    GemmArgs a{};
    a.mode = 0;
    a.layout = t.layout;
    a.M = M;
    a.N = N;
    a.K = K;
    a.Nw = (N + 31) / 32 * 32;
    a.X = X;
    a.ldx = K;
    a.W = Wt;
    a.S = t.splits;
    a.partial = mpartial_;
    attach_split(a);
    const int S = t.splits;
    ops.push_back({name, [a, S](hipStream_t s) { gemm(a, S, s); }, 2.0 * M * N * K,
                   4.0 * ((double)N * K + (double)M * K + (double)S * M * N)});
  };
  for (int l = 0; l < MNL; ++l) {
    const Layout::TL& t = L_.mdec[l];
    const std::string p = "mimi.l" + std::to_string(l);
    KvStore kv{ring_ + (long)l * ring_layer_, ring_slot_, RING};
    {  // QKV in one pass; RoPE + ring append inside the attention launch
      const BackTile tq = tile("mimi.qkv", 1);
      dense_op(ops, p + ".qkv_gemm", mh_, MR, W(t.in_proj), 3 * MD, MD, nullptr, ACT_NONE, nullptr, nullptr, mqkv_,
               tq.layout);
      const float* qkv = mqkv_;
      float* O = mo_;
      // per utterance: the K and V of its window (W keys x 8 heads x 64 x 2, read once for its 16
      // queries), its 16 QKV rows in, the 16 output rows, the appended K/V; 16 queries x W keys x
      // 8 heads x 64 x 4 flops = 65,536 W
      const double Wn = plan_win_ > 0 ? plan_win_ : (double)(MCTX + UP - 1);
      if (nfr == 1) {
        ops.push_back({p + ".attention", [=](hipStream_t s) { attention16_qkv(qkv, MR, MNH, mmap, kv, MCTX, O, s); },
                       (double)B * 65536.0 * Wn,
                       (double)B * (4.0 * 2 * MNH * 64 * Wn + 4.0 * UP * (3.0 * MD + MD + 2.0 * MD))});
      } else {  // two frames: the second frame's queries see the first frame's keys, appended by
        // other workgroups, so the append (with RoPE) is its own launch ahead of the attention
        float* Q = mq_;
        ops.push_back({p + ".qkv_rope", [=](hipStream_t s) { qkv_rope_append(nullptr, 0, qkv, MR, MNH, mmap, kv, Q, s); },
                       0.0, 4.0 * MR * (3.0 * MD + 3.0 * MD)});
        ops.push_back({p + ".attention", [=](hipStream_t s) { attention(Q, MR, MNH, mmap, kv, MCTX, 16, O, s); },
                       (double)B * nfr * 65536.0 * Wn,
                       (double)B * nfr * (4.0 * 2 * MNH * 64 * Wn + 4.0 * UP * (MD + MD))});
      }
    }
    {  // out projection, split-K; LayerScale + residual and this layer's norm2 in the reduce
      const BackTile to = tile("mimi.out", 4);
      split_gemm(p + ".out_gemm", mo_, MR, W(t.out_proj), MD, MD, to);
      RowReduceArgs r{};
      r.P = mpartial_;
      r.S = to.splits;
      r.M = MR;
      r.N = MD;
      r.gate = W(t.ls1);  // per-column LayerScale: gate row stride 0
      r.ldg = 0;
      r.R = mx_;
      r.ldr = MD;
      r.Y = mx_;
      r.ldy = MD;
      r.ln = 1;
      r.ln_w = W(t.n2w);
      r.ln_b = W(t.n2b);
      r.eps = 1e-5f;
      r.Hout = mh_;
      r.ldh = MD;
      ops.push_back(rr_op(p + ".out_reduce_ln2", r));
    }
    {  // linear1 + GELU in the tile epilogue
      const BackTile tf = tile("mimi.ff1", 1);
      dense_op(ops, p + ".ff1_gemm", mh_, MR, W(t.l1), MFF, MD, nullptr, ACT_GELU, nullptr, nullptr, mu_, tf.layout);
    }
    {  // linear2 (K = 2048), split-K; LayerScale + residual (+ the next layer's norm1) in the reduce.
       // Few rows (B < 16, the first-chunk path): 32x32 tiles, 8 slices (16 -> 128 workgroups)
      const BackTile tf = tile("mimi.ff2", 8);
      split_gemm(p + ".ff2_gemm", mu_, MR, W(t.l2), MD, MFF, tf);
      RowReduceArgs r{};
      r.P = mpartial_;
      r.S = tf.splits;
      r.M = MR;
      r.N = MD;
      r.gate = W(t.ls2);
      r.ldg = 0;
      r.R = mx_;
      r.ldr = MD;
      r.Y = mx_;
      r.ldy = MD;
      if (l + 1 < MNL) {  // the next layer's norm1 on the reduced rows (no separate LayerNorm launch)
        r.ln = 1;
        r.ln_w = W(L_.mdec[l + 1].n1w);
        r.ln_b = W(L_.mdec[l + 1].n1b);
        r.eps = 1e-5f;
        r.Hout = mh_;
        r.ldh = MD;
      }
      ops.push_back(rr_op(p + ".ff2_reduce", r));
    }
  }
  // SEANetDecoder (seanet.rs:396-402): conv0 -> [ELU, convtr(r), resblock] x3 -> ELU, conv(64->1).
  // Every ELU is applied once, by the producer of the activation (elu_out / the dual store Y2),
  // so the consumers' operand loads are plain: a0, ce and ca hold ELU'd activations (and so do the
  // histories of the convs that read them; elu(0) = 0 keeps the zero reset valid), cb stays raw for
  // the resblock skip. Transposed convs run with their r phases merged into N: one 2-tap conv over
  // rows (x[q-1], x[q]) whose output row q is the r time rows q*r .. q*r+r-1 of the channels-last
  // output, N = r * Cout (packed [r][Cout][2][Cin] = [r*Cout][2*Cin]).
  {  // conv0 (K = 7 x 512, M = 16 B rows): split-K fills the chip; bias + ELU in the reduce (every B:
     // at B = 1 the unsplit launch had 16 workgroups, 27.4 us)
    const BackTile tc = tile("seanet.conv0", 8);
    if (big && tc.splits == 1) {  // unsplit: bias + ELU in the tile epilogue, no reduce launch
      conv_op(ops, "seanet.conv0", mx_, B, 16 * nfr, 512, hist_[0], 6, 1, 0, W(L_.dc0_w), 512, 7, 1, W(L_.dc0_b),
              nullptr, a0_, 16 * nfr, 1, tc.layout, 1, nullptr, 1);
    } else {
    const int s_c0 = std::max(tc.splits, 2);
    conv_op(ops, "seanet.conv0", mx_, B, 16 * nfr, 512, hist_[0], 6, 1, 0, W(L_.dc0_w), 512, 7, 1, nullptr, nullptr,
            nullptr, 16 * nfr, 1, big ? tc.layout : 6, 0, nullptr, s_c0);
    RowReduceArgs r{};
    r.P = mpartial_;
    r.S = s_c0;
    r.M = B * 16 * nfr;
    r.N = 512;
    r.bias = W(L_.dc0_b);
    r.act = ACT_ELU;
    r.Y = a0_;
    r.ldy = 512;
    ops.push_back(rr_op("seanet.conv0_reduce", r));
    }
  }
  const float* cin_buf = a0_;
  int T = 16 * nfr, ch = 512;
  // a pass's PCM is [B][pcm_frames][1920] in its pass block (frames past nfr untouched)
  float* pcm_out = pcm_frames == 1 ? pcm_[hb] : pcmp_[hb / pcm_frames];
  const long pcm_ld = (long)pcm_frames * FRAME;
  bool fin_fused = false;  // the final conv ran in the stage-2 residual block's epilogue
  // fused residual blocks (k3 conv + ELU + k1 conv + skip + ELU, the hidden rows in LDS) where they
  // beat the two conv launches: stage 2 (480 workgroups; 22.5 us against 16.8 + 11.0). Stages
  // 0 and 1 have 96 / 160 workgroups of it and measured slower than their two tuned launches.
  // PTTS_RESBLOCK_STAGES (probe builds): bit mask of the stages that fuse.
  // Four-frame passes give stages 0 and 1 four times their single-frame workgroups (384 / 640 at
  // B = 32), and there the fused block of every stage pays: 0.5049 -> 0.5008 ms
  // (profiles/r06/ab_resblock.txt; stage 1 fused in pair passes: +0.8 %, round 5)
  int fused_stages = nfr >= 4 ? 7 : 4;
  if (probe_env("PTTS_RESBLOCK_STAGES")) fused_stages = atoi(probe_env("PTTS_RESBLOCK_STAGES"));
  // (f32 only: its own MFMA loop). A fused stage's (unsplit) transposed conv stores no ELU'd copy:
  // the block ELUs the raw rows as they enter LDS
  auto fuse_res = [&](int i) { return big && (fused_stages >> i & 1) && back_mfma_ == PTTS_BACK_F32; };
  // stages whose fused residual block reads the RAW transposed-conv rows (E = elu(R) applied as the
  // rows enter LDS): every fused stage whose transposed conv is unsplit (a split one's reduce stores
  // both the raw and the ELU'd rows)
  bool raw_only[3] = {false, false, false};
  for (int i = 0; i < 3; ++i) {
    const int r = RATIOS[i];
    const std::string p = "seanet.up" + std::to_string(i);
    const BackTile tt = tile(p + ".convtr", 1);
    raw_only[i] = fuse_res(i) && !(big && tt.splits > 1);
    if (big && tt.splits > 1) {  // stage 0 (M = 16 B rows): split-K; bias + dual raw / ELU store in the reduce
      PTTS_REQUIRE(i == 0, "split-K transposed conv: stage 0 only");
      conv_op(ops, p + ".convtr", cin_buf, B, T, ch, hist_[1], 1, 1, 0, W(L_.dtr_w[0]), r * (ch / 2), 2, 1, nullptr,
              nullptr, nullptr, T, 1, tt.layout, 0, nullptr, tt.splits);
      RowReduceArgs rr{};
      rr.P = mpartial_;
      rr.S = tt.splits;
      rr.M = B * T;
      rr.N = r * (ch / 2);
      rr.bias = trb_[0];
      rr.Y = cb_[0];
      rr.Y2 = ce_[0];
      rr.ldy = r * (ch / 2);
      ops.push_back(rr_op(p + ".convtr_reduce", rr));
    } else {
      // stage 2 fused below: no ELU'd copy (the residual block ELUs the raw rows as it loads them)
      conv_op(ops, p + ".convtr", cin_buf, B, T, ch, hist_[1 + 2 * i], 1, 1, 0, W(L_.dtr_w[i]), r * (ch / 2), 2, 1,
              trb_[i], nullptr, cb_[i], T, 1, tt.layout, 0, fuse_res(i) ? nullptr : ce_[i]);
    }
    T *= r;
    ch /= 2;
    if (fuse_res(i)) {
      ResBlockArgs rb{ce_[i], hist_[2 + 2 * i], cb_[i], W(L_.dra_w[i]), W(L_.dra_b[i]), W(L_.drb_w[i]),
                      W(L_.drb_b[i]), ca_[i], B, T, ch};
      const double hd = ch / 2;
      double fl = 2.0 * B * T * (hd * 3 * ch + ch * hd);
      double by = 4.0 * ((double)B * T * ch * 3 + B * 2.0 * ch + hd * 3 * ch + ch * hd + hd + ch);
      if (raw_only[i]) {  // E = elu(R) as the rows enter LDS (a split-K reduce stores both)
        rb.E = cb_[i];
        rb.e_raw = 1;
        by -= 4.0 * B * T * ch;  // E and R are the same rows: read once
      }
      if (i == 2 && T % RESBLOCK_FIN_TT == 0) {  // + the final conv (64 -> 1, k = 3) of the tile's rows
        rb.fw = W(L_.dfin_w);
        rb.fb = W(L_.dfin_b);
        rb.fH = hist_[7];
        rb.fout = pcm_out;
        rb.fld = pcm_ld;
        rb.fside = fin_side_;
        fin_fused = true;
        fl += 2.0 * B * T * 3 * 64;
        by += 4.0 * ((double)B * T + B * 2.0 * 64 + 3 * 64 + 1);
      }
      ops.push_back({p + ".resblock", [rb](hipStream_t s) { resblock(rb, s); }, fl, by});
    } else {  // the two convs (few rows: 32x32 tiles, more workgroups than the fused tiles)
      const int lr3 = big ? tile(p + ".res_conv3", 1).layout : 0, lr1 = big ? tile(p + ".res_conv1", 1).layout : 0;
      conv_op(ops, p + ".res_conv3", ce_[i], B, T, ch, hist_[2 + 2 * i], 2, 1, 0, W(L_.dra_w[i]), ch / 2, 3, 1,
              W(L_.dra_b[i]), nullptr, cv_[i], T, 1, lr3, 1);
      conv_op(ops, p + ".res_conv1", cv_[i], B, T, ch / 2, nullptr, 0, 1, 0, W(L_.drb_w[i]), ch, 1, 1,
              W(L_.drb_b[i]), cb_[i], ca_[i], T, 1, lr1, 1);
    }
    cin_buf = ca_[i];
  }
  if (!fin_fused) {
    const float *X = ca_[2], *H = hist_[7], *w = W(L_.dfin_w), *b = W(L_.dfin_b);
    float* Y = pcm_out;
    const int TF = FRAME * nfr;
    ops.push_back({"seanet.conv_final", [=](hipStream_t s) { conv_cout1(X, H, B, TF, 64, 3, w, b, Y, 0, s, pcm_ld); },
                   2.0 * B * TF * 3 * 64, 4.0 * ((double)B * TF * 64 + B * 2.0 * 64 + B * TF + 3 * 64 + 1)});
  }
  // ---- commit of the back part: conv histories and Mimi positions of rows with a frame
  {
    CommitArgs c{};
    const float* srcs[8] = {mx_, a0_, ce_[0], ca_[0], ce_[1], ca_[1], ce_[2], ca_[2]};
    for (int i = 0; i < 8; ++i) c.h[i] = HistDesc{srcs[i], hist_[i], hist_T_[i] * nfr, hist_C_[i], hist_P_[i]};
    for (int i = 0; i < 3; ++i)  // a raw-only fused stage's k3-conv history: elu(raw rows)
      if (raw_only[i]) c.h[2 + 2 * i] = HistDesc{cb_[i], hist_[2 + 2 * i], hist_T_[2 + 2 * i] * nfr, hist_C_[2 + 2 * i], hist_P_[2 + 2 * i], 1};
    c.nh = 8;
    c.B = B;
    for (int f = 0; f < NFR_MAX; ++f) c.flags[f] = flags_[hbs[f]];
    c.nfr = nfr;
    c.mpos = mpos_;
    c.qcur = qcur_;
    c.qprev = qprev_;
    if (fin_fused) {
      c.fin_pcm = pcm_out;
      c.fin_side = fin_side_;
      c.fin_T = FRAME * nfr;
      c.fin_ld = pcm_ld;
    }
    double hb_bytes = 0;  // every history row is read from its activation and stored
    for (int i = 0; i < 8; ++i) hb_bytes += 8.0 * B * hist_P_[i] * hist_C_[i];
    ops.push_back({"commit", [c](hipStream_t s) { step_commit(c, s); }, 0.0, hb_bytes + 16.0 * B});
  }
}

// The whole step in plan order (front then back, buffer 0): plan listing and per-op timing.
std::vector<Op> Engine::build_step(int B) {
  std::vector<Op> ops;
  build_front(ops, B, 0);
  build_back(ops, B, 0, nfr_, 0, nfr_);
  return ops;
}

std::vector<std::string> Engine::plan_names(int B) {
  PTTS_REQUIRE(B >= 1 && B <= max_slots_, "n_rows out of range");
  // the attention costs are for the rows' current positions (what time_op replays): the mean
  // FlowLM context over rows [0, B) and the mean Mimi window (positions + 16 queries, <= 265)
  sync();
  std::vector<int> fp(B), mp(B);
  PTTS_HIP(hipMemcpy(fp.data(), fpos_, sizeof(int) * B, hipMemcpyDeviceToHost));
  PTTS_HIP(hipMemcpy(mp.data(), mpos_, sizeof(int) * B, hipMemcpyDeviceToHost));
  double L = 0, Wn = 0, kvu = 0;
  std::vector<const float*> seen;  // distinct shared voice prefixes: read once per launch
  for (int b = 0; b < B; ++b) {
    L += fp[b] + 1;
    Wn += std::min(mp[b] + UP, MCTX + UP - 1);
    const int F = share_voice_ && h_vpre_[b] ? h_vlen_[b] : 0;
    kvu += fp[b] + 1 - F;
    if (F > 0 && std::find(seen.begin(), seen.end(), h_vpre_[b]) == seen.end()) {
      seen.push_back(h_vpre_[b]);
      kvu += F;
    }
  }
  plan_ctx_ = L / B;
  plan_win_ = Wn / B;
  plan_kvu_ = kvu;
  std::vector<std::string> v;
  char buf[64];
  for (auto& op : build_step(B)) {
    snprintf(buf, sizeof buf, "\t%.6g\t%.6g", op.flops, op.bytes);
    v.push_back(op.name + buf);
  }
  return v;
}

// A stream wait costs the front stream a few us at the graph boundary even on a completed event
// (profiles/r04/graph_boundary_ab.txt): the hand-off buffer waits are enqueued only when the host
// sees the event still pending (the pass that last read the buffer is three passes old, so it has
// normally completed by the time the call is issued).
void Engine::wait_unless_done(hipStream_t s, hipEvent_t e) {
  const hipError_t r = hipEventQuery(e);
  if (r == hipSuccess) return;
  (void)hipGetLastError();
  PTTS_HIP(hipStreamWaitEvent(s, e, 0));
}

// The frame(s) a back part decoded leave HBM by a copy enqueued right after its graph on the same
// stream (fetch() reads host memory): a DMA-engine transfer, not a blit-kernel node of the graph,
// whose workgroups held CUs beside the front part while the host writes drained.
void Engine::copy_out(int B, int hb, hipStream_t s) {
  if (nfr_ > 1) {  // every frame of the pass (PCM and meta) in one copy
    const size_t n = (size_t)max_slots_ * nfr_ * FRAME + nfr_ * ((meta_floats_ + 31) / 32 * 32);
    PTTS_HIP(hipMemcpyAsync(h_pcmp_[hb / nfr_], pcmp_[hb / nfr_], sizeof(float) * n, hipMemcpyDeviceToHost, s));
  } else {
    PTTS_HIP(hipMemcpyAsync(h_pcm_[hb], pcm_[hb], sizeof(float) * B * FRAME, hipMemcpyDeviceToHost, s));
    PTTS_HIP(hipMemcpyAsync(h_meta_[hb], meta_[hb], sizeof(float) * meta_floats_, hipMemcpyDeviceToHost, s));
  }
}

hipGraphExec_t Engine::part_graph(int part, int B, int hb, int qp, int nfr) {
  if (part == 0) qp = nfr = 0;  // the front part does not use the quantizer history
  const int key = (((B * 2 + part) * NHB + hb) * 2 + qp) * (NFR_MAX + 1) + nfr;
  auto it = graphs_.find(key);
  if (it != graphs_.end()) return it->second;
  std::vector<Op> ops;
  if (part == 0) build_front(ops, B, hb);
  else build_back(ops, B, hb, nfr, qp, nfr_);
  hipGraph_t g = nullptr;
  // captured on the stream it is launched on (the back part of a pipelined step: stream_be_)
  hipStream_t cs = part == 1 && pipeline_ ? stream_be_ : stream_;
  PTTS_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  // back part of a pipelined step: its launches leave room for the concurrent front part
  set_wg_cap(part == 1 && pipeline_ ? back_cap_ : 0);
  // the back part's tile waves issue at priority 3 beside the front part's (pair passes: steady step
  // 0.5533 -> 0.5496 ms, devfn.h back_prio), except in four-frame passes, whose back part has four
  // steps' time per pass: there the front part's waves keep the default order (0.5134 -> 0.5106
  // ms, profiles/r06/ab_bf8.txt)
  set_back_hi(part == 1 && pipeline_ && nfr_ >= 4 ? 0 : 1);
  // per-op cap override for back-part launches: PTTS_OP_CAP="name=cap,..." (tuning)
  const char* opcap = part == 1 && pipeline_ ? probe_env("PTTS_OP_CAP") : nullptr;
  try {
#ifdef PTTS_PROBES
    if (stamp_ring_) stamp(stamp_ring_, stamp_ctr_, (unsigned)(part << 8 | hb << 1), cs);
#endif
#ifdef PTTS_PROBES
    // PTTS_STAMP_OPS: a stamp ahead of every op as well (two back to back first: the stamp cost)
    const bool op_stamps = stamp_ring_ && probe_env("PTTS_STAMP_OPS");
    if (op_stamps) {
      stamp(stamp_ring_, stamp_ctr_, 0x10000u | part << 12 | 0xFFEu, cs);
      stamp(stamp_ring_, stamp_ctr_, 0x10000u | part << 12 | 0xFFFu, cs);
      stamp_names_[part].clear();
      for (const Op& op : ops) stamp_names_[part].push_back(op.name);
    }
    unsigned op_i = 0;
#endif
    for (const Op& op : ops) {
#ifdef PTTS_PROBES
      if (op_stamps) stamp(stamp_ring_, stamp_ctr_, 0x10000u | part << 12 | op_i++, cs);
#endif
      if (opcap) {
        int cap = back_cap_;
        const std::string e(opcap), key = op.name + "=";
        const size_t at = e.find(key);
        if (at != std::string::npos && (at == 0 || e[at - 1] == ',')) cap = atoi(e.c_str() + at + key.size());
        set_wg_cap(cap);
      }
      op.fn(cs);
    }
    // part 0: the hand-off timeout word (read by fetch() without a device round trip) and the
    // flags of rows past B are front_commit's side jobs; part 1: the frames leave HBM by copy_out()
    // after the graph (no copy nodes in either graph)
#ifdef PTTS_PROBES
    if (stamp_ring_) stamp(stamp_ring_, stamp_ctr_, (unsigned)(part << 8 | hb << 1 | 1), cs);
#endif
  } catch (...) {
    set_wg_cap(0);
    set_back_hi(1);
    (void)hipStreamEndCapture(cs, &g);
    throw;
  }
  set_wg_cap(0);
  set_back_hi(1);
  PTTS_HIP(hipStreamEndCapture(cs, &g));
  hipGraphExec_t ge = nullptr;
  PTTS_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  graph_defs_[key] = g;
  graphs_[key] = ge;
  return ge;
}

// One call = one step of the generation loop for rows [0, B).
//   sequential: front(k) then back(k) on one stream; the call's frame is frame k.
//   pipelined:  front(k) on stream_ || back(k-1) on stream_be_ (the back part decodes the frame
//               the previous call's front part produced); the call's frame is frame k-1. Frame
//               k's hand-off buffer is k % nhb_ (3): front(k)
//               waits only for back(k - nhb_), the last reader of its buffer, and back(k-1) for
//               front(k-1).
void Engine::step_async(int B) {
  PTTS_REQUIRE(B >= 1 && B <= max_slots_, "n_rows out of range");
  call_async(B, true);
}

// A flush call: frames already computed are decoded and delivered as by a step call, but no row
// computes a new frame (every row pauses for the call, as rows past n_rows do). Pipelined engines
// only, and not right after an admission (the admitted rows' first frame must fall on a step
// call: with multi-frame passes it must be the first frame of a pass).
void Engine::flush_async(int B) {
  PTTS_REQUIRE(B >= 1 && B <= max_slots_, "n_rows out of range");
  PTTS_REQUIRE(pipeline_, "flush: pipelined engines only");
  PTTS_REQUIRE(!admitted_since_call_ && act_slots_.empty(), "flush right after an admission: step first");
  call_async(B, false);
}

void Engine::call_async(int B, bool run_front) {
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_HIP(hipSetDevice(dev_));
  // Multi-frame passes (nfr = back_frames > 1): one back pass decodes a row's frames of the pass as
  // a prefix (frames nfr j, nfr j + 1, ..). A row the pass's first call did not cover must not
  // produce a later frame of the pass alone, so a call inside a pass covers at most the previous
  // call's rows; rows past that are paused for the call, as rows past n_rows are (a first call
  // that was a flush covered none: the rest of the pass are flushes too).
  if (pipeline_ && nfr_ > 1 && (k_ % nfr_)) {
    B = std::min(B, rows_hb_[(k_ - 1) % nhb_]);
    if (B == 0) run_front = false;
  }
  if (!run_front) B = 0;
  admitted_since_call_ = false;
  prev_hb_ = out_hb_;
  prev_rows_ = out_rows_;
  prev_k_ = out_k_;
  const int hb = (int)(k_ % nhb_), qp = (int)(k_ & 1);
  // the front part of this call, or (a flush) its hand-off buffer marked frame-less
  hipGraphExec_t front = B > 0 ? part_graph(0, B, hb, 0, 0) : nullptr;
  auto run_front_part = [&]() {
    if (pv_read_pending_[hb]) {  // a preview still gathers from this hand-off buffer
      PTTS_HIP(hipStreamWaitEvent(stream_, ev_pv_read_[hb], 0));
      pv_read_pending_[hb] = false;
    }
    if (front && xh_dirty_) refresh_xh();
    if (front) PTTS_HIP(hipGraphLaunch(front, stream_));
    else PTTS_HIP(hipMemsetAsync(flags_[hb], 0, sizeof(FrameFlags) * max_slots_, stream_));
    if (call_ev_from_ >= 0) PTTS_HIP(hipEventRecord(ev_call_[k_ % 4], stream_));
  };
  if (!pipeline_) {
    hipGraphExec_t back = part_graph(1, B, hb, qp, 1);
    run_front_part();
    PTTS_HIP(hipGraphLaunch(back, stream_));
    copy_out(B, hb, stream_);
    out_hb_ = hb;
    out_rows_ = B;
    out_k_ = k_;
  } else if (nfr_ > 1) {
    // Multi-frame passes (nfr = 2 or 4): call k runs front(k) into buffer k % (3 nfr); at k % nfr
    // == 0, k >= nfr, one back pass decodes frames k-nfr .. k-1 (buffers (k-nfr) % (3 nfr) ..) on
    // stream_be_, concurrently with the next fronts. Front(k) waits only for the pass over frame
    // k - 3 nfr, the last reader of its buffer. The call's frame is k - (2 nfr - 1) (its pass was
    // launched by an earlier call; fetch() waits for it).
    const int nf = nfr_, kr = (int)(k_ % nf);
    rows_hb_[hb] = B;
    if (!act_slots_.empty() && kr == 0) {  // rows admitted inside a pass start now
      for (size_t i = 0; i < act_slots_.size(); ++i)
        PTTS_HIP(hipMemcpyAsync(st_ + act_slots_[i], h_act_ + act_slots_[i], sizeof(SlotState), hipMemcpyHostToDevice,
                                stream_));
      PTTS_HIP(hipEventRecord(ev_act_, stream_));
      act_slots_.clear();
    }
    // front(k) overwrites hand-off buffer k % (3 nfr), last read by the pass over frames k - 3 nfr
    // .. k - 2 nfr - 1; the pass's first call waits for that pass, which also read the buffers of
    // the pass's other calls, so they need no wait of their own (stream order). A stream wait
    // costs the front stream ≈ 5 us at the graph boundary even on a completed event (graph
    // stamps, profiles/r04/graph_boundary_ab.txt).
    if (kr == 0) wait_unless_done(stream_, ev_back_[hb]);
    run_front_part();
    launch_previews(B, hb);
    // only the pass's last front part is waited for (by the pass, below)
    if (kr == nf - 1) PTTS_HIP(hipEventRecord(ev_front_[hb], stream_));
    if (kr == 0 && k_ >= nf) {
      const int h0 = (int)((k_ - nf) % nhb_), pq = (int)(((k_ - nf) / nf) & 1);
      // rows: the largest row count of the pass's calls (the first: a call inside a pass covers at
      // most the previous call's rows); nfe: the calls that started frames (the rest were flushes,
      // e.g. a job's drain), the only frames the pass decodes
      int rows = 0, nfe = 0;
      for (int f = 0; f < nf; ++f) {
        const int r = rows_hb_[(h0 + f) % nhb_];
        rows = std::max(rows, r);
        if (r > 0 && nfe == f) nfe = f + 1;
      }
      if (rows > 0) {  // no pass when every call of the pass was a flush
        hipGraphExec_t back = part_graph(1, rows, h0, pq, nfe);
        PTTS_HIP(hipStreamWaitEvent(stream_be_, ev_front_[(h0 + nf - 1) % nhb_], 0));
        if (admit_pending_) {
          PTTS_HIP(hipStreamWaitEvent(stream_be_, ev_admit_, 0));
          admit_pending_ = false;
        }
        PTTS_HIP(hipGraphLaunch(back, stream_be_));
        copy_out(rows, h0, stream_be_);
      }
      PTTS_HIP(hipEventRecord(ev_back_[h0], stream_be_));  // the pass over buffers h0 .. (fetch waits)
    }
    const int lag = 2 * nf - 1;
    out_hb_ = (int)((k_ + nhb_ - lag) % nhb_);
    out_rows_ = k_ >= lag ? rows_hb_[out_hb_] : 0;
    out_k_ = k_ - lag;
  } else {
    const int prev_rows = k_ > 0 ? front_rows_ : B;  // 0: the previous call was a flush
    const int hb1 = (hb + nhb_ - 1) % nhb_, qp1 = qp ^ 1;  // frame k-1
    wait_unless_done(stream_, ev_back_[hb]);
    run_front_part();
    launch_previews(B, hb);
    PTTS_HIP(hipEventRecord(ev_front_[hb], stream_));
    if (prev_rows > 0) {
      hipGraphExec_t back = part_graph(1, prev_rows, hb1, qp1, 1);
      PTTS_HIP(hipStreamWaitEvent(stream_be_, ev_front_[hb1], 0));
      if (admit_pending_) {  // slot state rewritten since the front part this back part decodes
        PTTS_HIP(hipStreamWaitEvent(stream_be_, ev_admit_, 0));
        admit_pending_ = false;
      }
      PTTS_HIP(hipGraphLaunch(back, stream_be_));
      copy_out(prev_rows, hb1, stream_be_);
    }
    PTTS_HIP(hipEventRecord(ev_back_[hb1], stream_be_));
    out_hb_ = hb1;
    out_rows_ = prev_rows;
    out_k_ = k_ - 1;
  }
  front_rows_ = B;
  ++k_;
}

void Engine::sync() {
  PTTS_HIP(hipSetDevice(dev_));
  PTTS_HIP(hipStreamSynchronize(stream_));
  PTTS_HIP(hipStreamSynchronize(stream_be_));
  if (stream_pv_) PTTS_HIP(hipStreamSynchronize(stream_pv_));
}

// Outputs of the last call's frame (see step_async); rows past the rows that frame covered
// report no frame. The step's graphs already copied the frame into pinned host memory.
void Engine::fetch(int B, float* pcm, uint8_t* valid, uint8_t* last, float* eos, float* lat, int calls_back) {
  PTTS_REQUIRE(B >= 1 && B <= max_slots_, "n_rows out of range");
  PTTS_REQUIRE(calls_back == 0 || calls_back == 1, "calls_back must be 0 or 1");
  // the host copies of a call's frame stay intact for two more calls (three hand-off buffers)
  const int q = calls_back ? prev_hb_ : out_hb_;
  const int rows = calls_back ? prev_rows_ : out_rows_;
  const long long fk = calls_back ? prev_k_ : out_k_;  // the call that produced the frame
  // Pipelined: wait only for the back part that produced this call's frame. The front part of
  // the next frame keeps running, so the front stream never idles across calls (the next call's
  // front graph is queued behind it while this one still runs).
  // (multi-frame passes: the pass over buffers nfr p .. records only the event of nfr p)
  if (pipeline_) PTTS_HIP(hipEventSynchronize(ev_back_[q - q % nfr_]));
  else sync();
  const int n = std::min(B, rows);
  if (*h_err_) {  // k_flow_head's bounded hand-off waits: a timeout poisons the frame, fail loudly
    sync();
    *h_err_ = 0;
    PTTS_HIP(hipMemsetAsync(herr_, 0, sizeof(int), stream_));
    // a timed-out launch leaves its hand-off regions part-filled: empty every set again
    if (ffn_hand_) PTTS_HIP(hipMemsetD32Async(ffn_hand_, 0xFFFFFFFFu, 2 * FFN_HAND_FLOATS, stream_));
    PTTS_HIP(hipStreamSynchronize(stream_));
    throw Error(PTTS_ERR_HIP, "persistent launch (FlowLM layers / flow head): an in-launch hand-off wait timed out");
  }
  const float* hl = h_meta_[q];
  const FrameFlags* hf = (const FrameFlags*)(h_meta_[q] + (size_t)max_slots_ * LDIM);
  const float* he = h_meta_[q] + (size_t)max_slots_ * (LDIM + 2);
  // a pass's PCM is [B][nfr][1920] (the frame of buffer q is frame q % nfr)
  auto pcm_row = [&](int b) {
    return nfr_ > 1 ? h_pcmp_[q / nfr_] + ((size_t)b * nfr_ + q % nfr_) * FRAME : h_pcm_[q] + (size_t)b * FRAME;
  };
  for (int b = 0; b < B; ++b) {
    const bool ok = b < n && hf[b].valid;
    // its last frame's pass has completed (waited above) - unless the slot was admitted again
    // after that frame's call (a driver that admits the next utterance before fetching the last
    // frame of the previous one, as bench.py does): then the frame is the previous utterance's and
    // the new one's back passes are still to come
    if (ok && hf[b].last && fk >= admit_call_[b]) drained_[b] = 1;
    if (valid) valid[b] = ok;
    if (last) last[b] = ok && hf[b].last;
    if (pcm) {
      if (b < n) memcpy(pcm + (size_t)b * FRAME, pcm_row(b), sizeof(float) * FRAME);
      else memset(pcm + (size_t)b * FRAME, 0, sizeof(float) * FRAME);
    }
    if (eos) eos[b] = b < n ? he[b] : 0.f;
    if (lat) {
      if (b < n) memcpy(lat + (size_t)b * LDIM, hl + (size_t)b * LDIM, sizeof(float) * LDIM);
      else memset(lat + (size_t)b * LDIM, 0, sizeof(float) * LDIM);
    }
  }
}

bool Engine::front_done(int calls_back, bool wait) {
  PTTS_REQUIRE(calls_back >= 0 && calls_back <= 3, "calls_back must be in [0, 3]");
  const long long k = k_ - 1 - calls_back;
  if (call_ev_from_ < 0) call_ev_from_ = k_;  // the calls issued from now on record their event
  if (k < 0) return true;
  if (k < call_ev_from_) {  // issued before the first query: no event of its own, the stream's state
    if (wait) {
      PTTS_HIP(hipStreamSynchronize(stream_));
      return true;
    }
    const hipError_t r = hipStreamQuery(stream_);
    if (r == hipErrorNotReady) {
      (void)hipGetLastError();
      return false;
    }
    PTTS_HIP(r);
    return true;
  }
  hipEvent_t e = ev_call_[k % 4];
  if (wait) {
    PTTS_HIP(hipEventSynchronize(e));
    return true;
  }
  const hipError_t r = hipEventQuery(e);
  if (r == hipErrorNotReady) {
    (void)hipGetLastError();
    return false;
  }
  PTTS_HIP(r);
  return true;
}

bool Engine::fetch_ready(int calls_back) {
  PTTS_REQUIRE(calls_back == 0 || calls_back == 1, "calls_back must be 0 or 1");
  const int q = calls_back ? prev_hb_ : out_hb_;
  hipError_t r;
  if (pipeline_) {
    r = hipEventQuery(ev_back_[q - q % nfr_]);
  } else {
    r = hipStreamQuery(stream_);
  }
  if (r == hipErrorNotReady) {
    (void)hipGetLastError();
    return false;
  }
  PTTS_HIP(r);
  return true;
}

// GEMM-core test hook: one dense GEMM (mode 0) on the given tile layout, split-K slabs (splits > 1:
// Y receives the [splits][M][N] partial slabs) or the split tail (tail_S > 0, layouts 34 / 35),
// from host operands; the tests compare it with an fp64 product (every shipped layout, shapes the
// model never runs).
void Engine::test_gemm(int layout, int M, int N, int K, int splits, int tail_S, const float* X, const float* Wt,
                       float* Y) {
  xh_dirty_ = true;
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(X && Wt && Y && M >= 1 && N >= 1 && K >= 32 && K % 32 == 0, "test_gemm: bad shape");
  PTTS_REQUIRE(splits >= 1 && splits <= 16 && (splits == 1 || tail_S == 0), "test_gemm: bad split");
  sync();
  const int Nw = (N + 31) / 32 * 32;
  float *dx = nullptr, *dw = nullptr, *dy = nullptr;
  unsigned* dhm = nullptr;  // bf16x6 layouts (>= 200): the split copy of W (split3)
  unsigned short* dlo = nullptr;
  PTTS_HIP(hipMalloc(&dx, sizeof(float) * M * K));
  PTTS_HIP(hipMalloc(&dw, sizeof(float) * Nw * K));
  PTTS_HIP(hipMalloc(&dy, sizeof(float) * splits * M * N));
  if (layout >= 200) {
    PTTS_HIP(hipMalloc(&dhm, sizeof(unsigned) * Nw * K));
    PTTS_HIP(hipMalloc(&dlo, sizeof(unsigned short) * Nw * K));
  }
  auto release = [&]() {
    (void)hipFree(dx), (void)hipFree(dw), (void)hipFree(dy);
    if (dhm) (void)hipFree(dhm);
    if (dlo) (void)hipFree(dlo);
  };
  try {
    PTTS_HIP(hipMemsetAsync(dw, 0, sizeof(float) * Nw * K, stream_));
    PTTS_HIP(hipMemcpyAsync(dx, X, sizeof(float) * M * K, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(dw, Wt, sizeof(float) * N * K, hipMemcpyHostToDevice, stream_));
    if (dhm) split3(dw, (long)Nw * K, dhm, dlo, stream_);
    GemmArgs a{};
    a.mode = 0;
    a.layout = layout;
    a.M = M;
    a.N = N;
    a.K = K;
    a.Nw = Nw;
    a.X = dx;
    a.ldx = K;
    a.W = dw;
    a.Whm = dhm;
    a.Wlo = dlo;
    a.S = splits;
    if (splits > 1) {
      a.partial = dy;
    } else {
      a.Y = dy;
      a.ldy = N;
    }
    if (tail_S > 0) {
      a.tail_S = tail_S;
      a.tail_slab = tslab_;
      a.tail_cap = (long)TAIL_CAP;
      a.tickets = tickets_;
      a.tickets_cap = TICKETS;
    }
    gemm(a, splits, stream_);
    PTTS_HIP(hipGetLastError());
    PTTS_HIP(hipMemcpyAsync(Y, dy, sizeof(float) * splits * M * N, hipMemcpyDeviceToHost, stream_));
    PTTS_HIP(hipStreamSynchronize(stream_));
  } catch (...) {
    (void)hipStreamSynchronize(stream_);
    release();
    throw;
  }
  release();
}

double Engine::time_op(int B, const std::string& name, int reps) {
  xh_dirty_ = true;  // replays write x_ / h_
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(B >= 1 && B <= max_slots_, "n_rows out of range");
  PTTS_REQUIRE(reps >= 1, "reps must be >= 1");
  PTTS_HIP(hipSetDevice(dev_));
  std::vector<Op> ops = build_step(B);
  const Op* sel = nullptr;
  bool back = false, in_back = false;
  for (const Op& op : ops) {
    in_back = in_back || op.name == "mimi.quant_upsample";
    if (op.name == name) sel = &op, back = in_back;
  }
  PTTS_REQUIRE(sel != nullptr, "no op named " + name + " in the step plan");
  // PTTS_TIME_CAP: time back-part ops with the per-CU cap of pipelined stepping
  const bool capped = back && pipeline_ && probe_env("PTTS_TIME_CAP");
  set_wg_cap(capped ? back_cap_ : 0);
  hipEvent_t e0, e1;
  PTTS_HIP(hipEventCreate(&e0));
  PTTS_HIP(hipEventCreate(&e1));
  float ms = 0.f;
  if (sel->prep) {  // each replay behind its own prep: (prep, op) x reps minus prep x reps
    sel->prep(stream_);
    sel->fn(stream_);  // warm
    PTTS_HIP(hipEventRecord(e0, stream_));
    for (int i = 0; i < reps; ++i) {
      sel->prep(stream_);
      sel->fn(stream_);
    }
    PTTS_HIP(hipEventRecord(e1, stream_));
    PTTS_HIP(hipEventSynchronize(e1));
    float both = 0.f, prep = 0.f;
    PTTS_HIP(hipEventElapsedTime(&both, e0, e1));
    PTTS_HIP(hipEventRecord(e0, stream_));
    for (int i = 0; i < reps; ++i) sel->prep(stream_);
    PTTS_HIP(hipEventRecord(e1, stream_));
    PTTS_HIP(hipEventSynchronize(e1));
    PTTS_HIP(hipEventElapsedTime(&prep, e0, e1));
    ms = both - prep;
    sel->prep(stream_);  // leave the op's state as a step finds it (flow.layers: its set empty)
    PTTS_HIP(hipStreamSynchronize(stream_));
  } else {
    sel->fn(stream_);  // warm
    PTTS_HIP(hipEventRecord(e0, stream_));
    for (int i = 0; i < reps; ++i) sel->fn(stream_);
    PTTS_HIP(hipEventRecord(e1, stream_));
    PTTS_HIP(hipEventSynchronize(e1));
    PTTS_HIP(hipEventElapsedTime(&ms, e0, e1));
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  set_wg_cap(0);
  return 1000.0 * ms / reps;
}

// Measurement hook: the step plan split at the FlowLM/flow-head -> Mimi boundary into two graphs;
// times each alone and both launched together on two streams (no dependency, data races are
// irrelevant for timing). us[0] = front alone, us[1] = back alone, us[2] = both concurrently.
void Engine::overlap_probe(int B, int reps, double* us) {
  xh_dirty_ = true;  // replays write x_ / h_
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(B >= 1 && B <= max_slots_ && reps >= 1, "bad probe arguments");
  PTTS_HIP(hipSetDevice(dev_));
  std::vector<Op> ops = build_step(B);
  size_t cut = 0;
  while (cut < ops.size() && ops[cut].name != "mimi.quant_upsample") ++cut;
  PTTS_REQUIRE(cut < ops.size(), "step plan has no Mimi stage");
  hipStream_t s2 = nullptr, s_hi = nullptr, s_lo = nullptr;
  PTTS_HIP(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int prio_lo = 0, prio_hi = 0;
  PTTS_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  PTTS_HIP(hipStreamCreateWithPriority(&s_hi, hipStreamNonBlocking, prio_hi));
  PTTS_HIP(hipStreamCreateWithPriority(&s_lo, hipStreamNonBlocking, prio_lo));
  hipGraphExec_t ge[2] = {};
  hipGraph_t g[2] = {};
  for (int part = 0; part < 2; ++part) {  // as captured for pipelined stepping (back part capped)
    PTTS_HIP(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    set_wg_cap(part == 1 ? back_cap_ : 0);
    for (size_t i = part ? cut : 0; i < (part ? ops.size() : cut); ++i) {
      // each replay of the persistent FlowLM launch needs its hand-off set empty
      if (ops[i].name == "flow.layers") ops[i].prep(stream_);
      ops[i].fn(stream_);
    }
    set_wg_cap(0);
    PTTS_HIP(hipStreamEndCapture(stream_, &g[part]));
    PTTS_HIP(hipGraphInstantiate(&ge[part], g[part], nullptr, nullptr, 0));
  }
  hipEvent_t e0, e1, e2;
  PTTS_HIP(hipEventCreate(&e0));
  PTTS_HIP(hipEventCreate(&e1));
  PTTS_HIP(hipEventCreate(&e2));
  auto timed = [&](int mode) {
    hipStream_t sa = mode == 3 ? s_hi : stream_, sb = mode == 3 ? s_lo : s2;
    for (int w = 0; w < 2; ++w) {
      if (mode != 1) PTTS_HIP(hipGraphLaunch(ge[0], sa));
      if (mode != 0) PTTS_HIP(hipGraphLaunch(ge[1], sb));
    }
    PTTS_HIP(hipStreamSynchronize(sa));
    PTTS_HIP(hipStreamSynchronize(sb));
    PTTS_HIP(hipEventRecord(e0, sa));
    PTTS_HIP(hipStreamWaitEvent(sb, e0, 0));
    for (int r = 0; r < reps; ++r) {
      if (mode != 1) PTTS_HIP(hipGraphLaunch(ge[0], sa));
      if (mode != 0) PTTS_HIP(hipGraphLaunch(ge[1], sb));
    }
    PTTS_HIP(hipEventRecord(e2, sb));
    PTTS_HIP(hipStreamWaitEvent(sa, e2, 0));
    PTTS_HIP(hipEventRecord(e1, sa));
    PTTS_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    PTTS_HIP(hipEventElapsedTime(&ms, e0, e1));
    return 1000.0 * ms / reps;
  };
  // us[7]: front || Mimi transformer || SEANet decoder on three streams (a 3-stage pipeline)
  if (probe_env("PTTS_PROBE_MODES") && strchr(probe_env("PTTS_PROBE_MODES"), '7')) {
    size_t cut2 = cut;
    while (cut2 < ops.size() && ops[cut2].name != "seanet.conv0") ++cut2;
    hipGraphExec_t g3[2] = {};
    hipGraph_t d3[2] = {};
    for (int part = 0; part < 2; ++part) {
      PTTS_HIP(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
      set_wg_cap(back_cap_);
      for (size_t i = part ? cut2 : cut; i < (part ? ops.size() : cut2); ++i) ops[i].fn(stream_);
      set_wg_cap(0);
      PTTS_HIP(hipStreamEndCapture(stream_, &d3[part]));
      PTTS_HIP(hipGraphInstantiate(&g3[part], d3[part], nullptr, nullptr, 0));
    }
    hipStream_t s3 = nullptr;
    PTTS_HIP(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    hipEvent_t a0, a1, a2, a3;
    PTTS_HIP(hipEventCreate(&a0));
    PTTS_HIP(hipEventCreate(&a1));
    PTTS_HIP(hipEventCreate(&a2));
    PTTS_HIP(hipEventCreate(&a3));
    auto run3 = [&](int n) {
      for (int r = 0; r < n; ++r) {
        PTTS_HIP(hipGraphLaunch(ge[0], stream_));
        PTTS_HIP(hipGraphLaunch(g3[0], s2));
        PTTS_HIP(hipGraphLaunch(g3[1], s3));
      }
    };
    run3(2);
    PTTS_HIP(hipDeviceSynchronize());
    PTTS_HIP(hipEventRecord(a0, stream_));
    PTTS_HIP(hipStreamWaitEvent(s2, a0, 0));
    PTTS_HIP(hipStreamWaitEvent(s3, a0, 0));
    run3(reps);
    PTTS_HIP(hipEventRecord(a2, s2));
    PTTS_HIP(hipEventRecord(a3, s3));
    PTTS_HIP(hipStreamWaitEvent(stream_, a2, 0));
    PTTS_HIP(hipStreamWaitEvent(stream_, a3, 0));
    PTTS_HIP(hipEventRecord(a1, stream_));
    PTTS_HIP(hipEventSynchronize(a1));
    float ms = 0.f;
    PTTS_HIP(hipEventElapsedTime(&ms, a0, a1));
    us[7] = 1000.0 * ms / reps;
    for (hipEvent_t e : {a0, a1, a2, a3}) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(s3);
    for (int part = 0; part < 2; ++part) {
      (void)hipGraphExecDestroy(g3[part]);
      (void)hipGraphDestroy(d3[part]);
    }
  }
  // PTTS_PROBE_MODES: digits of the measurements to run (default all: "0123456")
  const std::string modes = probe_env("PTTS_PROBE_MODES") ? probe_env("PTTS_PROBE_MODES") : "0123456";
  auto want = [&](int m) { return modes.find((char)('0' + m)) != std::string::npos; };
  for (int m = 0; m < 7; ++m) us[m] = -1.0;  // us[7]: see above
  for (int m = 0; m < 4; ++m)
    if (want(m)) us[m] = timed(m);
  // us[4..6]: front graph || back part launched op by op on a stream whose CU mask keeps
  // 8/8, 6/8, 4/8 of the CUs (graph launches do not honour a stream's CU mask)
  for (int v = 0; v < 3; ++v) {
    if (!want(4 + v)) continue;
    const int keep = 8 - 2 * v;
    std::vector<uint32_t> mask(8, 0u);  // 256 CUs
    for (int cu = 0; cu < 256; ++cu)
      if ((cu % 8) < keep) mask[cu / 32] |= 1u << (cu % 32);
    hipStream_t sm = nullptr;
    PTTS_HIP(hipExtStreamCreateWithCUMask(&sm, (uint32_t)mask.size(), mask.data()));
    auto back_eager = [&]() {  // capped as in pipelined stepping: the persistent flow-head launch of
      set_wg_cap(back_cap_);    // the concurrent front graph needs room for all its workgroups
      for (size_t i = cut; i < ops.size(); ++i) ops[i].fn(sm);
      set_wg_cap(0);
    };
    for (int w = 0; w < 2; ++w) {
      PTTS_HIP(hipGraphLaunch(ge[0], stream_));
      back_eager();
    }
    PTTS_HIP(hipStreamSynchronize(stream_));
    PTTS_HIP(hipStreamSynchronize(sm));
    PTTS_HIP(hipEventRecord(e0, stream_));
    PTTS_HIP(hipStreamWaitEvent(sm, e0, 0));
    for (int r = 0; r < reps; ++r) {
      PTTS_HIP(hipGraphLaunch(ge[0], stream_));
      back_eager();
    }
    PTTS_HIP(hipEventRecord(e2, sm));
    PTTS_HIP(hipStreamWaitEvent(stream_, e2, 0));
    PTTS_HIP(hipEventRecord(e1, stream_));
    PTTS_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    PTTS_HIP(hipEventElapsedTime(&ms, e0, e1));
    us[4 + v] = 1000.0 * ms / reps;
    (void)hipStreamDestroy(sm);
  }
  // PTTS_PROBE_SPLITS="F:K,...": spatial partition. The front part launched op by op on a stream
  // whose CU mask keeps the CUs with cu % 8 < F, the back part op by op on the CUs with
  // cu % 8 >= 8 - K (disjoint when F + K <= 8); F or K = 0 leaves that part out (alone timings).
  // One line per split on stderr: microseconds per step (front + back per call).
  if (probe_env("PTTS_PROBE_SPLITS")) {
    auto make_masked = [&](int lo, int hi) {  // CUs with lo <= cu % 8 < hi
      std::vector<uint32_t> m(8, 0u);
      for (int cu = 0; cu < 256; ++cu)
        if ((cu % 8) >= lo && (cu % 8) < hi) m[cu / 32] |= 1u << (cu % 32);
      hipStream_t st = nullptr;
      PTTS_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data()));
      return st;
    };
    const std::string spec = probe_env("PTTS_PROBE_SPLITS");
    size_t p = 0;
    while (p < spec.size()) {
      size_t q = spec.find(',', p);
      if (q == std::string::npos) q = spec.size();
      const std::string item = spec.substr(p, q - p);
      p = q + 1;
      // the back side may be a stand-in on the other CUs: "F:eN" N empty launches per step, "F:mN"
      // one copy kernel moving N MB (read + write) per step
      const std::string bs = item.substr(item.find(':') + 1);
      const char kind = bs.empty() ? '0' : bs[0];
      const bool dummy = kind == 'e' || kind == 'm';
      const int F = atoi(item.c_str()), K = dummy ? 8 - F : atoi(bs.c_str()), N = dummy ? atoi(bs.c_str() + 1) : 0;
      float* big = nullptr;
      if (kind == 'm') PTTS_HIP(hipMalloc(&big, (size_t)N << 20));
      fprintf(stderr, "split %d:%s: streams\n", F, bs.c_str());
      hipStream_t sf = F > 0 ? make_masked(0, F) : nullptr, sb = K > 0 ? make_masked(8 - K, 8) : nullptr;
      fprintf(stderr, "split %d:%s: warm\n", F, bs.c_str());
      auto one = [&]() {
        if (sf)
          for (size_t i = 0; i < cut; ++i) ops[i].fn(sf);
        if (sb && kind == 'e') {
          for (int i = 0; i < N; ++i) copy2d(x_, 1, q_, 1, 1, 1, sb);
        } else if (sb && kind == 'm') {
          const long half = ((long)N << 20) / 8;  // floats copied: N/2 MB read + N/2 MB written
          copy2d(big, 1024, big + half, 1024, (int)(half / 1024), 1024, sb);
        } else if (sb) {
          set_wg_cap(back_cap_);
          for (size_t i = cut; i < ops.size(); ++i) ops[i].fn(sb);
          set_wg_cap(0);
        }
      };
      for (int w = 0; w < 2; ++w) one();
      PTTS_HIP(hipDeviceSynchronize());
      hipStream_t s0 = sf ? sf : sb, s1 = sb ? sb : sf;
      PTTS_HIP(hipEventRecord(e0, s0));
      PTTS_HIP(hipStreamWaitEvent(s1, e0, 0));
      for (int r = 0; r < reps; ++r) one();
      PTTS_HIP(hipEventRecord(e2, s1));
      PTTS_HIP(hipStreamWaitEvent(s0, e2, 0));
      PTTS_HIP(hipEventRecord(e1, s0));
      PTTS_HIP(hipEventSynchronize(e1));
      float ms = 0.f;
      PTTS_HIP(hipEventElapsedTime(&ms, e0, e1));
      fprintf(stderr, "split front %d/8 back %d/8 (%s): %.1f us per step\n", F, K, dummy ? bs.c_str() : "ops",
              1000.0 * ms / reps);
      if (sf) (void)hipStreamDestroy(sf);
      if (sb) (void)hipStreamDestroy(sb);
      if (big) (void)hipFree(big);
    }
  }
  for (int part = 0; part < 2; ++part) {
    (void)hipGraphExecDestroy(ge[part]);
    (void)hipGraphDestroy(g[part]);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipEventDestroy(e2);
  (void)hipStreamDestroy(s2);
  (void)hipStreamDestroy(s_hi);
  (void)hipStreamDestroy(s_lo);
}

// ------------------------------------------------------------------ voices and slots
ptts_voice* Engine::voice_from_prompt(const float* prompt, int F) {
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(prompt != nullptr && F >= 1, "empty prompt");
  PTTS_REQUIRE(F < max_ctx_, "prompt longer than max_ctx");
  sync();
  const int scratch = max_slots_;
  for (int c0 = 0; c0 < F; c0 += PREFILL) {
    const int T = std::min(PREFILL, F - c0);
    PTTS_HIP(hipMemcpyAsync(x_, prompt + (size_t)c0 * D, sizeof(float) * T * D, hipMemcpyHostToDevice, stream_));
    std::vector<Op> ops;
    prefill_rows(ops, scratch, T, c0);
    run_ops(ops);
  }
  ptts_voice* v = new ptts_voice();
  v->F = F;
  v->owner = this;
  try {
    PTTS_HIP(hipMalloc(&v->kv, sizeof(float) * (size_t)NL * 2 * NH * F * 64));
    PTTS_HIP(hipMemcpy2DAsync(v->kv, sizeof(float) * F * 64, kv_ + (size_t)scratch * kv_slot_,
                              sizeof(float) * max_ctx_ * 64, sizeof(float) * F * 64, NL * 2 * NH,
                              hipMemcpyDeviceToDevice, stream_));
    PTTS_HIP(hipStreamSynchronize(stream_));
  } catch (...) {
    if (v->kv) (void)hipFree(v->kv);
    delete v;
    throw;
  }
  return v;
}

void Engine::encoder_transformer(std::vector<Op>& ops, float* x, int T, float* h, float* qkv, float* q, float* o,
                                 float* u, float* ring) {
  RowMap map{0, T, 0, nullptr};
  {
    const float *w = W(L_.menc[0].n1w), *b = W(L_.menc[0].n1b);
    ops.push_back({"enc.ln1", [=](hipStream_t s) { layernorm(x, MD, h, MD, T, MD, w, b, 1e-5f, s); }});
  }
  for (int l = 0; l < MNL; ++l) {
    const Layout::TL& t = L_.menc[l];
    KvStore kv{ring + (size_t)l * 2 * MNH * T * 64, 0, T};
    dense_op(ops, "enc.qkv", h, T, W(t.in_proj), 3 * MD, MD, nullptr, ACT_NONE, nullptr, nullptr, qkv);
    ops.push_back({"enc.rope", [=](hipStream_t s) { qkv_rope_append(nullptr, 0, qkv, T, MNH, map, kv, q, s); }});
    ops.push_back({"enc.attn", [=](hipStream_t s) { attention(q, T, MNH, map, kv, MCTX, 16, o, s); }});
    dense_op(ops, "enc.out", o, T, W(t.out_proj), MD, MD, nullptr, ACT_NONE, W(t.ls1), x, x);
    {
      const float *w = W(t.n2w), *b = W(t.n2b);
      ops.push_back({"enc.ln2", [=](hipStream_t s) { layernorm(x, MD, h, MD, T, MD, w, b, 1e-5f, s); }});
    }
    dense_op(ops, "enc.ff1", h, T, W(t.l1), MFF, MD, nullptr, ACT_GELU, nullptr, nullptr, u);
    dense_op(ops, "enc.ff2", u, T, W(t.l2), MD, MFF, nullptr, ACT_NONE, W(t.ls2), x, x);
    if (l + 1 < MNL) {
      const float *w = W(L_.menc[l + 1].n1w), *b = W(L_.menc[l + 1].n1b);
      ops.push_back({"enc.ln1", [=](hipStream_t s) { layernorm(x, MD, h, MD, T, MD, w, b, 1e-5f, s); }});
    }
  }
}

namespace {
// adaptive_voice_prompt_chunk_frames (tts_model.rs:562-577); override > 0 wins, < 0 = one pass.
int voice_chunk_frames(int F, int override_frames) {
  if (override_frames > 0) return override_frames;
  if (override_frames < 0 || F <= 120) return std::max(F, 1);
  if (F <= 600) return 120;
  if (F <= 1800) return 180;
  return 240;
}
}  // namespace

// The GPU resampler on its own (test hook of the voice front end): the resample_poly rule, or the
// Rust driver's rubato FastFixedIn / Septic (kernels.h septic_schedule). Equal rates copy the input,
// as audio.rs:198-200 returns the tensor unchanged.
void Engine::resample_host(const float* x, int n, int sr_from, int sr_to, float* y, int resampler) {
  PTTS_REQUIRE(x && y && n >= 1, "empty input");
  PTTS_REQUIRE(sr_from > 0 && sr_to > 0, "sample rates must be positive");
  PTTS_REQUIRE(resampler == PTTS_RESAMPLE_POLY || resampler == PTTS_RESAMPLE_RUBATO_SEPTIC, "unknown resampler");
  const bool septic = resampler == PTTS_RESAMPLE_RUBATO_SEPTIC && sr_from != sr_to;
  const ResamplePlan rp = resample_plan(sr_from, sr_to);
  std::vector<int> st;
  std::vector<float> fr;
  const long n_out = septic ? septic_schedule(n, sr_from, sr_to, &st, &fr) : sr_from == sr_to ? n : rp.out_len(n);
  PTTS_REQUIRE(n_out >= 1, "input too short for the resampler (no output samples)");
  PTTS_REQUIRE(rp.L <= (1 << 22) && n_out < (1L << 30), "resampling ratio or length too large");
  sync();
  std::vector<float> taps;
  if (!septic && sr_from != sr_to) taps = resample_taps(rp);
  void *dx = nullptr, *dh = nullptr, *dy = nullptr, *ds = nullptr;
  try {
    PTTS_HIP(hipMalloc(&dx, sizeof(float) * n));
    PTTS_HIP(hipMalloc(&dy, sizeof(float) * n_out));
    PTTS_HIP(hipMemcpyAsync(dx, x, sizeof(float) * n, hipMemcpyHostToDevice, stream_));
    if (sr_from == sr_to) {
      PTTS_HIP(hipMemcpyAsync(dy, dx, sizeof(float) * n, hipMemcpyDeviceToDevice, stream_));
    } else if (septic) {
      PTTS_HIP(hipMalloc(&ds, sizeof(int) * n_out));
      PTTS_HIP(hipMalloc(&dh, sizeof(float) * n_out));
      PTTS_HIP(hipMemcpyAsync(ds, st.data(), sizeof(int) * n_out, hipMemcpyHostToDevice, stream_));
      PTTS_HIP(hipMemcpyAsync(dh, fr.data(), sizeof(float) * n_out, hipMemcpyHostToDevice, stream_));
      resample_septic((const float*)dx, n, (const int*)ds, (const float*)dh, (int)n_out, (int)n_out, (float*)dy,
                      stream_);
    } else {
      PTTS_HIP(hipMalloc(&dh, sizeof(float) * taps.size()));
      PTTS_HIP(hipMemcpyAsync(dh, taps.data(), sizeof(float) * taps.size(), hipMemcpyHostToDevice, stream_));
      resample((const float*)dx, n, (const float*)dh, rp, (int)n_out, (int)n_out, (float*)dy, stream_);
    }
    PTTS_HIP(hipGetLastError());
    PTTS_HIP(hipMemcpyAsync(y, dy, sizeof(float) * n_out, hipMemcpyDeviceToHost, stream_));
    PTTS_HIP(hipStreamSynchronize(stream_));
  } catch (...) {
    (void)hipStreamSynchronize(stream_);
    (void)hipFree(dx), (void)hipFree(dh), (void)hipFree(dy), (void)hipFree(ds);
    throw;
  }
  (void)hipFree(dx), (void)hipFree(dh), (void)hipFree(dy), (void)hipFree(ds);
}

// Voice cloning (tts_model.rs:428-577): samples at `sr` -> resampled to 24 kHz on the GPU
// (resample_poly rule, kernels.h) -> zero-padded to whole frames (tts_model.rs:515-527) -> Mimi
// encoder (mimi.rs:113-141) -> speaker projection (:543-553) -> FlowLM prompt prefill (:580-599).
// The reference encodes chunk by chunk (adaptive chunk length, :530-541) with step=0 for every
// chunk: the streaming convs and the encoder transformer carry their state, which equals the
// single pass below, but ConvDownsample1d re-applies its replicate padding at each chunk's first
// frame (conv.rs:116-123); the downsample conv is therefore run per chunk.
ptts_voice* Engine::voice_from_audio(const float* pcm_in, int n_in, int sr, int chunk_frames, int resampler) {
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(pcm_in != nullptr && n_in >= 1, "empty PCM");
  PTTS_REQUIRE(sr > 0, "sample rate must be positive");
  PTTS_REQUIRE(resampler == PTTS_RESAMPLE_POLY || resampler == PTTS_RESAMPLE_RUBATO_SEPTIC, "unknown resampler");
  const ResamplePlan rp = resample_plan(sr, PTTS_SAMPLE_RATE);
  const bool septic = resampler == PTTS_RESAMPLE_RUBATO_SEPTIC && !rp.identity();
  std::vector<int> sst;  // rubato position schedule (host copies outlive the async uploads)
  std::vector<float> sfr;
  const long n_long = rp.identity() ? n_in : septic ? septic_schedule(n_in, sr, PTTS_SAMPLE_RATE, &sst, &sfr)
                                                    : rp.out_len(n_in);
  PTTS_REQUIRE(n_long >= 1 && n_long < (1L << 28) && rp.L <= (1 << 22), "voice prompt length or rate out of range");
  const int n = (int)n_long;
  sync();
  const int Np = (n + FRAME - 1) / FRAME * FRAME;  // zero-pad to whole frames (mimi.py:103)
  const int F = Np / FRAME, Te = Np / 120;
  PTTS_REQUIRE(F < max_ctx_, "voice prompt longer than max_ctx");
  const int cf = voice_chunk_frames(F, chunk_frames);
  std::vector<void*> tmp;
  auto talloc = [&](size_t cnt) {
    void* p = nullptr;
    PTTS_HIP(hipMalloc(&p, std::max<size_t>(cnt, 1) * sizeof(float)));
    tmp.push_back(p);
    return (float*)p;
  };
  ptts_voice* v = nullptr;
  try {
    float* dpcm = talloc(Np);
    float* A = talloc((size_t)Np * 64);
    float* Bf = talloc((size_t)Np * 64);
    float* V = talloc((size_t)Np * 32);
    float* zeros = talloc(16 * 512);
    PTTS_HIP(hipMemsetAsync(zeros, 0, sizeof(float) * 16 * 512, stream_));
    std::vector<float> taps;  // host copy must outlive the async upload
    if (rp.identity()) {
      PTTS_HIP(hipMemsetAsync(dpcm, 0, sizeof(float) * Np, stream_));
      PTTS_HIP(hipMemcpyAsync(dpcm, pcm_in, sizeof(float) * n, hipMemcpyHostToDevice, stream_));
    } else if (septic) {  // the Rust driver's resampler, straight into the frame-padded input
      float* dx = talloc(n_in);
      int* ds = (int*)talloc(n);
      float* df = talloc(n);
      PTTS_HIP(hipMemcpyAsync(dx, pcm_in, sizeof(float) * n_in, hipMemcpyHostToDevice, stream_));
      PTTS_HIP(hipMemcpyAsync(ds, sst.data(), sizeof(int) * n, hipMemcpyHostToDevice, stream_));
      PTTS_HIP(hipMemcpyAsync(df, sfr.data(), sizeof(float) * n, hipMemcpyHostToDevice, stream_));
      resample_septic(dx, n_in, ds, df, n, Np, dpcm, stream_);
      PTTS_HIP(hipGetLastError());
    } else {  // resample straight into the frame-padded encoder input (zeros past n)
      taps = resample_taps(rp);
      float* dx = talloc(n_in);
      float* dh = talloc(taps.size());
      PTTS_HIP(hipMemcpyAsync(dx, pcm_in, sizeof(float) * n_in, hipMemcpyHostToDevice, stream_));
      PTTS_HIP(hipMemcpyAsync(dh, taps.data(), sizeof(float) * taps.size(), hipMemcpyHostToDevice, stream_));
      resample(dx, n_in, dh, rp, n, Np, dpcm, stream_);
      PTTS_HIP(hipGetLastError());
    }
    std::vector<Op> ops;
    {
      const float *w = W(L_.ec0_w), *b = W(L_.ec0_b);
      ops.push_back({"enc.conv0", [=](hipStream_t s) { conv_cin1(dpcm, Np, 64, 7, w, b, A, s); }});
    }
    int T = Np, ch = 64;
    for (int i = 0; i < 3; ++i) {
      const int r = RATIOS[2 - i];
      conv_op(ops, "enc.res_conv3", A, 1, T, ch, zeros, 2, 1, 1, W(L_.era_w[i]), ch / 2, 3, 1, W(L_.era_b[i]),
              nullptr, V, T, 1);
      conv_op(ops, "enc.res_conv1", V, 1, T, ch / 2, nullptr, 0, 1, 1, W(L_.erb_w[i]), ch, 1, 1, W(L_.erb_b[i]), A,
              Bf, T, 1);
      conv_op(ops, "enc.down", Bf, 1, T, ch, zeros, r, r, 1, W(L_.edn_w[i]), 2 * ch, 2 * r, 1, W(L_.edn_b[i]),
              nullptr, A, T / r, 1);
      T /= r;
      ch *= 2;
    }
    conv_op(ops, "enc.conv_final", A, 1, T, 512, zeros, 2, 1, 1, W(L_.efin_w), 512, 3, 1, W(L_.efin_b), nullptr, Bf,
            T, 1);
    // encoder transformer on Bf rows [Te][512]
    float* h = talloc((size_t)Te * MD);
    float* qkv = talloc((size_t)Te * 3 * MD);
    float* q = talloc((size_t)Te * MD);
    float* o = talloc((size_t)Te * MD);
    float* u = talloc((size_t)Te * MFF);
    float* ring = talloc((size_t)MNL * 2 * MNH * Te * 64);
    encoder_transformer(ops, Bf, Te, h, qkv, q, o, u, ring);
    // ConvDownsample1d k32 s16 per chunk of cf frames, each with the replicate padding of its first
    // frame (conv.rs:116-123): full chunks run as one batched implicit GEMM (chunk = batch row,
    // history = that chunk's replicated first row), a shorter last chunk as a second launch.
    const int nfull = F / cf, rem = F - nfull * cf, nch = nfull + (rem ? 1 : 0);
    float* Hd = talloc((size_t)nch * 16 * 512);
    for (int c = 0; c < nch; ++c) {
      const float* src = Bf + (size_t)c * cf * 16 * 512;
      float* dst = Hd + (size_t)c * 16 * 512;
      ops.push_back({"enc.replicate", [=](hipStream_t s) { copy2d(src, 0, dst, 512, 16, 512, s); }});
    }
    float* lat = talloc((size_t)F * 512);
    if (nfull)
      conv_op(ops, "enc.downsample", Bf, nfull, cf * 16, 512, Hd, 16, 16, 0, W(L_.down_w), 512, 32, 1, nullptr,
              nullptr, lat, cf, 1);
    if (rem)
      conv_op(ops, "enc.downsample", Bf + (size_t)nfull * cf * 16 * 512, 1, rem * 16, 512,
              Hd + (size_t)nfull * 16 * 512, 16, 16, 0, W(L_.down_w), 512, 32, 1, nullptr, nullptr,
              lat + (size_t)nfull * cf * 512, rem, 1);
    float* cond = talloc((size_t)F * D);
    dense_op(ops, "enc.speaker_proj", lat, F, W(L_.speaker_proj), D, MD, nullptr, ACT_NONE, nullptr, nullptr, cond);
    run_ops(ops);
    std::vector<float> hcond((size_t)F * D);
    PTTS_HIP(hipMemcpyAsync(hcond.data(), cond, sizeof(float) * hcond.size(), hipMemcpyDeviceToHost, stream_));
    PTTS_HIP(hipStreamSynchronize(stream_));
    for (void* p : tmp) (void)hipFree(p);
    tmp.clear();
    v = voice_from_prompt(hcond.data(), F);
    v->cond = std::move(hcond);
  } catch (...) {
    (void)hipStreamSynchronize(stream_);
    for (void* p : tmp) (void)hipFree(p);
    throw;
  }
  return v;
}

void Engine::slot_open(int slot, const ptts_voice* v, const int32_t* ids, int n, const ptts_gen_params& p) {
  slots_open(1, &slot, &v, ids, &n, &p);
}

// Batched admission: the per-segment prologue of generate_stream_segment (tts_model.rs:938-1004)
// for n utterances at once. Voice KV prefixes are copied in (copy-on-admit, tts_model.rs:940),
// Mimi/conv state reset, and all utterances' text tokens are prefilled together: rows are laid out
// per slot, padded to 16-row groups (the 16-query attention tiles), and mapped to (slot, position)
// through a row table.
void Engine::slots_open(int n, const int* slots, const ptts_voice* const* voices, const int32_t* ids,
                        const int* n_ids, const ptts_gen_params* params) {
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(n >= 1 && n <= max_slots_, "number of admissions out of range");
  PTTS_REQUIRE(slots && voices && n_ids && params, "null argument");
  std::vector<char> seen(max_slots_, 0);
  long total_ids = 0;
  for (int i = 0; i < n; ++i) {
    const int slot = slots[i];
    PTTS_REQUIRE(slot >= 0 && slot < max_slots_, "slot out of range");
    PTTS_REQUIRE(!seen[slot], "slot admitted twice in one call");
    seen[slot] = 1;
    const ptts_voice* v = voices[i];
    PTTS_REQUIRE(v != nullptr && v->owner == this, "voice belongs to another engine");
    const ptts_gen_params& p = params[i];
    PTTS_REQUIRE(n_ids[i] >= 0 && (n_ids[i] == 0 || ids != nullptr), "bad token ids");
    PTTS_REQUIRE(p.max_frames >= 1, "max_frames must be >= 1");
    PTTS_REQUIRE(p.frames_after_eos >= 0, "frames_after_eos must be >= 0");
    PTTS_REQUIRE((long)v->F + n_ids[i] + p.max_frames <= max_ctx_, "voice + text + max_frames exceeds max_ctx");
    for (int j = 0; j < n_ids[i]; ++j)
      PTTS_REQUIRE(ids[total_ids + j] >= 0 && ids[total_ids + j] < VOCAB, "token id out of range");
    total_ids += n_ids[i];
  }
  // Stream-ordered admission (no drain of the pipeline: a full sync() here stalled the front part
  // at every admission, a large share of the serving path's time): the host waits only until the
  // previous admission has consumed the pinned staging buffers (its event), and stream_ waits on
  // the GPU for the back parts already queued on stream_be_ (which may still decode a frame of a
  // slot's previous utterance: they write its histories and Mimi position) only before the reset
  // of that state, after the text prefill.
  PTTS_HIP(hipEventSynchronize(ev_admit_));
  PTTS_HIP(hipEventSynchronize(ev_act_));  // pending start-of-utterance copies read h_act_
  if (share_voice_) {
    // shared voice prefixes: each slot's positions < F read the voice's own cache (no copy; the
    // reference copies the prompt's ModelState per utterance, tts_model.rs:940: same values)
    {
      std::lock_guard<std::mutex> lk(voice_mu());
      for (int i = 0; i < n; ++i) ++voices[i]->refs;
    }
    for (int i = 0; i < n; ++i) voice_release(slots[i], false);
    for (int i = 0; i < n; ++i) {
      slot_voice_[slots[i]] = voices[i];
      h_vpre_[slots[i]] = voices[i]->kv;
      h_vlen_[slots[i]] = voices[i]->F;
    }
    // the tables are read by the text prefill below and by the steps after it (stream order); the
    // steps queued before still read the old entries (a freed voice waited for them above)
    PTTS_HIP(hipMemcpyAsync(vpre_, h_vpre_, sizeof(float*) * max_slots_, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(vlen_, h_vlen_, sizeof(int) * max_slots_, hipMemcpyHostToDevice, stream_));
  } else {
    // copy-on-admit of the immutable voice prefixes
    for (int i = 0; i < n; ++i) {
      const ptts_voice* v = voices[i];
      PTTS_HIP(hipMemcpy2DAsync(kv_ + (size_t)slots[i] * kv_slot_, sizeof(float) * max_ctx_ * 64, v->kv,
                                sizeof(float) * v->F * 64, sizeof(float) * v->F * 64, NL * 2 * NH,
                                hipMemcpyDeviceToDevice, stream_));
    }
  }
  // text prefill (tts_model.rs:947-964) of every admitted utterance in shared passes
  std::vector<int> tab, rid;
  long off = 0;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < n_ids[i]; ++j) {
      tab.push_back(slots[i] << 16 | (voices[i]->F + j));
      rid.push_back(ids[off + j]);
    }
    while (tab.size() % 16) {
      tab.push_back(-1);
      rid.push_back(0);
    }
    off += n_ids[i];
  }
  // The GEMMs, reduces and RoPE run on the tokens only (Tc compact rows: 40 tokens are 40 rows, not
  // 48); the attention keeps the slot-aligned 16-row groups (RowMap::ptab / qrow / orow)
  for (size_t c0 = 0; c0 < tab.size(); c0 += PREFILL) {
    const int T = (int)std::min<size_t>(PREFILL, tab.size() - c0);  // PREFILL % 16 == 0
    if (c0 > 0) PTTS_HIP(hipStreamSynchronize(stream_));  // ids / row table / staging reused by this pass
    int* h_ptab = h_tab_;
    int* h_ctab = h_tab_ + PREFILL;
    int* h_qrow = h_tab_ + 2 * PREFILL;
    int* h_orow = h_tab_ + 3 * PREFILL;
    int Tc = 0;
    for (int r = 0; r < T; ++r) {
      const int v = tab[c0 + r];
      h_ptab[r] = v;
      h_orow[r] = v < 0 ? -1 : Tc;
      if (v >= 0) {
        h_ctab[Tc] = v;
        h_qrow[Tc] = r;
        h_ids_[Tc] = rid[c0 + r];
        ++Tc;
      }
    }
    if (Tc == 0) continue;
    PTTS_HIP(hipMemcpyAsync(ids_dev_, h_ids_, sizeof(int) * Tc, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(rowtab_dev_, h_ptab, sizeof(int) * T, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(ctab_dev_, h_ctab, sizeof(int) * Tc, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(qrow_dev_, h_qrow, sizeof(int) * Tc, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(orow_dev_, h_orow, sizeof(int) * T, hipMemcpyHostToDevice, stream_));
    std::vector<Op> ops;
    {
      const int* idp = ids_dev_;
      const float* tb = W(L_.embed);
      float* x = x_;
      ops.push_back({"prefill.embed", [=](hipStream_t s) { embed_gather(idp, Tc, tb, D, x, s); }});
    }
    {
      float* x = x_;
      float* h = h_;
      const float* w = W(L_.fl[0].n1w);
      const float* b = W(L_.fl[0].n1b);
      ops.push_back({"prefill.ln1", [=](hipStream_t s) { layernorm(x, D, h, D, Tc, D, w, b, 1e-5f, s); }});
    }
    RowMap map{0, 1, 0, nullptr, ctab_dev_};
    map.ptab = rowtab_dev_;
    map.mpad = T;
    map.qrow = qrow_dev_;
    map.orow = orow_dev_;
    flow_layers(ops, Tc, map, 16, false, "prefill");
    run_ops(ops);
  }
  // the slot state the back part owns (Mimi ring position, conv and overlap-add histories, frame
  // flags) is reset only after the back parts already queued, which may still decode the slot's
  // previous utterance; the voice-KV copy and the text prefill above touch front-owned state
  // only, so they run ahead of that wait, beside those back parts
  // That wait is needed only while an admitted slot may still have a frame in flight: a slot whose
  // utterance is drained (never admitted, closed, or its last frame fetched) is written by no
  // queued back part (the commit and the histories touch rows with a frame only), so the front
  // stream does not stall behind the queued back passes at such an admission (the server's case)
  bool drained = true;
  for (int i = 0; i < n; ++i) drained = drained && drained_[slots[i]];
  if (!drained) {
    PTTS_HIP(hipEventRecord(ev_be_tail_, stream_be_));
    PTTS_HIP(hipStreamWaitEvent(stream_, ev_be_tail_, 0));
  }
  for (int i = 0; i < n; ++i) {
    drained_[slots[i]] = 0;
    admit_call_[slots[i]] = k_;
  }
  // fresh Mimi decoder state (init_states(1, 1000) per segment, tts_model.rs:941) + slot states
  std::vector<SlotState> st(n);
  std::vector<int> fp(n);
  for (int i = 0; i < n; ++i) {
    const ptts_gen_params& p = params[i];
    SlotState& s = st[i];
    s = SlotState{};
    s.active = 1;
    s.step = 0;
    s.eos_step = -1;
    s.frames_after_eos = p.frames_after_eos;
    s.max_frames = p.max_frames;
    s.temp = p.temp;
    s.eos_threshold = p.eos_threshold;
    s.noise_clamp = p.noise_clamp;
    s.seed = p.seed;
    fp[i] = voices[i]->F + n_ids[i];
  }
  // staged through pinned buffers so the copies are truly asynchronous: admission returns with
  // the prefill still running and the caller's first step queued right behind it (no host
  // round trip in between); the event wait above guarantees the staging is free again
  // multi-frame passes: an utterance's frames group into passes from its first, so rows admitted
  // inside a pass stay inactive for the pass's remaining calls and start at the next pass (their
  // state is written then)
  admit_delay_ = nfr_ > 1 ? (int)((nfr_ - k_ % nfr_) % nfr_) : 0;
  if (admit_delay_)
    for (int i = 0; i < n; ++i) {
      h_act_[slots[i]] = st[i];
      act_slots_.push_back(slots[i]);
      st[i].active = 0;
    }
  // first-frame previews: each admitted row's first front part runs at call k_ + admit_delay_ (a
  // re-admitted slot's unfetched preview belonged to its previous utterance)
  for (int i = 0; i < n; ++i) pv_forget(slots[i]);
  if (pv_max_ > 0)
    for (int i = 0; i < n; ++i) pv_pending_.push_back({slots[i], k_ + admit_delay_});
  memcpy(h_slots_, slots, sizeof(int) * n);
  memcpy(h_st_, st.data(), sizeof(SlotState) * n);
  memcpy(h_fp_, fp.data(), sizeof(int) * n);
  PTTS_HIP(hipMemcpyAsync(admit_slots_, h_slots_, sizeof(int) * n, hipMemcpyHostToDevice, stream_));
  PTTS_HIP(hipMemcpyAsync(admit_st_, h_st_, sizeof(SlotState) * n, hipMemcpyHostToDevice, stream_));
  PTTS_HIP(hipMemcpyAsync(admit_fpos_, h_fp_, sizeof(int) * n, hipMemcpyHostToDevice, stream_));
  {
    ResetArgs r{};
    for (int i = 0; i < 8; ++i) {
      r.buf[i] = hist_[i];
      r.per_slot[i] = (long)hist_P_[i] * hist_C_[i];
    }
    r.buf[8] = qprev_;  // the overlap-add history
    r.per_slot[8] = MD;
    r.nb = 9;
    r.slots = admit_slots_;
    r.n = n;
    r.lat_in = lat_in_;
    r.bos = W(L_.bos);
    r.st_src = admit_st_;
    r.fpos_src = admit_fpos_;
    r.st = st_;
    r.fpos = fpos_;
    r.mpos = mpos_;
    for (int q = 0; q < NHB; ++q) r.flags[q] = flags_[q];
    slot_reset(r, stream_);
    PTTS_HIP(hipGetLastError());
  }
  mark_admission();
  admitted_since_call_ = true;
}

void Engine::mark_admission() {
  PTTS_HIP(hipEventRecord(ev_admit_, stream_));
  admit_pending_ = true;
  xh_dirty_ = true;  // lat_in_ (and, with a prefill, x_ / h_) rewritten
}

// x_, h_ rows of every slot from lat_in_ (the step's input projection + layer-0 norm1), on stream_
// ahead of the next front part: after an admission, a voice prefill or anything else that used
// x_ / h_ as scratch or wrote lat_in_ (the step graphs keep them current themselves)
void Engine::refresh_xh() {
  input_ln(lat_in_, inw_t_, W(L_.fl[0].n1w), W(L_.fl[0].n1b), x_, h_, max_slots_, stream_);
  PTTS_HIP(hipGetLastError());
  xh_dirty_ = false;
}

// MimiModel::decode_from_latent (mimi.rs:143-157) with the denorm + quantize of tts_model.rs:
// 1033-1038 in front, on `slot`'s own streaming state, for n frames in sequence: the back part
// of the step plan run eagerly for rows [0, slot], only `slot` marked as carrying a frame.
// Every pending frame of the engine is dropped and the slot is reset first (use on an idle
// engine, as the reference's test_decoder_parity builds its own state). Optional outputs per
// frame: quant [512] (the 32 -> 512 quantizer output), up [16][512] (after the upsample
// convtr), tr [16][512] (after the decoder transformer), time-major.
void Engine::decode_latents(int slot, const float* lat, int n, float* pcm, float* quant, float* up, float* tr) {
  PTTS_REQUIRE(ready_, "engine weights not finalized");
  PTTS_REQUIRE(slot >= 0 && slot < max_slots_, "slot out of range");
  PTTS_REQUIRE(lat != nullptr && n >= 1, "no latents");
  sync();
  for (int q = 0; q < NHB; ++q) PTTS_HIP(hipMemsetAsync(flags_[q], 0, sizeof(FrameFlags) * max_slots_, stream_));
  {
    SlotState s{};
    s.eos_step = -1;
    *h_slots_ = slot;
    *h_st_ = s;
    *h_fp_ = 0;
    PTTS_HIP(hipMemcpyAsync(admit_slots_, h_slots_, sizeof(int), hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(admit_st_, h_st_, sizeof(SlotState), hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(admit_fpos_, h_fp_, sizeof(int), hipMemcpyHostToDevice, stream_));
    ResetArgs r{};
    for (int i = 0; i < 8; ++i) {
      r.buf[i] = hist_[i];
      r.per_slot[i] = (long)hist_P_[i] * hist_C_[i];
    }
    r.buf[8] = qprev_;
    r.per_slot[8] = MD;
    r.nb = 9;
    r.slots = admit_slots_;
    r.n = 1;
    r.lat_in = lat_in_;
    r.bos = W(L_.bos);
    r.st_src = admit_st_;
    r.fpos_src = admit_fpos_;
    r.st = st_;
    r.fpos = fpos_;
    r.mpos = mpos_;
    for (int q = 0; q < NHB; ++q) r.flags[q] = flags_[q];
    slot_reset(r, stream_);
    PTTS_HIP(hipGetLastError());
  }
  const FrameFlags on{1, 0}, off{0, 0};
  auto rows16 = [&](float* dst, const float* src) {  // the slot's 16 Mimi rows [16][512]
    PTTS_HIP(hipMemcpyAsync(dst, src + (size_t)slot * UP * MD, sizeof(float) * UP * MD, hipMemcpyDeviceToHost,
                            stream_));
  };
  for (int i = 0; i < n; ++i) {
    const int par = i & 1;  // quant_upsample reads the previous frame's quantizer output from par ^ 1
    PTTS_HIP(hipMemcpyAsync(lat_out_[par] + (size_t)slot * LDIM, lat + (size_t)i * LDIM, sizeof(float) * LDIM,
                            hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(flags_[par] + slot, &on, sizeof on, hipMemcpyHostToDevice, stream_));
    std::vector<Op> ops;
    build_back(ops, slot + 1, par, 1, par, 1);
    size_t j = 0;
    for (; j < ops.size(); ++j) {
      if (ops[j].name == "seanet.conv0" && tr) rows16(tr + (size_t)i * UP * MD, mx_);
      ops[j].fn(stream_);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) throw Error(PTTS_ERR_HIP, "launch of " + ops[j].name + " failed: " + hipGetErrorString(e));
      if (j == 0 && up) rows16(up + (size_t)i * UP * MD, mx_);
    }
    if (pcm)
      PTTS_HIP(hipMemcpyAsync(pcm + (size_t)i * FRAME, pcm_[par] + (size_t)slot * FRAME, sizeof(float) * FRAME,
                              hipMemcpyDeviceToHost, stream_));
    if (quant)
      PTTS_HIP(hipMemcpyAsync(quant + (size_t)i * MD, qcur_ + (size_t)slot * NFR_MAX * MD,
                              sizeof(float) * MD, hipMemcpyDeviceToHost, stream_));
    PTTS_HIP(hipMemcpyAsync(flags_[par] + slot, &off, sizeof off, hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipStreamSynchronize(stream_));
  }
  mark_admission();
  drained_[slot] = 1;
  pv_forget(slot);
}

void Engine::slot_close(int slot) {
  PTTS_REQUIRE(slot >= 0 && slot < max_slots_, "slot out of range");
  sync();
  act_slots_.erase(std::remove(act_slots_.begin(), act_slots_.end(), slot), act_slots_.end());
  SlotState s{};
  s.eos_step = -1;
  memcpy(h_st_, &s, sizeof s);  // pinned staging (free: sync() above)
  PTTS_HIP(hipMemcpyAsync(st_ + slot, h_st_, sizeof s, hipMemcpyHostToDevice, stream_));
  for (int q = 0; q < NHB; ++q)  // drop a pending frame of the slot
    PTTS_HIP(hipMemsetAsync(flags_[q] + slot, 0, sizeof(FrameFlags), stream_));
  if (share_voice_ && slot_voice_[slot]) {  // the closed row (still stepped, discarded) reads its own rows
    h_vpre_[slot] = nullptr;
    h_vlen_[slot] = 0;
    PTTS_HIP(hipMemcpyAsync(vpre_ + slot, h_vpre_ + slot, sizeof(float*), hipMemcpyHostToDevice, stream_));
    PTTS_HIP(hipMemcpyAsync(vlen_ + slot, h_vlen_ + slot, sizeof(int), hipMemcpyHostToDevice, stream_));
  }
  mark_admission();
  PTTS_HIP(hipStreamSynchronize(stream_));
  drained_[slot] = 1;
  pv_forget(slot);
  voice_release(slot, true);
}

void Engine::voice_release(int slot, bool drained) {
  const ptts_voice* v = slot_voice_[slot];
  if (!v) return;
  slot_voice_[slot] = nullptr;
  bool free_now = false;
  {
    std::lock_guard<std::mutex> lk(voice_mu());
    free_now = --v->refs == 0 && v->dead;
  }
  if (!free_now) return;
  if (!drained) PTTS_HIP(hipStreamSynchronize(stream_));  // queued steps may still read it
  ptts_voice* w = const_cast<ptts_voice*>(v);
  if (w->kv) (void)hipFree(w->kv);
  delete w;
}

void voice_destroy(ptts_voice* v) {
  if (!v) return;
  {
    std::lock_guard<std::mutex> lk(voice_mu());
    if (v->refs > 0) {  // slots still read it: the last to let go frees it
      v->dead = true;
      return;
    }
  }
  if (v->kv) (void)hipFree(v->kv);
  delete v;
}

void Engine::set_latent(int slot, const float* lat) {
  PTTS_REQUIRE(slot >= 0 && slot < max_slots_ && lat != nullptr, "bad slot / latent");
  sync();
  PTTS_HIP(hipMemcpyAsync(lat_in_ + (size_t)slot * LDIM, lat, sizeof(float) * LDIM, hipMemcpyHostToDevice, stream_));
  mark_admission();
  PTTS_HIP(hipStreamSynchronize(stream_));
}

// ---- first-frame previews --------------------------------------------------------------------
// The pipelined engine returns a row's frame k frame_lag() calls after the call that computed its
// latent (2 n - 1 with n-frame passes): the back passes decode every row's frames together, so the
// first frame of a new utterance waits for a pass over frames of all rows. A preview decodes the
// first frame of each newly started row right after its front part, alone: a single-frame back
// pass over those rows (their latents gathered from the call's hand-off buffer into a compact
// batch of P = 1, 2, 4 or 8 rows) on its own high-priority stream, from the fresh Mimi decoder
// state every utterance starts from (tts_model.rs:941 init_states; zero conv and overlap-add
// histories, empty attention ring). That is exactly the state the row's regular pass decodes its
// frame 0 from, so the preview is that frame up to float rounding of the other tile shapes; the
// regular pass still decodes it (it advances the row's own state), and the caller delivers the
// first of the two to arrive (serve.py BatchScheduler).
void Engine::swap_back(BackBufs& b) {
  std::swap(ring_, b.ring);
  std::swap(qprev_, b.qprev);
  std::swap(qcur_, b.qcur);
  std::swap(mx_, b.mx);
  std::swap(mh_, b.mh);
  std::swap(mq_, b.mq);
  std::swap(mo_, b.mo);
  std::swap(mqkv_, b.mqkv);
  std::swap(mu_, b.mu);
  std::swap(a0_, b.a0);
  std::swap(mpartial_, b.mpartial);
  std::swap(mpcap_, b.mpcap);
  std::swap(fin_side_, b.fin_side);
  for (int i = 0; i < 3; ++i) {
    std::swap(cb_[i], b.cb[i]);
    std::swap(cv_[i], b.cv[i]);
    std::swap(ca_[i], b.ca[i]);
    std::swap(ce_[i], b.ce[i]);
  }
  for (int i = 0; i < 8; ++i) std::swap(hist_[i], b.hist[i]);
  std::swap(lat_out_[0], b.lat);
  std::swap(flags_[0], b.flags);
  std::swap(pcm_[0], b.pcm);
  std::swap(mpos_, b.mpos);
}

void Engine::preview_enable(int max_rows) {
  static_assert(PV_MAX <= GATHER_MAX, "preview rows travel in the gather's arguments");
  PTTS_REQUIRE(max_rows >= 0 && max_rows <= PV_MAX, "preview rows must be in [0, 8]");
  PTTS_REQUIRE(max_rows == 0 || pipeline_, "first-frame previews: pipelined engines only");
  PTTS_HIP(hipSetDevice(dev_));
  if (max_rows > 0 && !stream_pv_) {
    const size_t P = PV_MAX;
    BackBufs& b = pv_;
    b.ring = dalloc((size_t)ring_slot_ * P);
    b.mpos = (int*)dalloc(P);
    b.qprev = dalloc((size_t)(1 + NFR_MAX) * P * MD);
    b.qcur = b.qprev + P * MD;
    b.mx = dalloc(P * UP * MD);
    b.mh = dalloc(P * UP * MD);
    b.mq = dalloc(P * UP * MD);
    b.mo = dalloc(P * UP * MD);
    b.mqkv = dalloc(P * UP * 3 * MD);
    b.mu = dalloc(P * UP * MFF);
    b.a0 = dalloc(P * 16 * 512);
    int T = 16, ch = 512;
    for (int i = 0; i < 3; ++i) {
      T *= RATIOS[i];
      ch /= 2;
      b.cb[i] = dalloc(P * T * ch);
      b.ce[i] = dalloc(P * T * ch);
      b.cv[i] = dalloc(P * T * (ch / 2));
      b.ca[i] = dalloc(P * T * ch);
    }
    b.mpcap = std::max({(size_t)8 * P * UP * MD, (size_t)4 * P * UP * RATIOS[0] * (MD / 2)});
    b.mpartial = dalloc(b.mpcap);
    for (int i = 0; i < 8; ++i) b.hist[i] = dalloc(P * hist_P_[i] * hist_C_[i]);
    b.fin_side = dalloc(P * (FRAME / RESBLOCK_FIN_TT) * 2);
    b.lat = dalloc(P * LDIM);
    b.flags = (FrameFlags*)dalloc(P * 2);
    b.pcm = dalloc(P * FRAME);
    for (PvEntry& q : pv_q_) {
      PTTS_HIP(hipEventCreateWithFlags(&q.ev, hipEventDisableTiming));
      PTTS_HIP(hipHostMalloc((void**)&q.h_pcm, sizeof(float) * P * FRAME, hipHostMallocDefault));
    }
    for (int q = 0; q < NHB; ++q) PTTS_HIP(hipEventCreateWithFlags(&ev_pv_read_[q], hipEventDisableTiming));
    PTTS_HIP(hipEventCreateWithFlags(&ev_pv_front_, hipEventDisableTiming));
    int lo = 0, hi = 0;  // the preview is the one latency-bound part: the highest stream priority
    PTTS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    PTTS_HIP(hipStreamCreateWithPriority(&stream_pv_, hipStreamNonBlocking, hi));
  }
  pv_max_ = max_rows;
  if (!max_rows) pv_pending_.clear();
  for (int P = 1; P < 2 * max_rows; P *= 2) pv_graph(P);  // instantiated now, not at a first chunk
}

void Engine::pv_forget(int slot) {
  pv_pending_.erase(std::remove_if(pv_pending_.begin(), pv_pending_.end(),
                                   [slot](const std::pair<int, long long>& p) { return p.first == slot; }),
                    pv_pending_.end());
  for (int i = 0; i < pv_count_; ++i) {
    PvEntry& e = pv_q_[(pv_head_ + i) % PV_Q];
    for (int j = 0; j < e.n; ++j)
      if (e.slots[j] == slot) e.slots[j] = -1;
  }
}

// the preview pass over P compact rows (built once per P, captured on stream_pv_)
hipGraphExec_t Engine::pv_graph(int P) {
  auto it = pv_graphs_.find(P);
  if (it != pv_graphs_.end()) return it->second;
  std::vector<Op> ops;
  swap_back(pv_);  // build_back over the preview buffers (its lambdas capture the pointers)
  try {
    build_back(ops, P, 0, 1, 0, 1);
  } catch (...) {
    swap_back(pv_);
    throw;
  }
  swap_back(pv_);
  // The preview state must stay the fresh one (zero conv and overlap-add histories, Mimi position
  // 0): the pass's closing commit, the only op that writes it, is left out, so the buffers keep
  // the zeros dalloc gave them and no reset runs per preview. (The attention ring is rewritten at
  // positions 0..15 by each preview before it reads them. The small-row path has no fused final
  // conv, whose tile-boundary shares the commit would otherwise add.)
  PTTS_REQUIRE(P < 16 && !ops.empty() && ops.back().name == "commit", "preview pass: unexpected plan");
  ops.pop_back();
  hipGraph_t g = nullptr;
  PTTS_HIP(hipStreamBeginCapture(stream_pv_, hipStreamCaptureModeThreadLocal));
  try {
    set_wg_cap(0);
    set_back_hi(1);
    for (const Op& op : ops) op.fn(stream_pv_);
  } catch (...) {
    (void)hipStreamEndCapture(stream_pv_, &g);
    throw;
  }
  PTTS_HIP(hipStreamEndCapture(stream_pv_, &g));
  hipGraphExec_t ge = nullptr;
  PTTS_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  pv_graph_defs_[P] = g;
  pv_graphs_[P] = ge;
  return ge;
}

// After the front part of call k_ (buffer hb, rows [0, B)) is queued on stream_: the previews of
// the rows whose first front part that is (rows past B, or past pv_max_ rows, or with the FIFO
// full, take the regular path only)
void Engine::launch_previews(int B, int hb) {
  if (pv_max_ <= 0 || pv_pending_.empty()) return;
  std::vector<int> rows;
  std::vector<std::pair<int, long long>> keep;
  for (const auto& p : pv_pending_) {
    if (p.second > k_) keep.push_back(p);
    else if (p.second == k_ && p.first < B && (int)rows.size() < pv_max_) rows.push_back(p.first);
  }
  pv_pending_.swap(keep);
  if (rows.empty() || pv_count_ == PV_Q) return;
  const int n = (int)rows.size();
  int P = 1;
  while (P < n) P *= 2;
  hipGraphExec_t graph = pv_graph(P);
  PvEntry& e = pv_q_[(pv_head_ + pv_count_) % PV_Q];  // free: fetched (its copies done) or never used
  e.n = n;
  for (int i = 0; i < n; ++i) e.slots[i] = rows[i];
  PTTS_HIP(hipEventRecord(ev_pv_front_, stream_));
  PTTS_HIP(hipStreamWaitEvent(stream_pv_, ev_pv_front_, 0));
  gather_preview(lat_out_[hb], flags_[hb], rows.data(), n, P, pv_.lat, pv_.flags, stream_pv_);
  PTTS_HIP(hipGetLastError());
  PTTS_HIP(hipEventRecord(ev_pv_read_[hb], stream_pv_));  // front(k + nhb_) rewrites buffer hb
  pv_read_pending_[hb] = true;
  PTTS_HIP(hipGraphLaunch(graph, stream_pv_));
  PTTS_HIP(hipMemcpyAsync(e.h_pcm, pv_.pcm, sizeof(float) * n * FRAME, hipMemcpyDeviceToHost, stream_pv_));
  PTTS_HIP(hipEventRecord(e.ev, stream_pv_));
  ++pv_count_;
}

// Completed previews in launch order, whole previews only, at most max_n frames: slots[i] and
// pcm[i * 1920 ..]. wait: block until the launched previews complete (as many as fit).
int Engine::preview_fetch(int wait, int max_n, int* slots, float* pcm) {
  PTTS_REQUIRE(max_n >= 0 && (max_n == 0 || (slots && pcm)), "preview_fetch: null outputs");
  int got = 0;
  while (pv_count_ > 0) {
    PvEntry& e = pv_q_[pv_head_];
    int live = 0;
    for (int j = 0; j < e.n; ++j) live += e.slots[j] >= 0;
    if (got + live > max_n) break;
    if (wait) {
      PTTS_HIP(hipEventSynchronize(e.ev));
    } else {
      const hipError_t r = hipEventQuery(e.ev);
      if (r == hipErrorNotReady) {
        (void)hipGetLastError();  // not an error: clear it for the next PTTS_HIP(hipGetLastError())
        break;
      }
      PTTS_HIP(r);
    }
    for (int j = 0; j < e.n; ++j)
      if (e.slots[j] >= 0) {
        slots[got] = e.slots[j];
        memcpy(pcm + (size_t)got * FRAME, e.h_pcm + (size_t)j * FRAME, sizeof(float) * FRAME);
        ++got;
      }
    pv_head_ = (pv_head_ + 1) % PV_Q;
    --pv_count_;
  }
  return got;
}

}  // namespace ptts
