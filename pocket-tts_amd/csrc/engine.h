// Batched Pocket TTS engine: owns device weights, per-slot streaming state and the step plan.
#pragma once
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "weights.h"

// Immutable voice prefix (the reference's ModelState after the prompt prefill,
// tts_model.rs:490-501 / 504-560): FlowLM KV for F conditioning positions.
// Slots read the prefix from this copy (shared voice prefixes, KvStore::pre): `refs` counts the
// slots that do, and ptts_voice_destroy on a referenced voice only marks it `dead`; the last
// slot to let go of it frees it (ptts::voice_destroy, Engine::voice_release).
struct ptts_voice {
  int F = 0;
  float* kv = nullptr;      // device [NL][2][NH][F][64]
  std::vector<float> cond;  // conditioning rows [F][1024] (kept for PCM voices)
  const void* owner = nullptr;
  mutable int refs = 0;
  mutable bool dead = false;
};

namespace ptts {

// ptts_voice_destroy: frees the voice now, or (while slots still read its prefix) marks it for
// the last of them to free
void voice_destroy(ptts_voice* v);

struct Op {
  std::string name;
  std::function<void(hipStream_t)> fn;
  double flops = 0, bytes = 0;  // algorithmic cost of one launch (GEMM/conv ops)
  // state an isolated replay of `fn` needs first (time_op), which the step's previous ops provide
  std::function<void(hipStream_t)> prep = nullptr;
};

class Engine {
 public:
  explicit Engine(const ptts_engine_config& cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  void finalize();
  void load_blob(const float* host, size_t n_bytes);
  float* blob() { return blob_; }
  int max_slots() const { return max_slots_; }
  bool pipelined() const { return pipeline_; }
  // calls by which a frame trails its FlowLM step (ptts_frame_lag) and the latest admission's
  // start delay
  // (a pass over nfr frames: 2 nfr - 1 calls; single frames: 1)
  int frame_lag() const { return !pipeline_ ? 0 : 2 * nfr_ - 1; }
  int admit_delay() const { return admit_delay_; }

  ptts_voice* voice_from_prompt(const float* prompt, int F);
  ptts_voice* voice_from_pcm(const float* pcm, int n) { return voice_from_audio(pcm, n, PTTS_SAMPLE_RATE, 0); }
  // resampler: PTTS_RESAMPLE_POLY (resample_poly rule) or PTTS_RESAMPLE_RUBATO_SEPTIC (the Rust driver's)
  ptts_voice* voice_from_audio(const float* x, int n, int sample_rate, int chunk_frames,
                               int resampler = PTTS_RESAMPLE_POLY);
  void resample_host(const float* x, int n, int sr_from, int sr_to, float* y, int resampler = PTTS_RESAMPLE_POLY);
  void slot_open(int slot, const ptts_voice* v, const int32_t* ids, int n, const ptts_gen_params& p);
  void slots_open(int n, const int* slots, const ptts_voice* const* voices, const int32_t* ids, const int* n_ids,
                  const ptts_gen_params* params);
  void slot_close(int slot);
  void set_latent(int slot, const float* lat);
  void decode_latents(int slot, const float* lat, int n, float* pcm, float* quant, float* up, float* tr);

  void step_async(int B);
  // a pipelined call that starts no frame (ptts_flush_async): only the back parts of frames
  // already computed advance, so a caller whose rows have all finished drains the pipeline
  // without running front parts whose frames would be discarded
  void flush_async(int B);
  void sync();
  // the frame of the call calls_back (0 or 1) calls before the latest
  void fetch(int B, float* pcm, uint8_t* valid, uint8_t* last, float* eos, float* lat, int calls_back = 0);
  // fetch() of that call would not block (its frame's back pass has completed)
  bool fetch_ready(int calls_back);
  // the front part of the call calls_back (0..3) calls before the latest has completed (wait:
  // block until it has); true for calls before the first
  bool front_done(int calls_back, bool wait);

  // First-frame previews (ptts_preview_enable / ptts_preview_fetch): the first frame of up to
  // max_rows rows that start in one call is also decoded right after that call's front part, by a
  // single-frame back pass over those rows alone on a third stream, from a fresh Mimi state (the
  // state every utterance starts from), so a new stream's first chunk does not wait the
  // pipeline's frame lag. The rows' regular frame 0 is still decoded (it advances their state);
  // the caller delivers whichever arrives first.
  void preview_enable(int max_rows);
  int preview_fetch(int wait, int max_n, int* slots, float* pcm);

  double time_op(int B, const std::string& name, int reps);
  // GEMM-core test hook (ptts_test_gemm): Y = X W^T on tile `layout` (host buffers)
  void test_gemm(int layout, int M, int N, int K, int splits, int tail_S, const float* X, const float* Wt, float* Y);
  void overlap_probe(int B, int reps, double* us);
  std::vector<std::string> plan_names(int B);
  int int8_matrices() const { return (int)q8map_.size(); }
  int fp8_matrices() const { return (int)f8map_.size(); }

 private:
  float* dalloc(size_t n);
  const float* W(size_t off) const { return blob_ + off; }
  void upload_weights(TensorSource* src);
  void derive_int8();
  void derive_fp8();
  void prefill_rows(std::vector<Op>& ops, int slot, int T, int p0);
  void run_ops(const std::vector<Op>& ops);
  std::vector<Op> build_step(int B);
  // hb: front -> back hand-off buffer (frame index mod NHB); qp: parity of the back part's
  // quantizer history (frame index mod 2; the back part reads the previous frame's half)
  void build_front(std::vector<Op>& ops, int B, int hb);
  // back part over nfr consecutive frames from hand-off buffers hb, hb + 1, .. hb + nfr - 1; the
  // PCM goes to the pass block of hb (pcm_frames frames per row, pcmp_) or, with pcm_frames 1, to
  // pcm_[hb]
  void build_back(std::vector<Op>& ops, int B, int hb, int nfr, int qp, int pcm_frames);
  // multi-frame passes: a pass whose later calls were all flushes decodes only the frames its
  // calls started (nfr in part_graph's key)
  hipGraphExec_t part_graph(int part, int B, int hb, int qp, int nfr);
  void wait_unless_done(hipStream_t s, hipEvent_t e);
  void copy_out(int B, int hb, hipStream_t s);
  void push_rr(std::vector<Op>& ops, const std::string& name, const RowReduceArgs& r);
  void flow_layers(std::vector<Op>& ops, int M, RowMap map, int qg, bool out_norm, const std::string& tag);
  void linear_split(std::vector<Op>& ops, const std::string& name, const float* X, long ldx, int M, const float* Wt,
                    int N, int K, int* S_out);
  void conv_op(std::vector<Op>& ops, const std::string& name, const float* X, int B, int T_in, int cin, const float* H,
               int P, int stride, int elu, const float* Wt, int cout, int ktaps, int phases, const float* bias,
               const float* R, float* Y, int T_out, int tstride, int layout = 0, int elu_out = 0,
               float* Y2 = nullptr, int ksplit = 1);
  void dense_op(std::vector<Op>& ops, const std::string& name, const float* X, int M, const float* Wt, int N, int K,
                const float* bias, int act, const float* rscale, const float* R, float* Y,
                int layout = 0);
  void encoder_transformer(std::vector<Op>& ops, float* x, int T, float* h, float* qkv, float* q, float* o, float* u,
                           float* ring);

  // configuration
  int dev_ = 0, max_slots_ = 0, max_ctx_ = 0, lsd_ = 1;
  int wq_ = 0;  // weight_quant mode (QuantMode)
  // int8 code matrices of the quantized FlowLM step GEMMs: f32 weight pointer -> (codes, row scales)
  std::map<const float*, std::pair<const int8_t*, const float*>> q8map_;
  int fp8_ = 0;  // ptts_engine_config.fp8_gemm
  // e4m3 code matrices of the large FlowLM step GEMMs: f32 weight pointer -> (codes, row scales)
  std::map<const float*, std::pair<const uint8_t*, const float*>> f8map_;
  // fragment-packed copies of the f32 FlowLM step matrices for gemv_splitk: weight -> (copy, shape)
  struct Gemv {
    const float* packed;
    GemvShape g;
    int bit;  // PTTS_GEMV mask bit of the matrix
    const uint32_t* q8;   // weight_quant engines: the int8 codes in pack_q8 order, or nullptr
    const float* scale;   // their row scales
  };
  // int8 codes of a quantized matrix in the fragment order `pack` gives its f32 values (pack_q8)
  const uint32_t* pack_codes(const float* W, int N, int K, int nj, const std::function<void(const float*, float*)>& pack);
  // fused feed-forward of weight_quant engines: linear2 weight -> ((linear1 codes, scales), (linear2 codes, scales))
  std::map<const float*, std::pair<std::pair<const uint32_t*, const float*>, std::pair<const uint32_t*, const float*>>>
      ffn8map_;
  std::map<const float*, Gemv> gvmap_;
  // whole-K copies of the FlowLM linear1 matrices for gemv_fk (weight -> packed copy), and the
  // A-fragment-order copy of the norm2 output the step's out reduce writes for it
  std::map<const float*, const float*> fkmap_;
  float* hfrag_ = nullptr;
  // fused feed-forward of step passes (ffn_fused): linear2 fragment copies, the hand-off sets
  std::map<const float*, const float*> ffnmap_;
  float* ffn_hand_ = nullptr;
  int ffn_groups_ = 8;  // linear2 K slices (slabs) of the fused feed-forward
  int gemv_mask_ = 0;  // matrices that take the register-resident GEMM
  void derive_gemv();
  bool own_blob_ = true, ready_ = false;
  hipStream_t stream_ = nullptr;
  Layout L_{};
  float* blob_ = nullptr;
  std::vector<void*> allocs_;

  // per-slot streaming state
  float* kv_ = nullptr;  // [(max_slots+1)][NL][2][NH][max_ctx][64] (last slot = prefill scratch)
  long kv_slot_ = 0, kv_layer_ = 0;
  float* ring_ = nullptr;  // [max_slots][MNL][2][MNH][RING][64]
  long ring_slot_ = 0, ring_layer_ = 0;
  int* fpos_ = nullptr;
  int* mpos_ = nullptr;
  // shared voice prefixes (KvStore::pre): per slot, the voice cache its positions < F read from
  // and F (0: the slot's own rows, as for the prefill scratch slot); pinned host mirrors; the
  // voice each slot references. PTTS_NO_SHARED_VOICE (probe builds) copies the prefix in instead.
  bool share_voice_ = true;
  const float** vpre_ = nullptr;
  int* vlen_ = nullptr;
  const float** h_vpre_ = nullptr;
  int* h_vlen_ = nullptr;
  std::vector<const ptts_voice*> slot_voice_;
  // the slot lets go of its voice (freed here if it was destroyed meanwhile: `drained` = no queued
  // work may still read it, else stream_ is synchronized first)
  void voice_release(int slot, bool drained);
  SlotState* st_ = nullptr;
  float *lat_in_ = nullptr, *cur_ = nullptr, *qprev_ = nullptr, *qcur_ = nullptr, *eos_ = nullptr;
  float* hist_[8] = {};
  int hist_T_[8] = {}, hist_C_[8] = {}, hist_P_[8] = {};

  // activations
  static constexpr int PREFILL = 2048;  // rows per prefill pass (batched admission: all slots' text)
  size_t pcap_ = 0;
  float *x_ = nullptr, *h_ = nullptr, *q_ = nullptr, *o_ = nullptr, *u_ = nullptr, *partial_ = nullptr;
  // split-tail scratch of the prefill GEMMs (GemmArgs::tail_S; one stream at a time uses it)
  static constexpr size_t TAIL_CAP = (size_t)16 << 20;
  static constexpr int TICKETS = 1024;
  float* tslab_ = nullptr;
  int* tickets_ = nullptr;
  int* ids_dev_ = nullptr;
  int* rowtab_dev_ = nullptr;   // [PREFILL] slot << 16 | pos, -1 = padding row (16-row groups)
  int *ctab_dev_ = nullptr, *qrow_dev_ = nullptr, *orow_dev_ = nullptr;  // compact admission rows (RowMap)
  int* admit_slots_ = nullptr;  // [max_slots] staged admission list
  SlotState* admit_st_ = nullptr;
  int* admit_fpos_ = nullptr;
  float *ysilu_ = nullptr, *mods_ = nullptr, *xf_ = nullptr, *hf_ = nullptr, *uf_ = nullptr;
  // persistent flow-head chain (k_flow_head): hand-off rows, counters, timeout word
  bool head_uniform_stride() const;  // ResBlock tensors at one stride (k_flow_head, its packing)
  bool use_head_chain(int B) const;
  float* fhw_ = nullptr;  // the chain's matrices in fragment order (pack_flow_head, at finalize)
  float* hx_ = nullptr;   // flow-head hand-off regions [lsd * 13][roundup(B, 16)][512] (k_flow_head)
  float* fhm_ = nullptr;  // adaLN shift / scale in k_flow_head's fragment order (FlowHeadArgs::fhm)
  float* fh_inw_t_ = nullptr;  // flow-head input projection transposed [32][512] (x0 side job)
  size_t hx_floats(int B) const { return (size_t)lsd_ * 13 * ((B + 15) / 16 * 16) * FD; }
  float* inw_t_ = nullptr;  // input_linear weight transposed, [32][1024] (k_input_ln)
  int *hctr_ = nullptr, *herr_ = nullptr;
  float *mx_ = nullptr, *mh_ = nullptr, *mq_ = nullptr, *mo_ = nullptr, *mqkv_ = nullptr, *mu_ = nullptr;
  float* a0_ = nullptr;
  float *cb_[3] = {}, *cv_[3] = {}, *ca_[3] = {}, *ce_[3] = {};
  float* trb_[3] = {};  // transposed-conv biases replicated over the r output phases [r][Cout]
  // front -> back hand-off per step parity, and the back part's own split-K slabs
  // Up to three hand-off buffers: front(k) writes buffer k % nhb_ and waits only for back(k - nhb_)
  // (nhb_ = 3 lets front and back drift a step apart instead of running in lockstep).
  // 3 nfr hand-off buffers with passes over nfr = back_frames > 1 frames: a pass's nfr buffers
  // are read while the fronts of the next 2 nfr frames fill the others (the front part may run two
  // passes ahead of the back part).
  static constexpr int NHB = NHB_MAX;
  int nhb_ = 3;  // buffers in use: 3, or 3 nfr with multi-frame passes
  int nfr_ = 1;  // frames per back-part pass (ptts_engine_config.back_frames)
  int back_mfma_ = PTTS_BACK_F32;  // ptts_engine_config.back_mfma: the back part's tiles' arithmetic
  // bf16x6 back part: weight matrix -> its split3 copy (hi | mid, lo), derive_split at finalize
  std::map<const float*, std::pair<const unsigned*, const unsigned short*>> split_;
  void derive_split();
  void attach_split(GemmArgs& a) const;
  int rows_hb_[NHB] = {};  // rows of the front part that filled each hand-off buffer
  // multi-frame passes: PCM of one pass [B][nfr][1920] followed by the meta blocks of its nfr
  // buffers, per pass (buffers q with q / nfr = p), and its pinned host copy
  float* pcmp_[NHB / 2] = {};
  float* h_pcmp_[NHB / 2] = {};
  float* fin_side_ = nullptr;  // [slot][nfr * FRAME / 128][2]: the fused final conv's tile-boundary shares
  // rows admitted inside a pass's calls (not at a call k with k % nfr == 0) start at the next pass
  // boundary: their SlotState (active) is written right before that front part (pinned staging)
  SlotState* h_act_ = nullptr;
  std::vector<int> act_slots_;
  int admit_delay_ = 0;
  // positions the attention ops' algorithmic costs are stated for (plan_names; 0 = a default):
  // the mean FlowLM context and Mimi window of the rows, and the FlowLM cached positions one step
  // attention launch reads (every row's own positions + each distinct shared voice prefix once)
  double plan_ctx_ = 0, plan_win_ = 0, plan_kvu_ = 0;
  float* lat_out_[NHB] = {};
  float* eos_out_[NHB] = {};
  FrameFlags* flags_[NHB] = {};
  float* pcm_[NHB] = {};
  float* meta_[NHB] = {};  // per parity, one allocation: lat_out [B][32] | flags [B] | eos_out [B]
  size_t meta_floats_ = 0;
  float* mpartial_ = nullptr;
  size_t mpcap_ = 0;
  // in-launch split-K combine (front part only; the back part never uses it)
  int back_cap_ = 1;  // max workgroups per CU of the pipelined back part's kernels (PTTS_BACK_WG_CAP: probe builds)
  // pipelined stepping (cfg.pipeline): back part on its own stream, parity events
  bool pipeline_ = false;
  hipStream_t stream_be_ = nullptr;
  hipEvent_t ev_front_[NHB] = {}, ev_back_[NHB] = {};
  // admission / slot_close / set_latent write slot state on stream_ after the last front part the
  // next back part decodes: that back part (stream_be_) waits for this event first
  hipEvent_t ev_admit_ = nullptr;
  hipEvent_t ev_be_tail_ = nullptr;  // stream_be_'s queue at an admission (stream_ waits for it)
  hipEvent_t ev_act_ = nullptr;      // after the latest start-of-utterance copies from h_act_
  bool admit_pending_ = false;
  void mark_admission();
  long long k_ = 0;          // steps issued
  int out_hb_ = 0;           // hand-off buffer of the frame the last call produced
  int out_rows_ = 0;         // rows that frame covers
  int prev_hb_ = 0, prev_rows_ = 0;  // the same for the call before (fetch with calls_back = 1)
  long long out_k_ = -1, prev_k_ = -1;  // the call index of those frames
  // per slot: the index of the first call of its current utterance (the admission's k_): a fetched
  // frame of an earlier call belongs to the slot's previous utterance and does not drain the slot
  std::vector<long long> admit_call_;
  int front_rows_ = 0;       // rows of the last front part (0: the call was a flush)
  bool admitted_since_call_ = false;  // an admission since the last step / flush call
  // x_ / h_ / lat_in_ written outside the step graphs since the last front part (refresh_xh)
  bool xh_dirty_ = true;
  void refresh_xh();
  void call_async(int B, bool front);
  float *temb_ = nullptr, *temb_tmp_ = nullptr;
  float* rope_ = nullptr;  // FlowLM RoPE cos/sin table [max_ctx][32][2]

  // pinned host staging: each back graph ends in async D2H copies of its frame (PCM + metadata)
  // into the host set of its parity, so fetch() only reads host memory
  float* h_pcm_[NHB] = {};
  float* h_meta_[NHB] = {};
  int* h_err_ = nullptr;  // copy of herr_ made at the end of every front graph
  // probe builds (PTTS_STAMPS=path): realtime stamps at the start / end of every part graph,
  // written to the file at destruction (tools/stamps.py)
#ifdef PTTS_PROBES
  unsigned long long* stamp_ring_ = nullptr;
  unsigned* stamp_ctr_ = nullptr;
  std::vector<std::string> stamp_names_[2];  // op names of the stamped graphs (PTTS_STAMP_OPS)
#endif
  int head_resident_ = 0;  // k_flow_head workgroups that can be co-resident on this device
  int *h_slots_ = nullptr, *h_fp_ = nullptr, *h_ids_ = nullptr, *h_tab_ = nullptr;  // admission staging
  SlotState* h_st_ = nullptr;

  std::map<int, hipGraphExec_t> graphs_;
  std::map<int, hipGraph_t> graph_defs_;

  // slots whose utterance has no frame left in flight (never admitted, closed, or its last frame
  // fetched): their admission need not wait for the back parts already queued (ev_be_tail_)
  std::vector<char> drained_;

  // ---- first-frame previews (preview_enable)
  static constexpr int PV_MAX = 8;  // rows per preview pass (the small-tile back path: < 16 rows)
  static constexpr int PV_Q = 8;    // previews in flight / not yet fetched
  // the buffers build_back reads and writes, swapped in while the preview graphs are built
  struct BackBufs {
    float *ring = nullptr, *qprev = nullptr, *qcur = nullptr, *mx = nullptr, *mh = nullptr, *mq = nullptr,
          *mo = nullptr, *mqkv = nullptr, *mu = nullptr, *a0 = nullptr, *mpartial = nullptr, *fin_side = nullptr;
    float *cb[3] = {}, *cv[3] = {}, *ca[3] = {}, *ce[3] = {}, *hist[8] = {};
    float *lat = nullptr, *pcm = nullptr;
    FrameFlags* flags = nullptr;
    int* mpos = nullptr;
    size_t mpcap = 0;
  };
  void swap_back(BackBufs& b);
  struct PvEntry {
    int n = 0;
    int slots[PV_MAX] = {};
    hipEvent_t ev = nullptr;
    float* h_pcm = nullptr;  // pinned [PV_MAX][1920]
  };
  int pv_max_ = 0;
  hipStream_t stream_pv_ = nullptr;
  BackBufs pv_{};
  PvEntry pv_q_[PV_Q];
  int pv_head_ = 0, pv_count_ = 0;  // FIFO of launched, unfetched previews
  std::vector<std::pair<int, long long>> pv_pending_;  // (slot, call of its first front part)
  hipEvent_t ev_pv_front_ = nullptr;
  hipEvent_t ev_call_[4] = {};  // after the front part (or flush) of call k: ev_call_[k % 4]
  // calls from this one on record ev_call_ (set by the first front_done(): a caller that never
  // asks puts no event marker on the front stream per call); -1 = none yet
  long long call_ev_from_ = -1;
  hipEvent_t ev_pv_read_[NHB] = {};  // a preview's gather of hand-off buffer q (front(q + nhb) waits)
  bool pv_read_pending_[NHB] = {};
  std::map<int, hipGraphExec_t> pv_graphs_;
  std::map<int, hipGraph_t> pv_graph_defs_;
  void launch_previews(int B, int hb);
  hipGraphExec_t pv_graph(int P);
  void pv_forget(int slot);  // drop the slot's pending / unfetched previews (re-admitted or closed)
};

}  // namespace ptts
