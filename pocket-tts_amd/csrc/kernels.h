// Device kernels of the Pocket TTS hot path (gfx950 / CDNA4), launch-side declarations.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace ptts {

// ---------------------------------------------------------------------------------------------
// GEMM: Y[M][N] = epilogue(A[M][K] . W[N][K]^T), fp32 in / fp32 accumulate on
// v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain). A is either a dense row-major matrix
// (mode 0) or the implicit im2col of a streaming conv1d over channels-last activations
// (mode 1): row m = (b, q), k = (tap j, ci) reads X[b][q*stride + j - P][ci], or the
// per-slot history H[b][P + t][ci] when that time index is negative (t < 0).
// W rows are padded to a multiple of 32; K must be a multiple of 32 (and cin % 32 == 0).
// grid = (ceil(N/32), ceil(M/32), S) ; S > 1 = split-K partial slabs (mode 0 only),
// or the transposed-conv phase index (mode 1).
enum Act : int { ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_ELU = 3 };

// ---------------------------------------------------------------------------------------------
// Row reduce / epilogue of a split-K GEMM, fused with residual, gate, LayerNorm and modulate:
//   v = sum_z P[z][m][n] (+bias[n]) ; v = act(v) ; v *= gate[m][n] ; v += R[m][n] ;
//   Y[m][n] = v ; (euler) cur[m][n] += v*euler_scale
//   if ln: h = LN(v)*w+b (or non-affine) ; h = h*(1+mscale[m][n]) + mshift[m][n] ; H[m][n] = h
struct RowReduceArgs {
  const float* P;
  int S, M, N;
  const float* bias;
  int act;
  const float* gate;  // [M][ldg] or nullptr
  long ldg;
  const float* R;  // residual [M][ldr] or nullptr (may alias Y)
  long ldr;
  float* Y;  // [M][ldy] or nullptr
  long ldy;
  float* Y2;  // also store elu(v) here ([M][ldy]), or nullptr (SEANet dual raw / ELU'd output)
  float* euler;  // cur [M][32]: cur += v * euler_scale (N must be 32)
  float euler_scale;
  // LayerNorm of the final row (N <= 1024)
  int ln;
  const float* ln_w;
  const float* ln_b;
  float eps;
  const float* mshift;  // modulate (mlp.rs:135): [M][ldm] or nullptr
  const float* mscale;
  long ldm;
  float* Hout;
  long ldh;
  // side job: fill[0 .. 4 * fill_n4) = 0xFFFFFFFF (re-arms the flow-head hand-off regions in the
  // launch just ahead of k_flow_head), or nullptr
  float* fill;
  long fill_n4;
  // the adaLN reduce's second copy of the ResBlock / final shift and scale columns in k_flow_head's
  // fragment order (FlowHeadArgs::fhm) for a batch of fhm_B rows, or nullptr
  float* fhm;
  int fhm_B;
  // side job for k_flow_head's first hand-off: x0 = cur W_in^T + b_in (flow-head input projection,
  // mlp.rs:375) for x0_B rows, stored into hand-off region 0 in its tile layout, or nullptr;
  // x0_w is W_in transposed, [32][512]
  const float *x0_cur, *x0_w, *x0_b;
  float* x0_hx;
  int x0_B;
  int front;  // 1: a launch of the front part (issue priority, set_front_prio)
  // (ln, N == FK_K, M <= 32) also store the LayerNorm output in gemv_fk's A-fragment order, or nullptr
  float* Hfrag;
};
struct GemmArgs {
  int mode;    // 0 dense, 1 conv
  int layout;  // workgroup layout, see kernels.hip (0 ksplit 32x32, 1: 64x64, 2: 32x128, 3: 128x32)
  int M, N, K;
  int Nw;  // rows present in W (N rounded up to 32)
  // A operand
  const float* X;
  long ldx;
  const float* H;  // conv history [B][P][cin]
  int P, T_in, Tq, stride_in, cin, elu_in;
  // B operand
  const float* W;
  long w_phase_stride;  // floats between polyphase weight blocks (mode 1)
  // bf16x6 tiles (layout >= 200, ptts_engine_config.back_mfma = PTTS_BACK_F32X6): W split exactly
  // into three bf16 pieces, W = hi + mid + lo (split3): Whm[n][k] = hi << 16 | mid (the f32 layout
  // of W, 4 B per element), Wlo[n][k] = lo (2 B per element); same indexing as W
  const unsigned* Whm;
  const unsigned short* Wlo;
  // int8 B operand (weight_quant; mode 0, split-K slabs only): W[n][k] = float(Wq[n][k]) *
  // wscale[n], formed per element before the MFMA. Replaces W when non-null.
  const int8_t* Wq;
  const float* wscale;
  // fp8 W8A8 (ptts_engine_config.fp8_gemm; mode 0, split-K slabs only): W[n][k] ~= e4m3(Wf8[n][k])
  // * wscale[n]; the A rows are quantized to e4m3 in-kernel with one scale per (row, K slice)
  // and the tile runs on v_mfma_f32_32x32x16_fp8_fp8. Replaces W when non-null.
  const uint8_t* Wf8;
  // XCD placement of the tile grid (set by gemm(); speed only): the 8 XCDs split the N tiles
  // into xcd_pn parts and the M tiles into 8 / xcd_pn parts; 0 = contiguous runs of tiles
  int xcd_pn;
  // > 0: at most this many workgroups of the launch per CU (dynamic LDS reserved to enforce it),
  // leaving room on every CU for the concurrently running part of a pipelined step
  int max_wg_per_cu;
  // 1: the weight stream is read with non-temporal loads (once-read FlowLM step weights)
  int w_nt;
  // 1: a launch of the front part (FlowLM / flow head): its waves take the front issue priority
  int front;
  // 1: a back-part launch whose waves issue at priority 3 (set by the launcher from set_back_hi)
  int back_hi;
  // measurement probe, -DPTTS_PROBES builds only (tools/; PTTS_BACK_PROBE: back-part launches of a
  // pipelined step, PTTS_FRONT_PROBE: all other tiled launches; results are wrong): bit 0 skips
  // the MFMAs, bit 1 the operand loads of the K loop. Ignored by product builds.
  int probe;
  // split-K
  int S;
  float* partial;  // [S][M][N] when S > 1
  // split tail (dense, LDS-DMA ILV tiles, S == 1): the tiles that fill whole rounds of the CUs'
  // workgroup slots run over all of K; the remainder (fewer tiles than slots) is cut into tail_S
  // K slices, one workgroup each, whose partial tiles go to tail_slab [rem][tail_S][TM*TN]; the
  // last slice to finish (tickets[rem], zero between launches) sums them in slice order and
  // applies the epilogue. gemm() derives the split of the grid; capacities are checked.
  int tail_S;
  float* tail_slab;
  long tail_cap;  // floats in tail_slab
  int* tickets;
  int tickets_cap;
  int tail_full, tiles_n;  // set by gemm()
  int tiles_m, units_z;    // persistent tiles (layout 40): tile grid rows and z units, set by gemm()
  // epilogue (S == 1)
  const float* bias;
  int act;
  const float* R;  // residual (same row mapping as Y), may alias Y
  long ldr;
  const float* rscale;  // per-column scale of the update (LayerScale) or nullptr
  float* Y;
  long ldy;
  int T_out, out_tstride;  // mode 1 output row = b*T_out + q*out_tstride + phase
  // ELU on the way out (SEANet: the consumer's ELU applied once by the producer, seanet.rs:298-305):
  // elu_out: Y = elu(v) (after the residual); Y2 != null: Y = v and Y2 = elu(v) (same indexing)
  int elu_out;
  float* Y2;
};
void gemm(const GemmArgs& a, int grid_z, hipStream_t s);
// Exact three-piece bf16 split of n f32 values (the B operand of the bf16x6 tiles): x = hi + mid
// + lo with every piece a bf16 (round to nearest even at each step; the remainders are exact in
// f32 and the last one is exact in bf16), stored as hm = bits(hi) << 16 | bits(mid) and lo.
void split3(const float* W, long n, unsigned* hm, unsigned short* lo, hipStream_t s);

// Skinny split-K GEMM (M <= 64 rows: the FlowLM step, small prefills; one 32-row block per
// grid z) with register-resident weights: the
// workgroup tile is 32 rows x 32*wn columns over a K slice of ks = kw * (4 / wn); wave w takes
// 32 columns (w % wn) and kw of the slice's k ((w / wn) * kw ..). Its weight fragment (kw * 32
// floats) comes from a copy packed in fragment order (pack_gemv: every load instruction reads 1
// contiguous KB), all of it requested at the start; the slice of X is staged in LDS. Output:
// partial slab z = blockIdx.y of P [S][M][N], S = K / ks.
struct GemvShape {
  int wn, kw;
  int ks() const { return kw * (4 / wn); }
};
bool gemv_supported(GemvShape g, int N, int K);
// Whole-K skinny GEMM for K = 1024, M <= 32 (the FlowLM step's linear1): Y = act(A W^T + bias),
// one 512-thread workgroup per 16 output columns, the 8 waves splitting K in 128-k ranges, each
// wave's weight fragment (pack_gemv_fk) AND its A fragment requested at the start: A comes in
// fragment order (FK_A_FLOATS floats, written by the row reduce ahead of it: RowReduceArgs::Hfrag),
// so every load instruction reads one contiguous KB. v_mfma_f32_16x16x4f32 over two 16-row tiles;
// the waves' partial tiles are summed through LDS in wave order and the epilogue (bias, GELU)
// writes Y: no split-K slabs and no reduce launch.
constexpr int FK_K = 1024;
constexpr long FK_A_FLOATS = 32L * FK_K;
bool gemv_fk_supported(int M, int N, int K);
void pack_gemv_fk(const float* W, int N, int K, float* packed, hipStream_t s);
void gemv_fk(const float* Afrag, int M, int N, const float* packed, const float* bias, int act, float* Y, long ldy,
             hipStream_t s);
// FlowLM feed-forward of a step pass in ONE launch (M <= 32; D = 1024, FF = 4096): linear1 + GELU as
// gemv_fk, then linear2 split over `groups` K slices into the partial slabs P [groups][M][D] (the
// following row reduce sums them). The 256 workgroups form the groups, one per linear2 slice (8
// groups of 32: the product; 16 of 16: probe builds): the members of group z produce linear1's
// columns of slice z (16 each) and hand them to each other through `hand` (data-as-flag, sc1
// stores / loads, in the MFMA A-fragment order of linear2), then each computes its linear2
// columns of slice z, its linear2
// weight fragment requested at the start beside linear1's. `hand` holds two sets of
// FFN_HAND_FLOATS floats: the launch uses set `set` (emptied, 0xFFFFFFFF, by the launch before)
// and empties the other one for the launch after. A hand-off wait that times out sets *err.
constexpr long FFN_HAND_FLOATS = 16L * 32 * 256;
bool ffn_fused_supported(int M, int D, int FF);
// groups: 16 (linear2 K slices of 256, 16 slabs) or 8 (slices of 512 with 32 members, 8 slabs)
void pack_ffn2(const float* W2, int groups, float* packed, hipStream_t s);  // linear2 [1024][4096] -> fragment order
// Q1 / Q2 (optional, weight_quant engines): linear1 / linear2 as int8 codes in pack_q8 order with
// their row scales s1 / s2 (float(q) * s == the quantized f32 weight, bit for bit, derive_int8):
// the codes are widened to f32 in registers, so the MFMA chain and the result are those of the f32
// fragments (P1 / P2 unused when the codes are given)
// fp8: Q1 / Q2 are e4m3 codes (fp8_codes) and both GEMMs run W8A8 on the fp8 MFMA (8 groups)
void ffn_fused(const float* Afrag, int M, const float* P1, const float* P2, int groups, float* hand, int set, float* P,
               int* err, hipStream_t s, const uint32_t* Q1 = nullptr, const float* s1 = nullptr,
               const uint32_t* Q2 = nullptr, const float* s2 = nullptr, bool fp8 = false);
void pack_gemv(const float* W, int N, int K, GemvShape g, float* packed, hipStream_t s);
// q8 / scale (optional): the weight as int8 codes in pack_q8 order + row scales, as for ffn_fused;
// fp8: the codes are e4m3 (fp8_codes) and the tile runs W8A8 on the fp8 MFMA ({4, 128} tiles)
void gemv_splitk(const float* X, long ldx, int M, int N, int K, const float* packed, GemvShape g, float* partial,
                 hipStream_t s, const uint32_t* q8 = nullptr, const float* scale = nullptr, bool fp8 = false);
// int8 codes of the register-resident GEMMs: a fragment-packed copy (pack_gemv / pack_gemv_fk /
// pack_ffn2 applied to the codes widened to f32, codes_to_f32) re-packed to one byte per element
// with a lane's four consecutive fragment groups in one 16-B load: u32x4 (P * NJ / 4 + J) * 64 + l
// holds the groups 4 J .. 4 J + 3 of f32 float4 index (P * NJ + j) * 64 + l (NJ: groups per lane
// and wave, a multiple of 4; n4 float4 in the f32 copy)
void codes_to_f32(const int8_t* q, long n, float* out, hipStream_t s);
void codes_u8_to_f32(const uint8_t* q, long n, float* out, hipStream_t s);  // fp8 codes as their byte values
void pack_q8(const float* packed_codes, long n4, int nj, uint32_t* q8, hipStream_t s);

// int8 codes of a quantized weight matrix: q[n][k] = W[n][k] / s[n] (exact integers in
// [-127, 127] for a blob packed by the quantizer); rows with s[n] == 0 get code 0. Any element
// with float(q) * s[n] != W[n][k] (bitwise) increments *bad.
void quant_codes(const float* W, const float* s, int N, int K, int8_t* q, int* bad, hipStream_t st);
// fp8 (OCP e4m3) codes of W [N][K] with one scale per row: s[n] = max|W[n][:]| / 448
void fp8_codes(const float* W, int N, int K, uint8_t* q, float* s, hipStream_t st);
constexpr int FP8_KSLICE_MAX = 512;  // K elements per split-K slice the fp8 GEMM stages in LDS

void row_reduce(const RowReduceArgs& a, hipStream_t s);

// LayerNorm over rows of width N (<= 1024), biased variance (candle_nn::LayerNorm).
void layernorm(const float* x, long ldx, float* y, long ldy, int M, int N, const float* w, const float* b,
               float eps, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Packed QKV (sum of S partials, or dense) -> RoPE(q,k) -> q to Q[M][d], k/v into the KV store.
// Row r belongs to slot = slot0 + r / rps at position pos = (pos_arr ? pos_arr[slot] : p0) + r % rps.
// KV layout per slot: base + slot*slot_stride + (kv*nh + h)*cap*64 + (pos % cap)*64.
// Row -> (slot, position). Uniform form: slot = slot0 + row / rps, position = (pos_arr ?
// pos_arr[slot] : p0) + row % rps. Table form (tab != nullptr, batched admission): tab[row] =
// slot << 16 | position, or -1 for a padding row (no KV write, output unused).
struct RowMap {
  int slot0, rps, p0;
  const int* pos_arr;
  const int* tab;
  // compact batched admission (slots_open): the GEMM / reduce rows are the tokens only (tab), while
  // the 16-query attention runs on slot-aligned 16-row groups with padding (ptab, mpad rows): qkv
  // rope writes query row r at padded row qrow[r], the attention writes padded row p's output at
  // row orow[p] (-1: padding, not written)
  const int* ptab = nullptr;
  int mpad = 0;
  const int* qrow = nullptr;
  const int* orow = nullptr;
};
// Shared voice prefixes (FlowLM cache): when `pre` is set, positions < pre_len[slot] of slot
// `slot` live in the voice's own cache pre[slot] ([NL][2][nh][F][64], F = pre_len[slot]; layer
// `layer` of it) instead of the slot's rows, so every utterance of one voice reads one copy.
struct KvStore {
  float* base;
  long slot_stride;
  int cap;
  const float* const* pre = nullptr;
  const int* pre_len = nullptr;
  int layer = 0;
};
void qkv_rope_append(const float* P, int S, const float* dense, int M, int nh, RowMap map, KvStore kv,
                     float* Q, hipStream_t s);

// Causal (optionally windowed) softmax attention for rows mapped as above; rows are processed
// in groups of qg (<= 16) consecutive rows of one slot. O[M][nh*64].
// Mimi decoder step: RoPE + ring append of the dense QKV rows fused into the 16-row attention
void attention16_qkv(const float* qkv, int M, int nh, RowMap map, KvStore kv, int window, float* O, hipStream_t s);
void attention(const float* Q, int M, int nh, RowMap map, KvStore kv, int window, int qg, float* O,
               hipStream_t s);
// One-query-per-row step attention fused with the QKV slab sum, RoPE and KV append (positions
// must not wrap: FlowLM cache).
void attention_step_qkv(const float* P, int S, int M, int nh, RowMap map, KvStore kv, const float* rope, float* O,
                        hipStream_t s);
// RoPE table (rope.rs:9-60): tab[pos][2i] = cos(pos * f_i), tab[pos][2i+1] = sin(pos * f_i),
// f_i = exp(-ln(1e4) * 2i / 64), i < 32, pos < npos - the values the step kernels would compute.
void rope_table(float* tab, int npos, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Per-slot generation bookkeeping (device resident so the step can be replayed as a graph).
// The step is split into a FRONT part (FlowLM + flow head: produces this step's latent and
// frame flags, owns SlotState / FlowLM KV / positions) and a BACK part (Mimi decode of a frame
// produced by the front, owns the Mimi ring, conv histories and Mimi positions). They exchange
// frames through per-parity buffers, so the back part of frame k can run concurrently with the
// front part of frame k+1.
struct SlotState {
  int active;  // row still generating
  int step;    // generation step index within the segment
  int eos_step;
  int frames_after_eos, max_frames;
  float temp, eos_threshold, noise_clamp;
  unsigned long long seed;
};
struct FrameFlags {
  int valid;  // the front produced a frame for this row at this step
  int last;   // ... and it is the row's final frame (EOS tail reached or max_frames)
};

// After the cond_embed|out_eos split-K GEMM: c = sum + b, eos logit -> eos_out,
// y_s = silu(temb[s] + c) for each lsd step, x0 noise -> cur (reads SlotState only).
constexpr int FLOW_COND_MAX_SLABS = 16;  // k_flow_cond's unrolled slab loads
void flow_cond(const float* P, int S, int B, const float* bias, const float* temb, int lsd_steps,
               const SlotState* st, float* ysilu, float* cur, float* eos_out, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Flow-head chain (mlp.rs:146-213,370-383; flow_lm.rs:7-22) in one persistent launch: per lsd
// step, x = cur W_in^T + b_in; 6 ResBlocks x += gate * (silu(mod(LN(x)) W0^T + b0) W2^T + b2);
// cur += (mod(LN_noaffine(x)) W_f^T + b_f) / lsd. mods [lsd][B][ldm] holds the adaLN shift |
// scale | gate of each block and the final shift | scale (mlp.rs:322-368). xp/up: [B][512]
// hand-off buffers; ctr: 4*ceil(B/16)+1 ints, zero before the first launch (the kernel re-arms
// them); err: set to 1 if a hand-off wait timed out. Requires 1 <= B <= 128 (flow_head_fits).
constexpr int FH_D = 512, FH_L = 32, FH_DEPTH = 6;
struct FlowHeadArgs {
  int B, lsd;
  float euler_scale;
  float* cur;
  const float* mods;
  long ldm;
  const float *in_w, *in_b;
  // ResBlock 0's tensors; block i's are at + i * blk floats (the packed blob's uniform stride)
  const float *lnw, *lnb, *w0, *b0, *w2, *b2;
  long blk;
  const float *fin_w, *fin_b;
  // the 13 chain matrices (w0 / w2 of each ResBlock, then fin_w) in fragment order
  // (pack_flow_head): every operand load instruction reads one contiguous KB
  const float* wp;
  // adaLN shift / scale in fragment order, float4 ((((((st RG + rg) 7 + i) 2 + t) 8 + w) 4 + j) 64 +
  // lane) for Euler step st, row group rg, ResBlock i (6: final layer), t 0 shift / 1 scale
  // (written by the adaLN reduce: RowReduceArgs::fhm); mods itself is read for the gates
  const float* fhm;
  // hand-off regions: 13 per Euler step (x0, then u_i, x_{i+1} per ResBlock), each
  // [ceil(B/16)][32 column groups][16 rows][16 columns] (one producer tile = one contiguous KB),
  // all 0xFFFFFFFF (empty) at launch
  float* hx;
  int x0_ready;  // 1: hand-off region 0 already holds x0 of Euler step 0 (the adaLN reduce's side job)
  int* ctr;
  int* err;
  unsigned long long* dbg;  // probe only: s_memrealtime stamps of workgroups 0-3, or nullptr
};
// Launches issued while a cap > 0 is set reserve dynamic LDS so that at most `cap` workgroups of
// each kernel share a CU (0 = no cap). Per host thread; the engine sets it around graph capture.
void set_wg_cap(int cap);
// Issue priority of the back part's tile waves (k_gemm_glds outside the front part, k_gemm_rb,
// k_resblock) for the launches made on this host thread from now on: 1 (default) s_setprio 3,
// 0 none. Set while a back graph is captured (engine.cpp part_graph).
void set_back_hi(int on);
#ifdef PTTS_PROBES
// one {tag, s_memrealtime} record appended to a device ring (tools/stamps.py)
constexpr unsigned STAMP_CAP = 1u << 16;
void stamp(unsigned long long* ring, unsigned* ctr, unsigned tag, hipStream_t s);
#endif
// Issue priority of the front part's waves (s_setprio 0..3) when they share a SIMD with back-part
// waves: probe builds only (PTTS_FRONT_PRIO), for A/B runs; a no-op in product builds.
void set_front_prio(int prio);
void set_back_prio(int prio);  // probe builds only
void set_front_skip(int v);    // probe builds only
bool flow_head_fits(int B);
// x0 = cur W_in^T + b_in into hand-off region 0 as its own launch (the adaLN reduce's side job,
// for replaying k_flow_head alone)
void flow_head_x0(const float* cur, const float* w_t, const float* bias, float* hx, int B, hipStream_t s);
// fragment-order copy of the chain's matrices for FlowHeadArgs::wp: 12 * 512 * 512 + 32 * 512 floats
size_t flow_head_packed_floats();
void pack_flow_head(const float* w0, const float* w2, long blk, const float* fin_w, float* dst, hipStream_t s);
int flow_head_grid(int B);             // workgroups of one k_flow_head launch
int flow_head_max_resident(int dev);   // co-resident k_flow_head workgroups (occupancy x CUs)
// FlowLM input_linear (32 -> 1024, no bias) + layer-0 norm1: x = lat W^T, h = LN(x) (eps 1e-5).
void input_ln(const float* lat, const float* Wt, const float* lnw, const float* lnb, float* x, float* h, int M,
              hipStream_t s);
// dst [cols][rows] = src [rows][cols]^T
void transpose(const float* src, int rows, int cols, float* dst, hipStream_t s);
void flow_head(const FlowHeadArgs& a, hipStream_t s);

// End of the front part: EOS state machine (tts_model.rs:1055-1063), frame flags, the frame's
// latent / eos logit into the parity buffers, next backbone input, step / FlowLM position.
struct FrontCommitArgs {
  int B;
  SlotState* st;
  const float* eos;  // [B] this step's logits
  const float* cur;  // [B][32] this step's latent
  float* lat_in;     // [B][32] backbone input of the next step
  float* lat_out;    // [B][32] frame latent (parity buffer)
  float* eos_out;    // [B] frame eos logit (parity buffer)
  FrameFlags* flags; // [B] (parity buffer)
  int* fpos;         // FlowLM positions, += 1
  // the next step's input projection + layer-0 norm1 of every row (k_input_ln's x, h), from the
  // updated lat_in (Wt = input_linear transposed [32][1024])
  const float *Wt, *lnw, *lnb;
  float *x, *h;
  // side jobs of workgroup 0 (they used to be copy / fill nodes at the end of the front graph, a
  // blit launch on the step's critical chain): the hand-off timeout word err_dev -> err_host
  // (pinned host memory, a system-scope store) and zero flags for the rows B .. B + n_zero - 1
  // (multi-frame passes: a pass covers the largest row count of its frames)
  const int* err_dev;
  int* err_host;
  int n_zero;
};
void front_commit(const FrontCommitArgs& a, hipStream_t s);

// Frames per back-part pass (ptts_engine_config.back_frames: 1, 2, 4 or 8) and the front -> back
// hand-off buffers of the largest pass (three passes' worth: the front part may run two passes ahead)
constexpr int NFR_MAX = 8;
constexpr int NHB_MAX = 3 * NFR_MAX;

// Denorm + 1x1 quantizer conv + depthwise ConvTrUpsample1d (k32 s16) + LN of Mimi layer 0, for
// nfr (1 .. NFR_MAX; a partial pass may cover 3) consecutive frames of every row: latent[f] [B][32] -> x [B][16 nfr][512] (frame
// f at rows 16 f..), h = LN(x). The overlap-add history [B][512] is read from qprev_in (frame 0;
// frame f > 0 overlaps frame f - 1); the quantized rows of the pass go to qprev_out
// [B][NFR_MAX][512], and the commit copies the last valid frame's into the history (rows without a
// frame, or outside the pass, keep theirs).
void quant_upsample(const float* const latent[NFR_MAX], const FrameFlags* const fl[NFR_MAX], int nfr, int B, const float* emb_std,
                    const float* emb_mean, const float* wq, const float* wup, const float* qprev_in, float* qprev_out,
                    float* x, float* h, const float* ln_w, const float* ln_b, hipStream_t s);

// End of the back part, for rows with a valid frame: copy the last P rows of each conv input
// into its history and the last valid frame's quantizer output into the overlap-add history,
// advance the Mimi position. A launch over nfr frames (T rows per row of a
// buffer = nfr frames of T / nfr rows) commits through the row's last valid frame: its valid
// frames are a prefix (an utterance starts at a pass boundary and ends with its last frame).
struct HistDesc {
  const float* src;  // [B][T][C]
  float* dst;        // [B][P][C]
  int T, C, P;
  int elu = 0;  // dst = elu(src): the history of an ELU'd activation kept only raw (ResBlockArgs::e_raw)
};
struct CommitArgs {
  HistDesc h[10];
  int nh;
  int B;
  const FrameFlags* flags[NFR_MAX];  // frame f of the pass (f < nfr)
  int nfr;
  int* mpos;  // Mimi decoder positions, += 16 per committed frame
  const float* qcur;  // the pass's quantizer outputs [B][NFR_MAX][512] (quant_upsample)
  float* qprev;       // overlap-add history [B][512] <- qcur[b][last valid frame]
  // the fused final conv's tile-boundary shares (ResBlockArgs::fside): pcm[b][x * 128 + k] +=
  // fin_side[b][x][k], k < 2, for tiles x = 1 .. fin_T / 128 - 1 (fin_side == nullptr: none)
  float* fin_pcm = nullptr;
  const float* fin_side = nullptr;
  int fin_T = 0;
  long fin_ld = 0;  // fin_pcm's row stride (0: fin_T)
};
void step_commit(const CommitArgs& a, hipStream_t s);

// Admission reset of n slots (tts_model.rs:941 init_states per segment): zero the per-slot
// regions of up to 10 state buffers, backbone input = bos, SlotState / FlowLM / Mimi positions
// from the staged per-admission arrays (index i -> slots[i]).
struct ResetArgs {
  float* buf[10];
  long per_slot[10];
  int nb;
  const int* slots;
  int n;
  float* lat_in;
  const float* bos;
  const SlotState* st_src;
  const int* fpos_src;
  FrameFlags* flags[NHB_MAX];  // every hand-off buffer: an undrained frame of the slot's previous
                         // utterance is discarded (null entries skipped)
  SlotState* st;
  int* fpos;
  int* mpos;
};
void slot_reset(const ResetArgs& a, hipStream_t s);
// The first-frame preview pass's inputs, one launch: row i < n gets the latent and frame flags of
// row idx[i] of a hand-off buffer, rows n <= i < P zeros (no frame). idx travels in the kernel
// arguments (no host-to-device copy ahead of it).
constexpr int GATHER_MAX = 8;
void gather_preview(const float* lat, const FrameFlags* flags, const int* idx, int n, int P, float* lat_out,
                    FrameFlags* flags_out, hipStream_t s);

// TimestepEmbedder pair + RMSNorm + average (mlp.rs:76-133,296-319): out [n][512].
// tmp: scratch [2][n][512].
struct TimeEmbedWeights {
  const float* l1w[2];
  const float* l1b[2];
  const float* l2w[2];
  const float* l2b[2];
  const float* alpha[2];
};
void time_embeddings(const TimeEmbedWeights& w, int n, float* tmp, float* out, hipStream_t s);

// Token embedding gather: out[i] = table[ids[i]].
void embed_gather(const int* ids, int n, const float* table, int dim, float* out, hipStream_t s);

// Strided copy: dst[r][c] = src[r][c] for rows x cols (used for small packing jobs).
void copy2d(const float* src, long lds, float* dst, long ldd, int rows, int cols, hipStream_t s);

// out[m] = sum_k x[m*ldx + k] * w[k] + b  (tiny GEMV column, e.g. the N=1 final conv)
// Streaming conv with Cout == 1: pcm[b][t] = bias + sum_{j,ci} elu(xin)[...] * w[j][ci] (Y's row
// stride ldy, 0: T).
void conv_cout1(const float* X, const float* H, int B, int T, int cin, int k, const float* w, const float* bias,
                float* Y, int elu_in, hipStream_t s, long ldy = 0);

// Fused SEANet residual block of one decoder stage (seanet.rs:43-89, kernels [3, 1], true skip):
// Y = elu(R + b1 + conv_k1(elu(b3 + conv_k3(E)))) over [B][T][C] channels-last rows, E's two rows
// before the frame from HE [B][2][C]. W3 [H][3][C] ([Cout][k][Cin]), W1 [C][H]. The intermediate
// stays in LDS. Stages: (C, H, T) = (256, 128, 96), (128, 64, 480), (64, 32, 1920).
struct ResBlockArgs {
  const float *E, *HE, *R, *W3, *b3, *W1, *b1;
  float* Y;
  int B, T, C;
  // stage 2 only (C == 64), optional: the final conv (64 -> 1, k = 3, seanet.rs:396-402) of the
  // tile's own rows in the epilogue, into fout [B][T]. A tile's first two outputs also need the
  // previous tile's last two rows: the tile stores its part of them, and its own two-row share of
  // the next tile's (fside [B][T / 128][2]) is added by the commit (CommitArgs::fin_*). The
  // utterance's first tile reads the conv history fH [B][2][64] instead.
  const float *fw = nullptr, *fb = nullptr, *fH = nullptr;
  float *fout = nullptr, *fside = nullptr;
  // E == R (the raw transposed-conv output): the k3 conv's input is elu(R), applied as the rows
  // enter LDS, so the transposed conv stores no ELU'd copy (HE stays ELU'd: the commit ELUs it)
  int e_raw = 0;
  int back_hi = 1;  // issue priority 3 (set by the launcher from set_back_hi)
  long fld = 0;     // fout's row stride (0: T; a pass block of more frames than this launch covers)
};
constexpr int RESBLOCK_FIN_TT = 128;  // stage-2 time tile (the side buffer's granularity)
void resblock(const ResBlockArgs& a, hipStream_t s);

// Encoder first conv (Cin == 1): Y[b][t][co] = bias[co] + sum_j w[co][j] * xpad[t + j], with
// the 6-sample zero history (constant padding, conv.py:90-108).
void conv_cin1(const float* X, int T, int cout, int k, const float* w, const float* bias, float* Y,
               hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Voice-prompt resampler: the polyphase FIR of scipy.signal.resample_poly (the Python reference's
// convert_audio, data/audio_utils.py:8-28; audio.rs:197-255 claims the same for Rust). Rates
// reduce by their gcd to up/down; taps h[0, L) with L = 2*half + 1, half = 10*max(up, down);
// y[m] = sum_j x[j] * h[m*down + half - j*up] for m < n_out, zeros for n_out <= m < n_pad.
struct ResamplePlan {
  int up = 1, down = 1, half = 0, L = 1;
  bool identity() const { return up == 1 && down == 1; }
  long out_len(long n) const { return (n * up + down - 1) / down; }
};
ResamplePlan resample_plan(int sr_from, int sr_to);
std::vector<float> resample_taps(const ResamplePlan& p);  // host FIR design (f32 taps x up)
void resample(const float* x, int n_in, const float* taps, const ResamplePlan& p, int n_out, int n_pad, float* y,
              hipStream_t s);

// The Rust driver's resampler instead (audio.rs:197-255): rubato 0.14.1 FastFixedIn with
// PolynomialDegree::Septic, one process() call over the whole input (chunk = n). Its source is not
// in the reference; the published algorithm restated here: a read position idx starts at -4
// (half the 8-point window), advances by t = sr_from / sr_to in f64 before each output, and
// outputs continue while the position before the step is < n - 9; output m is the degree-7
// Lagrange polynomial through x[s-3 .. s+4] (zeros outside the input), s = floor(idx), at
// frac = (f32)(idx - s). septic_schedule() replays the f64 position walk on the host (count, and
// per output s and frac when the vectors are given); resample_septic() evaluates the outputs, one
// lane each, in a fixed f32 operation order (no contraction), zeros for n_out <= m < n_pad.
long septic_schedule(long n, int sr_from, int sr_to, std::vector<int>* start, std::vector<float>* frac);
void resample_septic(const float* x, int n_in, const int* start, const float* frac, int n_out, int n_pad, float* y,
                     hipStream_t s);

}  // namespace ptts
