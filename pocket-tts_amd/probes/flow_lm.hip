// The FlowLM step's transformer (6 layers) in ONE persistent launch, for B <= 32 rows.
//
// Reference: StreamingTransformerLayer::forward (crates/pocket-tts/src/modules/transformer.rs:66-90):
//   h = norm1(x); x += out_proj(attention(rope(in_proj(h)))); h = norm2(x); x += linear2(gelu(linear1(h)))
// with the KV append and the single-query attention of attention.rs:104-283 / sdpa.rs:3-18, and
// the next layer's norm1 (the last layer: FlowLM's out_norm, flow_lm.rs:131) on the new x.
//
// As separate launches a step is 48 kernels here (a GEMM and a row reduce per matrix, the fused
// attention): each a launch gap, a ramp and a tail, and every weight load waits for its launch.
// Here 256 workgroups (one per CU, all co-resident) run seven phases per layer with in-launch
// hand-offs in which the data is its own flag (as in k_flow_head): every hand-off region of every
// layer is 0xFFFFFFFF (empty) at launch; a producer stores with sc1 (write-through) and moves on,
// a consumer re-reads (sc1) only the float4s that still hold the empty pattern. Regions are never
// reused within a launch, so there is no write-after-read hazard and no counter. The workspace has
// three sets (the front part's hand-off buffer index k % 3): step k reads set k % 3 and empties
// set (k + 1) % 3 for the next step as a side job (fire-and-forget stores between the MFMAs).
//   QKV   [32 x 3072] = h W_qkv^T: 96 column tiles x 8 K slices of 128; slabs QKV[8]
//   ATT   per (row, head) item, two waves each: slab sum, RoPE, K/V append, attention -> O
//   OUT   [32 x 1024] = O W_o^T: 32 tiles x 8 slices; slabs OUT[8]
//   RED2  one workgroup per row: x += sum OUT; h2 = norm2(x) -> H2
//   FF1   [32 x 4096] = h2 W_1^T: 128 tiles x 4 slices of 256; slabs FF1[4]
//   FF2   [32 x 1024] = gelu(sum FF1) W_2^T: 32 tiles x 16 slices of 256; slabs FF2[16]
//   RED1  one workgroup per row: x += sum FF2; h = norm1'(x) -> HN (the last layer: out_norm -> h)
// Every workgroup loads the weight fragments of its next GEMM phase before it waits for that
// phase's input (weights do not depend on the step), and the attention items load their first
// block of cached keys / values before the QKV wait (the cached keys do not depend on this step's
// token). Workgroup w sits on XCD w % 8 (round-robin dispatch, speed only): the units of one K
// slice share an XCD, so each A slice is fetched into one L2.
// GEMM units are those of k_gemv (kernels.hip): 4 waves split the unit's K slice, each a
// v_mfma_f32_32x32x2f32 chain over its fragment, the 4 partials summed through LDS in wave order.
// Split-K partials are summed by their consumers in slice order: deterministic results.
// Measured slower than the launches it replaces, so it is compiled only into the
// -DPTTS_PROBES measurement build (in place of csrc/flow_lm.hip, the product's stubs).
#include <stdexcept>

#include "../csrc/devfn.h"
#include "../csrc/kernels.h"

namespace ptts {
namespace {

constexpr int D = 1024, NH = 16, FF = 4096, NL = FL_NL, GRID = 256, ROWS = 32;
// hand-off regions of one layer in a workspace set (floats); layer l's block is at l * R_END
constexpr long R_QKV = 0;                             // [8][32][3072]
constexpr long R_O = R_QKV + 8L * ROWS * 3 * D;       // [32][1024]
constexpr long R_OUT = R_O + (long)ROWS * D;          // [8][32][1024]
constexpr long R_H2 = R_OUT + 8L * ROWS * D;          // [32][1024]
constexpr long R_FF1 = R_H2 + (long)ROWS * D;         // [4][32][4096]
constexpr long R_FF2 = R_FF1 + 4L * ROWS * FF;        // [16][32][1024]
constexpr long R_HN = R_FF2 + 16L * ROWS * D;         // [32][1024]: norm1 of the next layer
constexpr long R_END = R_HN + (long)ROWS * D;
constexpr long SET = NL * R_END;                      // one workspace set

// re-read the float4s at byte offsets off(i) (sc1) until none holds the empty pattern (bounded:
// a timeout sets *err and stops waiting for the rest of the launch; the loop condition is
// wave-uniform). The offsets are recomputed on a re-read rather than held in registers.
template <int N, typename Off>
__device__ __forceinline__ void sweep(__amdgpu_buffer_rsrc_t ws, Off off, float4 (&v)[N], int* err, bool& dead) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = fh_ld(ws, off(i));
  unsigned spins = 0;
  while (!dead) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) ok &= !fh_empty(v[i]);
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (fh_empty(v[i])) v[i] = fh_ld(ws, off(i));
    if (++spins > (1u << 20)) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dead = true;
    }
  }
}

typedef float f4v __attribute__((ext_vector_type(4)));

// this wave's weight fragments of NT column tiles (pack_gemv layout, WN = 1): NV float4 per tile
template <int KW, int NT>
struct Frag {
  f4v w[NT][KW / 8];
};
template <int KW, int NT>
__device__ __forceinline__ void load_frag(Frag<KW, NT>& f, const float* P, int S, int z, const int (&t)[NT], int wave,
                                          int lane) {
  constexpr int NV = KW / 8;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const f4v* p = reinterpret_cast<const f4v*>(P) + (((long)t[i] * S + z) * 4 + wave) * NV * 64 + lane;
#pragma unroll
    for (int j = 0; j < NV; ++j) f.w[i][j] = __builtin_nontemporal_load(p + j * 64);  // read once per step
  }
}

// A slice [32 rows][KS] (columns c0.. of a row-major [rows][ld] matrix) into LDS, rows past B
// read row B - 1 (their results are never stored). From a hand-off region of the workspace (sc1
// sweep), or, for the launch's input (src != nullptr), plain loads.
template <int KS>
__device__ __forceinline__ void stage(float* sA, const float* src, __amdgpu_buffer_rsrc_t ws, long base, int ld, int c0,
                                      int B, int tid, int* err, bool& dead) {
  constexpr int LDA = KS + 4, C4 = KS / 4, PER = ROWS * C4 / 256;
  float4 v[PER];
  if (src) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + 256 * i, row = e / C4, c4 = e % C4;
      v[i] = *reinterpret_cast<const float4*>(src + (long)min(row, B - 1) * ld + c0 + 4 * c4);
    }
  } else {
    sweep(ws, [&](int i) {
      const int e = tid + 256 * i, row = e / C4, c4 = e % C4;
      return (int)((base + (long)min(row, B - 1) * ld + c0 + 4 * c4) * 4);
    }, v, err, dead);
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + 256 * i, row = e / C4, c4 = e % C4;
    *reinterpret_cast<float4*>(&sA[row * LDA + 4 * c4]) = v[i];
  }
}

// linear2's A slice: gelu(sum of the 4 FF1 slabs at ff1) of columns c0 .. c0 + KS
// (transformer.rs:85), in two rounds (all PER x 4 loads at once would not fit beside the
// prefetched linear2 fragments in the register budget)
template <int KS>
__device__ __forceinline__ void stage_gelu(float* sA, __amdgpu_buffer_rsrc_t ws, long ff1, int c0, int B, int tid,
                                           int* err, bool& dead) {
  constexpr int LDA = KS + 4, C4 = KS / 4, PER = ROWS * C4 / 256, HALF = PER / 2;
#pragma unroll 1
  for (int hf = 0; hf < 2; ++hf) {
    float4 p[HALF * 4];
    sweep(ws, [&](int q) {
      const int e = tid + 256 * (hf * HALF + q / 4), row = e / C4, c4 = e % C4;
      return (int)((ff1 + (long)(q % 4) * ROWS * FF + (long)min(row, B - 1) * FF + c0 + 4 * c4) * 4);
    }, p, err, dead);
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const int e = tid + 256 * (hf * HALF + i), row = e / C4, c4 = e % C4;
      const float4 s = f4add(f4add(f4add(p[4 * i], p[4 * i + 1]), p[4 * i + 2]), p[4 * i + 3]);
      *reinterpret_cast<float4*>(&sA[row * LDA + 4 * c4]) =
          make_float4(gelu_tanh(s.x), gelu_tanh(s.y), gelu_tanh(s.z), gelu_tanh(s.w));
    }
  }
}

// NT 32x32 tiles of one K slice: the 4 waves' MFMA chains over their KW-wide part of the slice
// (the NT chains interleaved), then per tile the 4 partials summed through LDS in wave order; the
// tile (rows < B) goes to the slab at obase (row stride ldo) with sc1 stores (NaN canonical). Ends with a barrier:
// the caller may overwrite sA and red.
template <int KW, int NT>
__device__ __forceinline__ void tiles(const float* sA, const Frag<KW, NT>& f, float* red, __amdgpu_buffer_rsrc_t ws,
                                      long obase, int ldo, const int (&t)[NT], int wave, int lane, int B) {
  constexpr int NV = KW / 8, LDA = 4 * KW + 4;
  const int m = lane & 31, hh = lane >> 5;
  const float* ar = sA + m * LDA + wave * KW + hh * (KW / 2);
  floatx16 acc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[i][g] = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float4 a = *reinterpret_cast<const float4*>(ar + 4 * j);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, f.w[i][j].x, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, f.w[i][j].y, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, f.w[i][j].z, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, f.w[i][j].w, acc[i], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
#pragma unroll
    for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[i][g];
    __syncthreads();
#pragma unroll
    for (int ff = 0; ff < 4; ++ff) {
      const int g = wave * 4 + ff;
      float v = red[g * 64 + lane];
#pragma unroll
      for (int kk = 1; kk < 4; ++kk) v += red[(kk * 16 + g) * 64 + lane];
      const int row = (g & 3) + 8 * (g >> 2) + 4 * hh;
      if (row < B) fh_put1(ws, (int)((obase + (long)row * ldo + t[i] * 32 + m) * 4), v);
    }
    __syncthreads();
  }
}

// Row b of a reduce phase: x[b] += sum of the S slabs at slab (slice order), stored back (the
// row's only writer), then LayerNorm (eps 1e-5, affine) of the new row into hout (plain) or the
// hand-off region at hreg (sc1, NaN canonical).
template <int S>
__device__ __forceinline__ void reduce_row(float* x, __amdgpu_buffer_rsrc_t ws, long slab, int b, const float* lnw,
                                           const float* lnb, float* hout, long hreg, float* sh, int tid, int* err,
                                           bool& dead) {
  const int col = 4 * tid;
  float4 p[S];
  float4* xp = reinterpret_cast<float4*>(x + (long)b * D + col);
  const float4 xr = *xp;
  sweep(ws, [&](int z) { return (int)((slab + ((long)z * ROWS + b) * D + col) * 4); }, p, err, dead);
  float4 v = p[0];
#pragma unroll
  for (int z = 1; z < S; ++z) v = f4add(v, p[z]);
  v = f4add(v, xr);
  *xp = v;
  const float mean = block_sum((v.x + v.y) + (v.z + v.w), sh) / (float)D;
  const float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
  const float den = sqrtf(block_sum((d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w), sh) / (float)D + 1e-5f);
  const float4 w = *reinterpret_cast<const float4*>(lnw + col), bb = *reinterpret_cast<const float4*>(lnb + col);
  const float4 h = make_float4(d.x / den * w.x + bb.x, d.y / den * w.y + bb.y, d.z / den * w.z + bb.z,
                               d.w / den * w.w + bb.w);
  if (hout) *reinterpret_cast<float4*>(hout + (long)b * D + col) = h;
  else fh_put(ws, (int)((hreg + (long)b * D + col) * 4), h);
}

struct AttnLds {
  float q[2][3][64];  // per item: q | k | v of the new position (after RoPE)
  float ml[2][2][2];  // per item, per wave: running max, running sum
  float o[2][2][64];  // per item, per wave: unnormalised output
};

// The ATT phase of layer l: items (row b, head) 2w and 2w + 1 on waves {0, 1} and {2, 3}.
// Within an item, the two waves take alternate 32-key blocks of the cached positions 0..qp-1
// (the load / score / P.V scheme of k_attn_decode_qkv: a 1-KB wave load gives lane l the 4 dims
// 4(l % 16).. of key 4i + l/16, scores are 4-term dots summed over 16 lanes with DPP); wave 0 of
// the item adds the new key from LDS, and the two waves' partial softmaxes are merged.
__device__ __forceinline__ void attend(const FlowLmArgs& a, int l, int wave, int lane, int tid,
                                       __amdgpu_buffer_rsrc_t ws, long lb, AttnLds& s, bool& dead) {
  constexpr int KQ = 8, BLK = 2 * 4 * KQ;
  const int it = wave >> 1, wi = wave & 1;
  const int item = 2 * (int)blockIdx.x + it, b = item / NH, hd = item % NH;
  const bool live = b < a.B;
  const int g = lane >> 4, c4 = (lane & 15) * 4;
  int slot = 0, qp = 0;
  if (live) row_slot_pos(a.map, b, slot, qp);
  // a finished row is still stepped (its frame is discarded): once it has filled the cache its
  // key / value are not appended (position cap would spill into the next head's position 0)
  const bool append = live && qp < a.cap;
  qp = min(qp, a.cap - 1);
  float* kvs = a.kv + (long)l * a.kv_layer + (long)max(slot, 0) * a.kv_slot;
  float* kb = kvs + (long)hd * a.cap * 64;
  float* vb = kvs + (long)(NH + hd) * a.cap * 64;
  const int last = qp - 1;
  float4 k[KQ], v[KQ];
  auto load_block = [&](int base) {
#pragma unroll
    for (int i = 0; i < KQ; ++i) {
      const long off = (long)min(base + 4 * i + g, last) * 64 + c4;
      const f4v kk = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(kb + off));
      const f4v vv = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(vb + off));
      k[i] = make_float4(kk.x, kk.y, kk.z, kk.w);
      v[i] = make_float4(vv.x, vv.y, vv.z, vv.w);
    }
  };
  int base = 4 * KQ * wi;
  if (live && base < qp) load_block(base);
  const int t = tid & 127;  // thread of the item's two waves
  if (live && t < 64) {     // q | k | v float4 t (t < 48): the 8 slabs summed in slice order
    const int tt = min(t, 47), part = tt >> 4, d4 = (tt & 15) * 4;
    const long col = (long)part * D + hd * 64 + d4;
    float4 p[8];
    sweep(ws, [&](int z) { return (int)((lb + R_QKV + ((long)z * ROWS + b) * 3 * D + col) * 4); }, p, a.err, dead);
    float4 sum = p[0];
#pragma unroll
    for (int z = 1; z < 8; ++z) sum = f4add(sum, p[z]);
    if (t < 48) *reinterpret_cast<float4*>(&s.q[it][part][d4]) = sum;
  }
  __syncthreads();
  if (live && wi == 0) {  // rotate the (2i, 2i+1) pairs of q (lanes < 32) and k; append k
    const int i = lane & 31, part = lane >> 5;
    const float2 cssn = *reinterpret_cast<const float2*>(a.rope + (long)qp * 64 + 2 * i);
    const float x0 = s.q[it][part][2 * i], x1 = s.q[it][part][2 * i + 1];
    const float y0 = x0 * cssn.x - x1 * cssn.y, y1 = x0 * cssn.y + x1 * cssn.x;  // one wave: reads precede writes
    s.q[it][part][2 * i] = y0;
    s.q[it][part][2 * i + 1] = y1;
    if (part == 1 && append) {
      kb[(long)qp * 64 + 2 * i] = y0;
      kb[(long)qp * 64 + 2 * i + 1] = y1;
    }
  } else if (append && wi == 1) {
    vb[(long)qp * 64 + lane] = s.q[it][2][lane];
  }
  __syncthreads();
  float m = -INFINITY, lsum = 0.f;
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    const float4 q = *reinterpret_cast<const float4*>(&s.q[it][0][c4]);
    for (; base < qp; base += BLK) {  // cached keys 0 .. qp-1, block `base` already in registers
      float sc[KQ];
      float bm = -INFINITY;
#pragma unroll
      for (int i = 0; i < KQ; ++i) {
        const float part = q.x * k[i].x + q.y * k[i].y + q.z * k[i].z + q.w * k[i].w;
        const float tt = row16_sum(part) * 0.125f;  // 1/sqrt(64) (attention.rs:191,229)
        sc[i] = base + 4 * i + g <= last ? tt : -INFINITY;
        bm = fmaxf(bm, sc[i]);
      }
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mn = fmaxf(m, bm);
      const float alpha = expf(m - mn);
      float ps = 0.f;
      o.x *= alpha; o.y *= alpha; o.z *= alpha; o.w *= alpha;
#pragma unroll
      for (int i = 0; i < KQ; ++i) {
        const float p = expf(sc[i] - mn);  // 0 for masked keys
        ps += p;
        o.x += p * v[i].x; o.y += p * v[i].y; o.z += p * v[i].z; o.w += p * v[i].w;
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      lsum = lsum * alpha + ps;
      m = mn;
      if (base + BLK < qp) load_block(base + BLK);
    }
    // combine the 4 key rows (lanes l, l^16, l^32, l^48 hold the same dims)
    o.x += __shfl_xor(o.x, 16, 64); o.y += __shfl_xor(o.y, 16, 64);
    o.z += __shfl_xor(o.z, 16, 64); o.w += __shfl_xor(o.w, 16, 64);
    o.x += __shfl_xor(o.x, 32, 64); o.y += __shfl_xor(o.y, 32, 64);
    o.z += __shfl_xor(o.z, 32, 64); o.w += __shfl_xor(o.w, 32, 64);
    if (wi == 0) {  // the new key (position qp) from LDS
      const float sc = wave_sum(s.q[it][0][lane] * s.q[it][1][lane]) * 0.125f;
      const float mn = fmaxf(m, sc);
      const float alpha = expf(m - mn);
      const float p = expf(sc - mn);
      lsum = lsum * alpha + p;
      const float4 vn = *reinterpret_cast<const float4*>(&s.q[it][2][c4]);
      o.x = o.x * alpha + p * vn.x; o.y = o.y * alpha + p * vn.y;
      o.z = o.z * alpha + p * vn.z; o.w = o.w * alpha + p * vn.w;
      m = mn;
    }
  }
  if (lane == 0) {
    s.ml[it][wi][0] = m;
    s.ml[it][wi][1] = lsum;
  }
  if (lane < 16) *reinterpret_cast<float4*>(&s.o[it][wi][c4]) = o;
  __syncthreads();
  if (live && wi == 0) {
    const float m0 = s.ml[it][0][0], m1 = s.ml[it][1][0], mx = fmaxf(m0, m1);
    const float e0 = m0 == -INFINITY ? 0.f : expf(m0 - mx), e1 = m1 == -INFINITY ? 0.f : expf(m1 - mx);
    const float num = s.o[it][0][lane] * e0 + s.o[it][1][lane] * e1;
    const float den = s.ml[it][0][1] * e0 + s.ml[it][1][1] * e1;
    fh_put1(ws, (int)((lb + R_O + (long)b * D + hd * 64 + lane) * 4), num / den);
  }
}

__global__ __launch_bounds__(256, 2) void k_flow_lm(FlowLmArgs a) {
  __shared__ __attribute__((aligned(16))) float sA[ROWS * (256 + 4)];
  __shared__ __attribute__((aligned(16))) float red[4 * 16 * 64];
  __shared__ __attribute__((aligned(16))) AttnLds att;
  __shared__ float sh[4];
  const int tid0 = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  const int w = blockIdx.x, xcd = w & 7, r = w >> 3;
  const int B = a.B;
  const __amdgpu_buffer_rsrc_t ws = fh_rsrc(a.ws);
  bool dead = false;
  // unit maps (see the file comment): K slice z and column tiles t of each GEMM phase
  const int zq = xcd, zo = xcd, z1 = xcd & 3, z2 = xcd + 8 * (r >> 4);
  const int tq[3] = {3 * r, 3 * r + 1, 3 * r + 2};
  const int to[1] = {r};
  const int t1[2] = {2 * (r + 32 * (xcd >> 2)), 2 * (r + 32 * (xcd >> 2)) + 1};
  const int t2[2] = {2 * (r & 15), 2 * (r & 15) + 1};
  Frag<32, 3> fq;
  Frag<32, 1> fo;
  Frag<64, 2> f1, f2;
#ifdef PTTS_PROBES
  const int dbg_slot = w == 0 ? 0 : (w == 37 ? 1 : (w == 255 ? 2 : -1));
  int sk = 0;
#define FLM_STAMP() \
  if (a.dbg && dbg_slot >= 0 && tid0 == 0 && sk < 128) a.dbg[dbg_slot * 128 + sk++] = __builtin_amdgcn_s_memrealtime()
#else
#define FLM_STAMP() (void)0
#endif
  FLM_STAMP();
#pragma unroll 1
  for (int l = 0; l < NL; ++l) {
    const long lb = (long)l * R_END;  // this layer's hand-off regions
    // thread ids made opaque per layer: the per-lane addresses below are recomputed each layer
    // instead of being hoisted out of the loop (they exceeded the register budget and spilled)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    // ---- QKV: h W_qkv^T, K slice zq (128), tiles tq (weights requested before the wait for h;
    // a prefetch across the loop's back edge made the register budget spill)
    load_frag(fq, a.lw[FL_LW * l], 8, zq, tq, wave, lane);
    stage<128>(sA, l == 0 ? a.h : nullptr, ws, lb - R_END + R_HN, D, 128 * zq, B, tid, a.err, dead);
    __syncthreads();
    FLM_STAMP();
    tiles<32, 3>(sA, fq, red, ws, lb + R_QKV + (long)zq * ROWS * 3 * D, 3 * D, tq, wave, lane, B);
    load_frag(fo, a.lw[FL_LW * l + 1], 8, zo, to, wave, lane);
    FLM_STAMP();
    // ---- ATT
    attend(a, l, wave, lane, tid, ws, lb, att, dead);
    FLM_STAMP();
    // ---- OUT: O W_o^T, K slice zo, tile to
    stage<128>(sA, nullptr, ws, lb + R_O, D, 128 * zo, B, tid, a.err, dead);
    __syncthreads();
    FLM_STAMP();
    tiles<32, 1>(sA, fo, red, ws, lb + R_OUT + (long)zo * ROWS * D, D, to, wave, lane, B);
    load_frag(f1, a.lw[FL_LW * l + 2], 4, z1, t1, wave, lane);
    FLM_STAMP();
    // ---- RED2: x += attention output; h2 = norm2(x)
    if (w < B) {
      reduce_row<8>(a.x, ws, lb + R_OUT, w, a.lw[FL_LW * l + 6], a.lw[FL_LW * l + 7], nullptr, lb + R_H2, sh, tid,
                    a.err, dead);
    } else if (w >= ROWS) {  // side job of the idle workgroups: empty this layer's regions of the
      // next step's set (plain stores; their completion overlaps the wait for h2)
      uint4* nx = reinterpret_cast<uint4*>(a.ws_next + lb);
      for (long i = (long)(w - ROWS) * 256 + tid; i < R_END / 4; i += (long)(GRID - ROWS) * 256)
        nx[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    FLM_STAMP();
    // ---- FF1: h2 W_1^T, K slice z1 (256), tiles t1
    stage<256>(sA, nullptr, ws, lb + R_H2, D, 256 * z1, B, tid, a.err, dead);
    __syncthreads();
    FLM_STAMP();
    tiles<64, 2>(sA, f1, red, ws, lb + R_FF1 + (long)z1 * ROWS * FF, FF, t1, wave, lane, B);
    load_frag(f2, a.lw[FL_LW * l + 3], 16, z2, t2, wave, lane);
    FLM_STAMP();
    // ---- FF2: gelu(u) W_2^T, K slice z2 (256), tiles t2
    stage_gelu<256>(sA, ws, lb + R_FF1, 256 * z2, B, tid, a.err, dead);
    __syncthreads();
    FLM_STAMP();
    tiles<64, 2>(sA, f2, red, ws, lb + R_FF2 + (long)z2 * ROWS * D, D, t2, wave, lane, B);
    FLM_STAMP();
    // ---- RED1: x += feed-forward output; h = norm1 of the next layer (last layer: out_norm)
    if (w < B) {
      const bool fin = l + 1 == NL;
      reduce_row<16>(a.x, ws, lb + R_FF2, w, fin ? a.onw : a.lw[FL_LW * (l + 1) + 4],
                     fin ? a.onb : a.lw[FL_LW * (l + 1) + 5], fin ? a.h : nullptr, lb + R_HN, sh, tid, a.err, dead);
    }
    FLM_STAMP();
  }
}

}  // namespace

bool flow_lm_fits(int B) { return B >= 1 && B <= ROWS; }
size_t flow_lm_set_floats() { return (size_t)SET; }
int flow_lm_grid() { return GRID; }

int flow_lm_max_resident(int dev) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_flow_lm, 256, 0) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return per_cu * cus;
}

void flow_lm(const FlowLmArgs& a, hipStream_t s) {
  if (!flow_lm_fits(a.B)) throw std::runtime_error("flow_lm: B out of range");
  hipLaunchKernelGGL(k_flow_lm, dim3(GRID), dim3(256), 0, s, a);
}

}  // namespace ptts
