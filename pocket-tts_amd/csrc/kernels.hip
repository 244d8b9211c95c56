// Device kernels of the Pocket TTS hot path, written for gfx950 (CDNA4, wave64).
//
// Reference semantics (ykevinc/pocket-tts, crates/pocket-tts/src):
//   GEMMs      <- candle Linear / Conv1d / ConvTranspose1d calls (transformer.rs:43-44,85;
//                 attention.rs:59-60,129,280; mlp.rs; conv.rs:90-136,219-267; seanet.rs)
//   attention  <- attention.rs:104-283 + sdpa.rs:36-280 (causal + context-window mask)
//   RoPE       <- rope.rs:18-60 (interleaved pairs)
//   flow head  <- mlp.rs:135-383, flow_lm.rs:7-22,98-164
//   Mimi front <- tts_model.rs:1033-1038, mimi.rs:8-37,143-157, conv.rs:315-346
#include "kernels.h"

#include <cmath>
#include <stdexcept>

#include "devfn.h"

namespace ptts {

// Measurement probes (PTTS_PROBES builds only, tools/): GemmArgs::probe bit 0 skips the MFMAs,
// bit 1 the operand loads of the tiled GEMMs (results wrong). A product build compiles them out.
#ifdef PTTS_PROBES
#define PTTS_PROBE(a) ((a).probe)
#else
#define PTTS_PROBE(a) 0
#endif

// Workgroups-per-CU cap of the launches issued while it is set (set_wg_cap; the engine sets it
// while capturing the back part of a pipelined step): dynamic LDS is reserved so that at most
// `cap` workgroups of a kernel share a CU, leaving room for the concurrently running front part.
// Per host thread: engines of one process (serve --gpus N threads) capture graphs concurrently.
static thread_local int g_wg_cap = 0;
void set_wg_cap(int cap) { g_wg_cap = cap; }
static thread_local int g_back_hi = 1;
void set_back_hi(int on) { g_back_hi = on; }
#ifdef PTTS_PROBES
__device__ int g_front_prio = 0;
void set_front_prio(int prio) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_front_prio), &prio, sizeof prio) != hipSuccess)
    throw std::runtime_error("set_front_prio failed");
}
__device__ int g_back_prio = 3;  // the product level (devfn.h back_prio)
__device__ int g_front_skip = 0;
void set_front_skip(int v) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_front_skip), &v, sizeof v) != hipSuccess)
    throw std::runtime_error("set_front_skip failed");
}
void set_back_prio(int prio) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_back_prio), &prio, sizeof prio) != hipSuccess)
    throw std::runtime_error("set_back_prio failed");
}
#else
void set_front_prio(int) {}  // product builds: no front priority
void set_back_prio(int) {}
void set_front_skip(int) {}
#endif
template <typename K>
static size_t cap_lds(K kernel, int cap) {
  if (cap <= 0) return 0;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kernel)) != hipSuccess) return 0;
  const size_t need = 163840 / (cap + 1) + 16;  // cap + 1 workgroups no longer fit (160 KiB per CU)
  return need > fa.sharedSizeBytes ? need - fa.sharedSizeBytes : 0;
}


// Sum over S (<= 16) split-K slabs p[z * stride] in z order, every load issued before the first
// add (a runtime-bounded loop waited on each load in turn: one L2 round trip per slab).
__device__ __forceinline__ float slab_sum(const float* p, long stride, int S) {
  float v[16];
#pragma unroll
  for (int z = 0; z < 16; ++z) v[z] = z < S ? p[(long)z * stride] : 0.f;
  float acc = 0.f;
#pragma unroll
  for (int z = 0; z < 16; ++z)
    if (z < S) acc += v[z];
  return acc;
}

// =============================================================================================
// GEMM (see kernels.h). One 256-thread workgroup = 4 waves owns a 32x32 output tile; the
// tile's K chunks (32 wide) are dealt round-robin to the 4 waves, each wave accumulates with
// v_mfma_f32_32x32x2_f32 straight from registers (weights are read once per tile: the GEMV
// regime of the CDNA guide, no LDS staging), and the 4 partial tiles are summed through LDS.
//
// Fragment maps for v_mfma_f32_32x32x2_f32 (lane l, r = l & 31, h = l >> 5):
//   A[i = r][k = h], B[k = h][j = r], D reg g -> row (g&3) + 8*(g>>2) + 4*h, col r.
// Lane (r, h) loads 16 consecutive k of its A row and of its W row (k0 + 16h ... +15);
// MFMA #j of a chunk consumes element j of both, i.e. k-pair {k0 + j, k0 + 16 + j}.
// =============================================================================================
// Workgroup layouts (4 waves, each accumulating one 32x32 tile):
//   LAYOUT 0  "ksplit": WG tile 32x32, the tile's K chunks dealt round-robin to the 4 waves,
//             partial tiles summed through LDS (skinny M <= 32 GEMMs: more waves per tile)
//   LAYOUT 1  2x2 waves = WG tile 64x64     LAYOUT 2  1x4 = 32x128     LAYOUT 3  4x1 = 128x32
//   (each wave runs the whole K chain of its z-slice; neighbours share A rows / W rows in L1/L2)
//   K-split variants of LAYOUT 0: LAYOUT 9 = 8 waves (2 per SIMD at one workgroup per CU),
//   LAYOUT 10 = 4 waves with two chunks in flight, LAYOUT 17 = 8 waves, two chunks in flight.
// Epilogue of one output element v of GEMM row `row`, column `col` (S == 1 path): bias,
// activation, per-column scale, residual, ELU-out / dual store. Mode 1 maps row (b, q) to the
// output time row b*T_out + q*out_tstride + phase; `ident` (wave-uniform) marks the identity map
// (mode 0, or stride-1 single-phase convs) and skips the per-element division.
__device__ __forceinline__ void gemm_store(const GemmArgs& a, int row, int col, int phase, bool ident, float v) {
  if (a.bias) v += a.bias[col];
  if (a.act == ACT_GELU) v = gelu_tanh(v);
  else if (a.act == ACT_SILU) v = silu(v);
  long yrow = row;
  if (!ident) {
    const int b2 = row / a.Tq;
    const int q2 = row - b2 * a.Tq;
    yrow = (long)b2 * a.T_out + (long)q2 * a.out_tstride + phase;
  }
  if (a.rscale) v *= a.rscale[col];
  if (a.R) v += a.R[yrow * a.ldr + col];
  if (a.Y2) {
    a.Y[yrow * a.ldy + col] = v;
    a.Y2[yrow * a.ldy + col] = elu1(v);
  } else {
    a.Y[yrow * a.ldy + col] = a.elu_out ? elu1(v) : v;
  }
}
__device__ __forceinline__ bool gemm_ident(const GemmArgs& a, int mode, int phase) {
  return mode == 0 || (phase == 0 && a.out_tstride == 1 && a.T_out == a.Tq);
}

// Fast epilogue of NG accumulator values g = g0 .. g0+NG-1 of one in-bounds 32x32 tile
// (identity row map, no split-K; row of g = tm0 + (g&3) + 8(g>>2) + 4h, column tn0 + r). The
// column is fixed per lane, so bias / scale load once, row offsets are compile-time multiples of
// the leading dimensions, and the uniform options branch once per call instead of per element
// (the generic per-element path costs ~150 VALU per output, which dominated short-K tiles).
template <int NG>
__device__ __forceinline__ void gemm_store_fast(const GemmArgs& a, const float* acc, int g0, int tm0, int tn0, int h,
                                                int r) {
  const int col = tn0 + r;
  const long rb = (long)(tm0 + 4 * h);
  auto roff = [&](int k) { const int g = g0 + k; return (long)((g & 3) + 8 * (g >> 2)); };
  const float bcol = a.bias ? a.bias[col] : 0.f;
  float v[NG];
#pragma unroll
  for (int k = 0; k < NG; ++k) v[k] = acc[k] + bcol;
  if (a.act == ACT_GELU) {
#pragma unroll
    for (int k = 0; k < NG; ++k) v[k] = gelu_tanh(v[k]);
  } else if (a.act == ACT_SILU) {
#pragma unroll
    for (int k = 0; k < NG; ++k) v[k] = silu(v[k]);
  }
  if (a.rscale) {
    const float sc = a.rscale[col];
#pragma unroll
    for (int k = 0; k < NG; ++k) v[k] *= sc;
  }
  if (a.R) {
    const float* rp = a.R + rb * a.ldr + col;
    float rv[NG];
#pragma unroll
    for (int k = 0; k < NG; ++k) rv[k] = rp[roff(k) * a.ldr];
#pragma unroll
    for (int k = 0; k < NG; ++k) v[k] += rv[k];
  }
  float* yp = a.Y + rb * a.ldy + col;
  if (a.Y2) {
    float* y2 = a.Y2 + rb * a.ldy + col;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      yp[roff(k) * a.ldy] = v[k];
      y2[roff(k) * a.ldy] = elu1(v[k]);
    }
  } else if (a.elu_out) {
#pragma unroll
    for (int k = 0; k < NG; ++k) yp[roff(k) * a.ldy] = elu1(v[k]);
  } else {
#pragma unroll
    for (int k = 0; k < NG; ++k) yp[roff(k) * a.ldy] = v[k];
  }
}
__device__ __forceinline__ void gemm_store_tile(const GemmArgs& a, const floatx16& acc, int tm0, int tn0, int h,
                                                int r) {
  float v[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) v[g] = acc[g];
  gemm_store_fast<16>(a, v, 0, tm0, tn0, h, r);
}

// XCD-aware tile order (speed only; any placement is correct). Workgroups are dealt round-robin
// to the 8 XCDs by linear id (MI355X_MICROARCH.md §Workgroup dispatch), so XCD x runs ids
// x, x + 8, ... Each XCD is given one block of the tile grid: the N tiles split into xcd_pn
// parts, the M tiles into 8 / xcd_pn, so an XCD reads 1/xcd_pn of the weights and
// xcd_pn/8 of the A rows, each once through its L2 (gemm() picks xcd_pn to minimise
// (8/pn) * |W| + pn * |A|: weight-heavy Mimi GEMMs and SEANet convs share weight tiles, the
// activation-heavy late SEANet stages share A row blocks). xcd_pn = 0, or a grid that does not
// split evenly: contiguous runs of T/8 tiles per XCD (x fastest); identity when T % 8 != 0 or
// when `on` is false.
__device__ __forceinline__ void xcd_tile(const GemmArgs& a, bool on, int& bx, int& by) {
  const int gx = gridDim.x, gy = gridDim.y, T = gx * gy;
  const int L = blockIdx.x + blockIdx.y * gx;
  const int pn = a.xcd_pn;
  if (on && (T & 7) == 0 && pn > 0) {
    const int pm = 8 / pn, xcd = L & 7, j = L >> 3, tnx = gx / pn;
    bx = (xcd % pn) * tnx + j % tnx;
    by = (xcd / pn) * (gy / pm) + j / tnx;
    return;
  }
  const int t = (on && (T & 7) == 0) ? (L & 7) * (T >> 3) + (L >> 3) : L;
  bx = t % gx;
  by = t / gx;
}

template <int LAYOUT>
struct Lay {
  static constexpr bool KSPLIT = LAYOUT == 0 || LAYOUT == 9 || LAYOUT == 10 || LAYOUT == 17;
  static constexpr int NW = (LAYOUT == 9 || LAYOUT == 17) ? 8 : 4;  // waves per workgroup
  static constexpr int PF = (LAYOUT == 10 || LAYOUT == 17) ? 2 : 1;  // chunks in flight per wave
  static constexpr int WM = LAYOUT == 1 ? 2 : (LAYOUT == 3 ? 4 : 1);
  static constexpr int WN = LAYOUT == 1 ? 2 : (LAYOUT == 2 ? 4 : 1);
};

template <int MODE, int LAYOUT>
__global__ __launch_bounds__(64 * Lay<LAYOUT>::NW) void k_gemm(GemmArgs a) {
  if (a.front) front_prio();
  constexpr bool KS = Lay<LAYOUT>::KSPLIT;
  constexpr int NW = Lay<LAYOUT>::NW;
  __shared__ float red[KS ? NW * 16 * 64 : 1];
  const int lane = threadIdx.x & 63;
  // wave-uniform (SGPR) so that the chunk loop is a scalar loop: no exec-masked joins, and
  // the compiler can keep the next chunk's loads in flight across the MFMAs (counted vmcnt)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  constexpr int WM = Lay<LAYOUT>::WM, WN = Lay<LAYOUT>::WN;
  const int wm = KS ? 0 : wave / WN, wn = KS ? 0 : wave % WN;
  int bx, by;
  xcd_tile(a, true, bx, by);
  const int n0 = (bx * WN + wn) * 32, m0 = (by * WM + wm) * 32, z = blockIdx.z;
  const int nchunks = a.K >> 5;
  int cb = 0, ce = nchunks, phase = 0;
  if (MODE == 0) {
    cb = (int)((long)nchunks * z / a.S);
    ce = (int)((long)nchunks * (z + 1) / a.S);
  } else {
    phase = z;
  }
  // waves whose tile lies wholly outside W's padded rows or outside M have nothing to do
  // (wave-uniform; LAYOUT 0 never has such waves)
  const bool wave_live = n0 < a.Nw && m0 < a.M;
  const float* wrow = a.W + (long)phase * a.w_phase_stride + (long)(wave_live ? n0 + r : r) * a.K + 16 * h;
  const int m = m0 + r;
  const bool mvalid = m < a.M;
  const float* xrow = nullptr;
  const float *xb = nullptr, *hb = nullptr;  // conv: this row's batch base in X and in H (t = 0)
  int qs = 0;                                // conv: q * stride - P
  if (MODE == 0) {
    xrow = a.X + (long)(mvalid ? m : 0) * a.ldx + 16 * h;
  } else {
    const int mm = mvalid ? m : 0;
    const int bq = mm / a.Tq;
    qs = (mm - bq * a.Tq) * a.stride_in - a.P;
    xb = a.X + (long)bq * a.T_in * a.ldx + 16 * h;
    hb = a.H + ((long)bq * a.P + a.P) * a.cin + 16 * h;
  }

  // select, not branch: both candidate addresses are formed and one is picked per lane
  auto a_ptr = [&](int k0) -> const float* {
    if (MODE == 0) return xrow + k0;
    const int j = k0 / a.cin;  // wave-uniform (scalar)
    const int ci = k0 - j * a.cin;
    const int t = qs + j;
    const float* px = xb + t * a.ldx + ci;
    const float* ph = hb + t * a.cin + ci;
    return t >= 0 ? px : ph;
  };

  floatx16 acc;
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;

  // Rows >= M were clamped to a valid row above: their garbage only reaches output rows that
  // are never stored, so the loads are unconditional (no exec-masked branches around them).
  (void)mvalid;
  constexpr bool elu = MODE == 2;  // compile-time: an if-converted ELU costs ~250 VALU per chunk
  auto load = [&](int cc, float4 (&A)[4], float4 (&Bv)[4]) {
    const float* ap = a_ptr(cc << 5);
    if (a.w_nt) {  // wave-uniform: the once-read weight stream with the non-temporal hint
      typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(wrow + (cc << 5) + 4 * i));
        Bv[i] = make_float4(w.x, w.y, w.z, w.w);
        A[i] = *reinterpret_cast<const float4*>(ap + 4 * i);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Bv[i] = *reinterpret_cast<const float4*>(wrow + (cc << 5) + 4 * i);
        A[i] = *reinterpret_cast<const float4*>(ap + 4 * i);
      }
    }
  };
  auto mma = [&](float4 (&A)[4], float4 (&Bv)[4]) {
    float af[16], bf[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[4 * i + 0] = A[i].x; af[4 * i + 1] = A[i].y; af[4 * i + 2] = A[i].z; af[4 * i + 3] = A[i].w;
      bf[4 * i + 0] = Bv[i].x; bf[4 * i + 1] = Bv[i].y; bf[4 * i + 2] = Bv[i].z; bf[4 * i + 3] = Bv[i].w;
    }
    if (elu) {
#pragma unroll
      for (int j = 0; j < 16; ++j) af[j] = elu1(af[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], acc, 0, 0, 0);
  };
  // rotating register sets: chunk c is multiplied while the next PF chunks are in flight
  float4 a0[4], b0[4], a1[4], b1[4];
  constexpr int CSTEP = KS ? NW : 1;
  int c = KS ? cb + wave : cb;
  if (!wave_live) c = ce;
  // The prefetch is unconditional (past the end it re-reads a valid chunk, never used), so no
  // control-flow join sits between a load and the MFMAs that must not wait for it.
  if (Lay<LAYOUT>::PF == 1) {
    // n chunks for this wave; loop body = two chunks with fixed register roles and no exits,
    // odd tail peeled (keeps the accumulator in place and the loads one chunk ahead)
    const int n = c < ce ? (ce - c + CSTEP - 1) / CSTEP : 0;
    const int clast = c + (n - 1) * CSTEP;
    auto chunk = [&](int i) { return i < n ? c + i * CSTEP : clast; };
    if (n > 0) {
      load(c, a0, b0);
      int i = 0;
      for (; i + 2 <= n; i += 2) {
        load(chunk(i + 1), a1, b1);
        mma(a0, b0);
        load(chunk(i + 2), a0, b0);
        mma(a1, b1);
      }
      if (i < n) mma(a0, b0);
    }
  } else {
    float4 a2[4], b2[4];
    if (c < ce) {
      load(c, a0, b0);
      load(c + CSTEP < ce ? c + CSTEP : c, a1, b1);
      for (;;) {  // invariant: a0 = chunk c, a1 = chunk c+CSTEP (if any), a2 free
        const int c1 = c + CSTEP, c2 = c + 2 * CSTEP, c3 = c + 3 * CSTEP, c4 = c + 4 * CSTEP;
        load(c2 < ce ? c2 : c, a2, b2);
        mma(a0, b0);
        if (c1 >= ce) break;
        load(c3 < ce ? c3 : c, a0, b0);
        mma(a1, b1);
        if (c2 >= ce) break;
        load(c4 < ce ? c4 : c, a1, b1);
        mma(a2, b2);
        if (c3 >= ce) break;
        c = c3;
      }
    }
  }

  const bool ident = gemm_ident(a, MODE, phase);
  auto store = [&](int g, float v) {
    const int row = m0 + (g & 3) + 8 * (g >> 2) + 4 * h;
    const int col = n0 + r;
    if (row >= a.M || col >= a.N) return;
    if (a.partial) {
      a.partial[((long)z * a.M + row) * a.N + col] = v;
      return;
    }
    gemm_store(a, row, col, phase, ident, v);
  };
  if (KS) {
#pragma unroll
    for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[g];
    __syncthreads();
    constexpr int GPW = 16 / NW;  // output registers finished per wave
    float vs[GPW];
#pragma unroll
    for (int gg = 0; gg < GPW; ++gg) {
      const int g = wave * GPW + gg;
      float v = red[(0 * 16 + g) * 64 + lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[(w * 16 + g) * 64 + lane];
      vs[gg] = v;
    }
    if (ident && !a.partial && m0 + 32 <= a.M && n0 + 32 <= a.N) {
      gemm_store_fast<GPW>(a, vs, wave * GPW, m0, n0, h, r);
    } else {
#pragma unroll
      for (int gg = 0; gg < GPW; ++gg) store(wave * GPW + gg, vs[gg]);
    }
  } else if (wave_live) {
    if (ident && !a.partial && m0 + 32 <= a.M && n0 + 32 <= a.N) {
      gemm_store_tile(a, acc, m0, n0, h, r);
    } else {
#pragma unroll
      for (int g = 0; g < 16; ++g) store(g, acc[g]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-staged variant: operands are fetched with fully coalesced float4 loads (8 lanes cover one
// 128-byte row segment of a 32-wide K chunk), written to LDS rows padded to 36 floats
// (conflict-free ds_read_b128 in the MFMA fragment order), and read back per lane as the
// 32x32x2 fragments. The next chunk's global loads are in flight while the current one is
// multiplied.
//   SHARED 0 (layout 4): WG tile 32x32, 4 waves split K, wave-private LDS, LDS reduce at the end.
//   SHARED 1 (layout 5): WG tile 64x64, 2x2 waves share the A/B chunk through double-buffered
//                        LDS (one barrier per chunk), each wave runs the full K chain.
// ---------------------------------------------------------------------------------------------
constexpr int LROW = 36;  // padded LDS row (floats)

template <int MODE, int SHARED>
__global__ __launch_bounds__(256) void k_gemm_lds(GemmArgs a) {
  // SHARED 0: 4 waves x (A 32 rows + B 32 rows) x LROW ; SHARED 1: 2 buffers x (A 64 + B 64) x LROW
  __shared__ __attribute__((aligned(16))) float lds[SHARED ? 2 * 128 * LROW : 4 * 64 * LROW];
  __shared__ float red[SHARED ? 1 : 4 * 16 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int TM = SHARED ? 64 : 32, TN = SHARED ? 64 : 32;
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM, z = blockIdx.z;
  const int nchunks = a.K >> 5;
  int cb = 0, ce = nchunks, phase = 0;
  if (MODE == 0) {
    cb = (int)((long)nchunks * z / a.S);
    ce = (int)((long)nchunks * (z + 1) / a.S);
  } else {
    phase = z;
  }
  const float* W = a.W + (long)phase * a.w_phase_stride;
  // loader mapping: row = base + lane/8 (+8 per instruction), 4 floats at col 4*(lane&7)
  const int lrow = SHARED ? (tid >> 3) : (lane >> 3);  // 0..31 (SHARED) / 0..7 (per wave)
  const int lcol = 4 * (tid & 7);
  constexpr int NLD = SHARED ? 2 : 4;  // float4 loads per operand per chunk per thread
  constexpr int RSTEP = SHARED ? 32 : 8;
  // A and W rows this thread loads
  const float* wp[NLD];
  bool wv[NLD];
  const float* ap_dense[NLD];
  int abq[NLD], aqq[NLD];
  bool av_ok[NLD];
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const int row = lrow + RSTEP * i;
    const int m = m0 + row;
    av_ok[i] = m < a.M;
    const int mm = av_ok[i] ? m : 0;
    if (MODE == 0) {
      ap_dense[i] = a.X + (long)mm * a.ldx + lcol;
    } else {
      abq[i] = mm / a.Tq;
      aqq[i] = mm - abq[i] * a.Tq;
    }
    const int n = n0 + row;
    wv[i] = n < a.Nw;
    wp[i] = W + (long)(wv[i] ? n : 0) * a.K + lcol;
  }
  auto a_src = [&](int i, int k0) -> const float* {
    if (MODE == 0) return ap_dense[i] + k0;
    const int j = k0 / a.cin;
    const int ci = k0 - j * a.cin + lcol;
    const int t = aqq[i] * a.stride_in + j - a.P;
    if (t >= 0) return a.X + ((long)abq[i] * a.T_in + t) * a.ldx + ci;
    return a.H + ((long)abq[i] * a.P + (a.P + t)) * a.cin + ci;
  };
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 ra[NLD], rb[NLD];
  auto gload = [&](int c) {
    const int k0 = c << 5;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      ra[i] = av_ok[i] ? *reinterpret_cast<const float4*>(a_src(i, k0)) : zero4;
      rb[i] = wv[i] ? *reinterpret_cast<const float4*>(wp[i] + k0) : zero4;
      if (MODE == 2)
        ra[i] = make_float4(elu1(ra[i].x), elu1(ra[i].y), elu1(ra[i].z), elu1(ra[i].w));
    }
  };
  // LDS regions
  const int wm = SHARED ? wave >> 1 : 0, wn = SHARED ? wave & 1 : 0;
  auto lds_a = [&](int buf) -> float* { return SHARED ? lds + buf * 128 * LROW : lds + wave * 64 * LROW; };
  auto lds_b = [&](int buf) -> float* { return lds_a(buf) + (SHARED ? 64 : 32) * LROW; };

  floatx16 acc;
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;
  const int cstep = SHARED ? 1 : 4;
  int c = SHARED ? cb : cb + wave;
  int buf = 0;
  if (c < ce) gload(c);
  for (; c < ce; c += cstep) {
    float* la = lds_a(buf);
    float* lb = lds_b(buf);
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      *reinterpret_cast<float4*>(la + (lrow + RSTEP * i) * LROW + lcol) = ra[i];
      *reinterpret_cast<float4*>(lb + (lrow + RSTEP * i) * LROW + lcol) = rb[i];
    }
    if (SHARED) __syncthreads();
    if (c + cstep < ce) gload(c + cstep);
    float af[16], bf[16];
    const float* pa = la + (32 * wm + r) * LROW + 16 * h;
    const float* pb = lb + (32 * wn + r) * LROW + 16 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 x = *reinterpret_cast<const float4*>(pa + 4 * i);
      const float4 y = *reinterpret_cast<const float4*>(pb + 4 * i);
      af[4 * i + 0] = x.x; af[4 * i + 1] = x.y; af[4 * i + 2] = x.z; af[4 * i + 3] = x.w;
      bf[4 * i + 0] = y.x; bf[4 * i + 1] = y.y; bf[4 * i + 2] = y.z; bf[4 * i + 3] = y.w;
    }
    if (!(PTTS_PROBE(a) & 1)) {
#pragma unroll
      for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], acc, 0, 0, 0);
    }
    if (SHARED) buf ^= 1;
  }

  const int tm0 = m0 + 32 * wm, tn0 = n0 + 32 * wn;
  auto store = [&](int g, float v) {
    const int row = tm0 + (g & 3) + 8 * (g >> 2) + 4 * h;
    const int col = tn0 + r;
    if (row >= a.M || col >= a.N) return;
    if (a.partial) {
      a.partial[((long)z * a.M + row) * a.N + col] = v;
      return;
    }
    gemm_store(a, row, col, phase, gemm_ident(a, MODE, phase), v);
  };
  if (!SHARED) {
#pragma unroll
    for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[g];
    __syncthreads();
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int g = wave * 4 + gg;
      float v = red[(0 * 16 + g) * 64 + lane] + red[(1 * 16 + g) * 64 + lane];
      v += red[(2 * 16 + g) * 64 + lane];
      v += red[(3 * 16 + g) * 64 + lane];
      store(g, v);
    }
  } else {
#pragma unroll
    for (int g = 0; g < 16; ++g) store(g, acc[g]);
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA GEMM (the CDNA guide's 2-buffer global_load_lds structure): operand tiles go
// global -> LDS with global_load_lds_dwordx4 (one 1-KiB wave instruction = RPI rows of one
// BK-wide chunk; no VGPRs), two LDS buffers, one barrier per chunk: the DMA of chunk c+1 is in
// flight while chunk c is multiplied. LDS rows are unpadded and XOR-swizzled by 16-byte column
// (BK 32: col ^ ((row>>1)&7), BK 64: col ^ (row&15)) so the ds_read_b128 fragment reads are
// conflict-free; the swizzle is applied on the per-lane global SOURCE address (the DMA writes
// lane-linearly).  WG tile (32*WM) x (32*WN), 4 waves, each one 32x32 accumulator.
// Requires K % BK == 0 and, for convs, cin % BK == 0.
// ---------------------------------------------------------------------------------------------
template <int BK>
__device__ __forceinline__ int swz(int row) {
  return BK == 32 ? ((row >> 1) & 7) : (row & 15);
}

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at
// lds_byte + 16*l. Issued through inline asm so hipcc neither counts it in vmcnt nor fences the
// ds_reads of the other buffer behind it (it cannot prove they do not alias); the caller drains
// it with an explicit `s_waitcnt vmcnt(0)` before the barrier that precedes reading it
// (cdna_hip_programming.md §5.7, M0 saved and restored inside the statement).
__device__ __forceinline__ void glds16(const float* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}
// The same with the non-temporal hint (weights that one CU reads once per step: the decode's
// weight stream, MI355X_MICROARCH.md price row nt-weights).
__device__ __forceinline__ void glds16_nt(const float* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}
// write-through (sc1) 16-byte store and L2-bypassing load: partial tiles handed between
// workgroups on different XCDs (each XCD has its own L2)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sc1_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
typedef unsigned int sc1_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void sc1_st(__amdgpu_buffer_rsrc_t r, int byte_off, float4 f) {
  const sc1_u32x4 v = {__float_as_uint(f.x), __float_as_uint(f.y), __float_as_uint(f.z), __float_as_uint(f.w)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, 16);
}
__device__ __forceinline__ float4 sc1_ld(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const sc1_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(p);
}

// bf16x6 operand pieces (k_gemm_glds PREC 2). split3_frag: 8 f32 values -> their exact three-piece
// bf16 split by truncation (x0 = the upper 16 bits of x; r = x - x0 is exact (Sterbenz) with at
// most 16 significant bits; x1 = the upper 16 bits of r; x2 = r - x1 is exact with at most 8
// significant bits, so its lower 16 bits are zero): 4 VALU ops per value plus one v_perm_b32 per
// pair and piece. hm_frag: the hi and mid pieces of 8 pre-split W values (hm = hi << 16 | mid).
__device__ __forceinline__ void split3_frag(const float* x, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  u32x4 h, m, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const unsigned u0 = __float_as_uint(x[2 * p]), u1 = __float_as_uint(x[2 * p + 1]);
    const float r0 = x[2 * p] - __uint_as_float(u0 & 0xffff0000u), r1 = x[2 * p + 1] - __uint_as_float(u1 & 0xffff0000u);
    const unsigned v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
    const float s0 = r0 - __uint_as_float(v0 & 0xffff0000u), s1 = r1 - __uint_as_float(v1 & 0xffff0000u);
    h[p] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
    m[p] = __builtin_amdgcn_perm(v1, v0, 0x07060302u);
    l[p] = __builtin_amdgcn_perm(__float_as_uint(s1), __float_as_uint(s0), 0x07060302u);
  }
  p0 = __builtin_bit_cast(bf16x8, h);
  p1 = __builtin_bit_cast(bf16x8, m);
  p2 = __builtin_bit_cast(bf16x8, l);
}
__device__ __forceinline__ void hm_frag(const float* w, bf16x8& p0, bf16x8& p1) {
  u32x4 h, m;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const unsigned e0 = __float_as_uint(w[2 * p]), e1 = __float_as_uint(w[2 * p + 1]);
    h[p] = __builtin_amdgcn_perm(e1, e0, 0x07060302u);
    m[p] = __builtin_amdgcn_perm(e1, e0, 0x05040100u);
  }
  p0 = __builtin_bit_cast(bf16x8, h);
  p1 = __builtin_bit_cast(bf16x8, m);
}

// s_waitcnt with only vmcnt = n (expcnt/lgkmcnt left at "no wait"), gfx9 simm16 encoding
#define PTTS_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | (7 << 4) | (15 << 8))

// TMW x TNW: 32x32 accumulators per wave (register blocking: one A fragment feeds TNW MFMAs,
// one B fragment TMW), WG tile (32*WM*TMW) x (32*WN*TNW).
// MODE 1 with S > 1 (single-phase convs): z is a K slice and the tile goes to partial slab z.
// MINB: workgroups per CU the register allocation must allow (__launch_bounds__ min waves per
// SIMD = MINB). ILV: the DMAs of chunk c + NBUF - 1 are issued between the MFMAs of chunk c (one
// per 16 / IPW k-steps) instead of as a burst ahead of its fragment reads: an f32 MFMA leaves 56
// of its 64 issue cycles free, so the DMA issue (60-185 cycles each) hides behind the matrix pipe.
// PREC 1, bf16 (engine back_mfma = PTTS_BACK_BF16, a variant beside the f32 path): the same tiles,
// operands still f32 in HBM and LDS, rounded to bf16 (v_cvt_pk_bf16_f32, RNE) as the fragments are
// read, and multiplied on v_mfma_f32_32x32x16_bf16 with f32 accumulation: lane half h feeds
// elements j of MFMA q from its chunk columns 16h + 8q + j for A and B alike, so each chunk's 32 k
// are summed once (2 MFMAs per 32-k chunk instead of 16). The next chunk's DMAs are issued after
// the two MFMAs.
// PREC 2, bf16x6 (PTTS_BACK_F32X6): f32 products on the bf16 matrix pipe. Every f32 operand is the
// exact sum of three bf16 pieces, x = x0 + x1 + x2 (split3: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|),
// and the tile sums the six products whose order is <= 2, a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 +
// a2 b0: each piece product is exact, the dropped three are below 2^-24 |a b| together, so the
// result has f32 accuracy (test_gpu_gemm_core: error against fp64 no larger than the f32 MFMA
// tile's) at 6 bf16 MFMAs (32 cycles each) per 16 k instead of 8 f32 ones (64 cycles each). W
// comes pre-split from finalize (GemmArgs::Whm = hi | mid in W's f32 layout, Wlo = lo: one more
// 64-B LDS row per W row and chunk, its 16-B columns swizzled by (row >> 2) & 3 so the ds_read_b128
// of a 16-lane group hit distinct banks); A is split as its fragments are read (truncation:
// x0 = x & 0xffff0000, x1 = trunc(x - x0), x2 = x - x0 - x1, all exact).
template <int MODE, int WM, int WN, int BK, int NBUF, int TMW = 1, int TNW = 1, int MINB = 1, bool ILV = false,
          int PREC = 0>
__global__ __launch_bounds__(256, MINB) void k_gemm_glds(GemmArgs a) {
  if (a.front) front_prio();
  else if (a.back_hi) back_prio();
  constexpr bool BF16 = PREC == 1, X6 = PREC == 2;
  constexpr int TM = 32 * WM * TMW, TN = 32 * WN * TNW, ROWS = TM + TN;
  constexpr int CPR = BK / 4;        // 16-byte columns per LDS row
  constexpr int RPI = 64 / CPR;      // rows per 1-KiB wave instruction
  constexpr int NMAIN = ROWS / RPI;  // DMA instructions per chunk for the A and W rows
  constexpr int NLO = X6 ? TN / 16 : 0;  // ... for the W lo rows (64 B each: 16 per instruction)
  constexpr int NINS = NMAIN + NLO;  // DMA instructions per chunk (whole workgroup)
  static_assert(NINS % 4 == 0, "every wave issues the same number of DMAs per chunk");
  static_assert(!X6 || BK == 32, "bf16x6 tiles: BK 32");
  constexpr int IPW = NINS / 4;
  constexpr int DIST = NBUF - 1;     // chunks in flight ahead of the one being multiplied
  static_assert(NBUF >= 2 && NBUF <= 4, "counted waits below cover up to 3 chunks in flight");
  constexpr int BUF = ROWS * BK + (X6 ? TN * 16 : 0);  // floats per LDS buffer (A | W | W lo)
  __shared__ __attribute__((aligned(16))) float lds[NBUF * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, h = lane >> 5;
  int bx, by;
  int tail_u = -1;  // split tail: this workgroup's (tile, slice) unit among the remainder tiles
  if (ILV && MODE == 0 && a.tail_S > 0) {
    // 1-D grid: whole tiles first (contiguous runs of them per XCD), then tail_S units per
    // remainder tile
    const int L = blockIdx.x, F = a.tail_full;
    int t;
    if (L < F) {
      t = (F & 7) == 0 ? (L & 7) * (F >> 3) + (L >> 3) : L;
    } else {
      tail_u = L - F;
      t = F + tail_u / a.tail_S;
    }
    bx = t % a.tiles_n;
    by = t / a.tiles_n;
  } else {
    xcd_tile(a, true, bx, by);
  }
  const int n0 = bx * TN, m0 = by * TM, z = blockIdx.z;
  const int nchunks = a.K / BK;
  int cb = 0, ce = nchunks, phase = 0;
  if (MODE == 0 || a.S > 1) {
    cb = (int)((long)nchunks * z / a.S);
    ce = (int)((long)nchunks * (z + 1) / a.S);
  } else {
    phase = z;
  }
  if (tail_u >= 0) {
    const int zt = tail_u % a.tail_S;
    cb = (int)((long)nchunks * zt / a.tail_S);
    ce = (int)((long)nchunks * (zt + 1) / a.tail_S);
  }
  const float* Wp = (X6 ? reinterpret_cast<const float*>(a.Whm) : a.W) + (long)phase * a.w_phase_stride;
  const unsigned lds_base = lds_addr(lds);
  // this lane's DMA sources: instruction j = wave + 4*ins covers rows j*RPI .. +RPI-1, all of
  // them A rows or all of them W rows (TM % RPI == 0), so the A/W choice is wave-uniform.
  // Conv A rows keep two base pointers (activation X and history H, both at time index 0 and
  // this lane's column); a chunk picks one per lane with a select, never a branch.
  // bf16x6: instructions j >= NMAIN move W lo rows (16 per instruction, 4 lanes of 16 B each).
  const float* src_base[IPW];
  const float* src_hist[IPW];
  int src_qs[IPW];
#pragma unroll
  for (int ins = 0; ins < IPW; ++ins) {
    const int j = wave + 4 * ins;
    if (X6 && j >= NMAIN) {
      const int lrow = (j - NMAIN) * 16 + lane / 4;
      const int lcol = (lane % 4) ^ ((lrow >> 2) & 3);
      const int n = min(n0 + lrow, a.Nw - 1);
      src_base[ins] = reinterpret_cast<const float*>(a.Wlo + (long)phase * a.w_phase_stride + (long)n * a.K + 8 * lcol);
      continue;
    }
    const int row = (j < NINS ? j : 0) * RPI + lane / CPR;
    const int lcol = (lane % CPR) ^ swz<BK>(row);
    if ((j < NINS ? j : 0) * RPI < TM) {
      const int m = min(m0 + row, a.M - 1);  // rows >= M only feed output rows that are never stored
      if (MODE == 0) {
        src_base[ins] = a.X + (long)m * a.ldx + 4 * lcol;
      } else {
        const int bq = m / a.Tq;
        const int qq = m - bq * a.Tq;
        src_qs[ins] = qq * a.stride_in - a.P;
        src_base[ins] = a.X + (long)bq * a.T_in * a.ldx + 4 * lcol;
        src_hist[ins] = a.H + ((long)bq * a.P + a.P) * a.cin + 4 * lcol;
      }
    } else {
      const int n = min(n0 + row - TM, a.Nw - 1);
      src_base[ins] = Wp + (long)n * a.K + 4 * lcol;
    }
  }
  const long ldx = a.ldx, hld = a.cin;
  // source of this lane's 16 bytes for DMA instruction `ins` of this wave and chunk c
  auto dma_src = [&](int c, int ins) -> const float* {
    const int j = wave + 4 * ins;
    const int k0 = c * BK;
    if (X6 && j >= NMAIN)  // W lo row: bf16 elements
      return reinterpret_cast<const float*>(reinterpret_cast<const unsigned short*>(src_base[ins]) + k0);
    if (MODE != 0 && j * RPI < TM) {
      const int tap = k0 / a.cin;  // scalar
      const int ci = k0 - tap * a.cin;
      const int t = src_qs[ins] + tap;
      const float* px = src_base[ins] + t * ldx + ci;
      const float* ph = src_hist[ins] + t * hld + ci;
      return t >= 0 ? px : ph;
    }
    return src_base[ins] + k0;
  };
  // DMA instruction `ins` of this wave from src into LDS buffer buf
  auto dma = [&](const float* src, int buf, int ins) {
    if (PTTS_PROBE(a) & 2) return;
    const int j = wave + 4 * ins;
    if (j >= NINS) return;  // wave-uniform
    // wave-uniform LDS base of this instruction; lane l -> + 16*l bytes
    const int off = X6 && j >= NMAIN ? buf * BUF + ROWS * BK + (j - NMAIN) * 256 : buf * BUF + j * RPI * BK;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_base + (unsigned)(off * 4));
    if (a.w_nt && j * RPI >= TM) glds16_nt(src, dst);  // wave-uniform: a W row instruction
    else glds16(src, dst);
  };
  auto issue = [&](int c, int buf) {
#pragma unroll
    for (int ins = 0; ins < IPW; ++ins) dma(dma_src(c, ins), buf, ins);
  };
  static_assert(!ILV || (BK == 32 && IPW <= 16), "interleaved DMA issue: BK 32, at most one DMA per k-step");
  constexpr bool elu = MODE == 2;  // compile-time: an if-converted ELU costs ~250 VALU per chunk
  floatx16 acc[TMW][TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.f;
  const int arow = 32 * TMW * wm + r, brow = TM + 32 * TNW * wn + r;
  for (int d = 0; d < DIST; ++d)
    if (cb + d < ce) issue(cb + d, d);
  for (int c = cb; c < ce; ++c) {
    {  // chunk c landed for this wave once only the younger chunks' DMAs remain outstanding
      const int younger = min(DIST - 1, ce - 1 - c);
      if (younger >= 2) PTTS_WAIT_VM(2 * IPW);
      else if (younger == 1) PTTS_WAIT_VM(IPW);
      else PTTS_WAIT_VM(0);
    }
    // every wave's DMAs of chunk c have landed, and every wave is done with chunk c-1's buffer,
    // which the DMA issued next (chunk c+DIST) overwrites
    __syncthreads();
    const bool pf = c + DIST < ce;
    const int pc = c + DIST, pbuf = (c + DIST - cb) % NBUF;
    if (!ILV && pf) issue(pc, pbuf);
    // ILV: the next chunk's DMA sources are formed here, ahead of this chunk's fragment reads, and
    // pinned (an empty asm that rewrites them), so no address arithmetic lands between the MFMAs:
    // with it there, the compiler reused the registers of queued MFMAs' operands for the address
    // (v_lshl_add_u64 right behind the MFMA that reads it) and tiles came out wrong
    const float* nsrc[IPW];
    if (ILV) {
#pragma unroll
      for (int ins = 0; ins < IPW; ++ins) {
        nsrc[ins] = dma_src(pf ? pc : c, ins);
        asm volatile("" : "+v"(nsrc[ins]));
      }
    }
    {
      const int buf = (c - cb) % NBUF;
#pragma unroll
      for (int half = 0; half < BK / 32; ++half) {
        float af[TMW][16], bf[TNW][16];
#pragma unroll
        for (int ii = 0; ii < TMW; ++ii) {
          const int row = arow + 32 * ii;
          const float* la = lds + buf * BUF + row * BK;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int lc = 8 * half + 4 * h + i;
            const float4 x = *reinterpret_cast<const float4*>(la + 4 * (lc ^ swz<BK>(row)));
            af[ii][4 * i + 0] = x.x; af[ii][4 * i + 1] = x.y; af[ii][4 * i + 2] = x.z; af[ii][4 * i + 3] = x.w;
          }
          if (elu) {
#pragma unroll
            for (int j = 0; j < 16; ++j) af[ii][j] = elu1(af[ii][j]);
          }
        }
#pragma unroll
        for (int jj = 0; jj < TNW; ++jj) {
          const int row = brow + 32 * jj;
          const float* lb = lds + buf * BUF + row * BK;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int lc = 8 * half + 4 * h + i;
            const float4 y = *reinterpret_cast<const float4*>(lb + 4 * (lc ^ swz<BK>(row)));
            bf[jj][4 * i + 0] = y.x; bf[jj][4 * i + 1] = y.y; bf[jj][4 * i + 2] = y.z; bf[jj][4 * i + 3] = y.w;
          }
        }
        if (BF16) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            bf16x8 ab[TMW], bb[TNW];
#pragma unroll
            for (int ii = 0; ii < TMW; ++ii) {
              floatx8 v;
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = af[ii][8 * q + j];
              ab[ii] = __builtin_convertvector(v, bf16x8);
            }
#pragma unroll
            for (int jj = 0; jj < TNW; ++jj) {
              floatx8 v;
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = bf[jj][8 * q + j];
              bb[jj] = __builtin_convertvector(v, bf16x8);
            }
#pragma unroll
            for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
              for (int jj = 0; jj < TNW; ++jj)
                acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab[ii], bb[jj], acc[ii][jj], 0, 0, 0);
          }
          if (ILV && pf) {
#pragma unroll
            for (int ins = 0; ins < IPW; ++ins) dma(nsrc[ins], pbuf, ins);
          }
        } else if (X6) {
          const float* llo = lds + buf * BUF + ROWS * BK;  // W lo rows, 16 floats (32 bf16) each
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            bf16x8 a0[TMW], a1[TMW], a2[TMW], b0[TNW], b1[TNW], b2[TNW];
#pragma unroll
            for (int ii = 0; ii < TMW; ++ii) split3_frag(&af[ii][8 * q], a0[ii], a1[ii], a2[ii]);
#pragma unroll
            for (int jj = 0; jj < TNW; ++jj) {
              hm_frag(&bf[jj][8 * q], b0[jj], b1[jj]);
              const int lrow = brow - TM + 32 * jj;
              const int lc = (2 * h + q) ^ ((lrow >> 2) & 3);
              b2[jj] = *reinterpret_cast<const bf16x8*>(llo + lrow * 16 + 4 * lc);
            }
#pragma unroll
            for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
              for (int jj = 0; jj < TNW; ++jj) {
                floatx16 t = acc[ii][jj];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[ii], b0[jj], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[ii], b1[jj], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ii], b2[jj], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[ii], b0[jj], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ii], b1[jj], t, 0, 0, 0);
                acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[ii], b0[jj], t, 0, 0, 0);
              }
            if (ILV && pf && q == 0) {  // the next chunk's DMAs between the two halves
#pragma unroll
              for (int ins = 0; ins < IPW; ++ins) dma(nsrc[ins], pbuf, ins);
            }
          }
        } else if (!(PTTS_PROBE(a) & 1)) {
#pragma unroll
          for (int j = 0; j < 16; ++j) {
#pragma unroll
            for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
              for (int jj = 0; jj < TNW; ++jj)
                acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[ii][j], bf[jj][j], acc[ii][jj], 0, 0, 0);
            if (ILV && pf && ((j + 1) * IPW) / 16 != (j * IPW) / 16) dma(nsrc[(j * IPW) / 16], pbuf, (j * IPW) / 16);
          }
        } else if (ILV && pf) {
          issue(pc, pbuf);
        }
      }
    }
  }
  if (ILV && MODE == 0 && tail_u >= 0) {
    // split tail: publish this slice's partial tile (register order, 1 KB per float4 row of the
    // wave), count in; the last of the tile's tail_S slices sums them in slice order
    const int ti = tail_u / a.tail_S, zt = tail_u % a.tail_S;
    const auto rs = sc1_rsrc(a.tail_slab + (long)ti * a.tail_S * TM * TN);
    auto off = [&](int zz, int ii, int jj, int q) {
      return (((zz * 4 + wave) * TMW * TNW + ii * TNW + jj) * 4 + q) * 1024 + 16 * lane;
    };
#pragma unroll
    for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
      for (int jj = 0; jj < TNW; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          sc1_st(rs, off(zt, ii, jj, q),
                 make_float4(acc[ii][jj][4 * q], acc[ii][jj][4 * q + 1], acc[ii][jj][4 * q + 2], acc[ii][jj][4 * q + 3]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int last;
    if (tid == 0)
      last = __hip_atomic_fetch_add(a.tickets + ti, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.tail_S - 1;
    __syncthreads();
    if (!last) return;
    if (tid == 0) __hip_atomic_store(a.tickets + ti, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the slab loads below the ticket
    // slice order: t = P0 + P1 + ... ; one slice's 4 * TMW * TNW loads in flight at a time
    float4 t[TMW][TNW][4];
#pragma unroll
    for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
      for (int jj = 0; jj < TNW; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          t[ii][jj][q] = zt == 0 ? make_float4(acc[ii][jj][4 * q], acc[ii][jj][4 * q + 1], acc[ii][jj][4 * q + 2],
                                               acc[ii][jj][4 * q + 3])
                                 : sc1_ld(rs, off(0, ii, jj, q));
#pragma unroll 1
    for (int zz = 1; zz < a.tail_S; ++zz) {
      float4 v[TMW][TNW][4];
#pragma unroll
      for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
        for (int jj = 0; jj < TNW; ++jj)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[ii][jj][q] = zz == zt ? make_float4(acc[ii][jj][4 * q], acc[ii][jj][4 * q + 1], acc[ii][jj][4 * q + 2],
                                                  acc[ii][jj][4 * q + 3])
                                    : sc1_ld(rs, off(zz, ii, jj, q));
#pragma unroll
      for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
        for (int jj = 0; jj < TNW; ++jj)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            t[ii][jj][q].x += v[ii][jj][q].x;
            t[ii][jj][q].y += v[ii][jj][q].y;
            t[ii][jj][q].z += v[ii][jj][q].z;
            t[ii][jj][q].w += v[ii][jj][q].w;
          }
    }
#pragma unroll
    for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
      for (int jj = 0; jj < TNW; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[ii][jj][4 * q] = t[ii][jj][q].x;
          acc[ii][jj][4 * q + 1] = t[ii][jj][q].y;
          acc[ii][jj][4 * q + 2] = t[ii][jj][q].z;
          acc[ii][jj][4 * q + 3] = t[ii][jj][q].w;
        }
  }
  const bool ident = gemm_ident(a, MODE, phase);
#pragma unroll
  for (int ii = 0; ii < TMW; ++ii)
#pragma unroll
    for (int jj = 0; jj < TNW; ++jj) {
      const int tm0 = m0 + 32 * TMW * wm + 32 * ii, tn0 = n0 + 32 * TNW * wn + 32 * jj;
      if (ident && !a.partial && tm0 + 32 <= a.M && tn0 + 32 <= a.N) {
        gemm_store_tile(a, acc[ii][jj], tm0, tn0, h, r);
      } else {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int row = tm0 + (g & 3) + 8 * (g >> 2) + 4 * h;
          const int col = tn0 + r;
          if (row < a.M && col < a.N) {
            const float v = acc[ii][jj][g];
            if (a.partial) a.partial[((long)z * a.M + row) * a.N + col] = v;
            else gemm_store(a, row, col, phase, ident, v);
          }
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Register-blocked K-split GEMM: each wave accumulates a (32*TM) x (32*TN) block (TM*TN
// 32x32 accumulators); one A fragment feeds TN MFMAs and one B fragment TM, so operand bytes per
// flop fall to (TM+TN)/(2*TM*TN) of the 32x32 tile's. The 4 waves split the K chunks of the
// workgroup tile and are summed through LDS; loads run one chunk ahead in an exit-free loop.
// LAYOUT 18: 32x64 per workgroup (TM 1, TN 2), 19: 64x32 (2, 1), 20: 64x64 (2, 2).
// ---------------------------------------------------------------------------------------------
template <int MODE, int TM, int TN>
__global__ __launch_bounds__(256) void k_gemm_rb(GemmArgs a) {
  if (a.back_hi) back_prio();
  __shared__ float red[4 * 16 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  int bx, by;
  xcd_tile(a, true, bx, by);
  const int n0 = bx * 32 * TN, m0 = by * 32 * TM, z = blockIdx.z;
  const int nchunks = a.K >> 5;
  int cb = 0, ce = nchunks, phase = 0;
  if (MODE == 0) {
    cb = (int)((long)nchunks * z / a.S);
    ce = (int)((long)nchunks * (z + 1) / a.S);
  } else {
    phase = z;
  }
  const float* wrow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = min(n0 + 32 * j + r, a.Nw - 1);
    wrow[j] = a.W + (long)phase * a.w_phase_stride + (long)n * a.K + 16 * h;
  }
  const float* xrow[TM];
  const float *xb[TM], *hb[TM];
  int qs[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mm = min(m0 + 32 * i + r, a.M - 1);  // rows past M only feed unstored outputs
    if (MODE == 0) {
      xrow[i] = a.X + (long)mm * a.ldx + 16 * h;
    } else {
      const int bq = mm / a.Tq;
      qs[i] = (mm - bq * a.Tq) * a.stride_in - a.P;
      xb[i] = a.X + (long)bq * a.T_in * a.ldx + 16 * h;
      hb[i] = a.H + ((long)bq * a.P + a.P) * a.cin + 16 * h;
    }
  }
  auto a_ptr = [&](int i, int k0) -> const float* {
    if (MODE == 0) return xrow[i] + k0;
    const int j = k0 / a.cin;
    const int ci = k0 - j * a.cin;
    const int t = qs[i] + j;
    const float* px = xb[i] + t * a.ldx + ci;
    const float* ph = hb[i] + t * a.cin + ci;
    return t >= 0 ? px : ph;
  };
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.f;
  constexpr bool elu = MODE == 2;  // compile-time: an if-converted ELU costs ~250 VALU per chunk
  auto load = [&](int cc, float4 (&A)[TM][4], float4 (&Bv)[TN][4]) {
    if (PTTS_PROBE(a) & 2) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) A[i][q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) Bv[j][q] = make_float4(0.f, 0.f, 0.f, 0.f);
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* ap = a_ptr(i, cc << 5);
#pragma unroll
      for (int q = 0; q < 4; ++q) A[i][q] = *reinterpret_cast<const float4*>(ap + 4 * q);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) Bv[j][q] = *reinterpret_cast<const float4*>(wrow[j] + (cc << 5) + 4 * q);
  };
  auto mma = [&](float4 (&A)[TM][4], float4 (&Bv)[TN][4]) {
    float af[TM][16], bf[TN][16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        af[i][4 * q] = A[i][q].x; af[i][4 * q + 1] = A[i][q].y; af[i][4 * q + 2] = A[i][q].z; af[i][4 * q + 3] = A[i][q].w;
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bf[j][4 * q] = Bv[j][q].x; bf[j][4 * q + 1] = Bv[j][q].y; bf[j][4 * q + 2] = Bv[j][q].z; bf[j][4 * q + 3] = Bv[j][q].w;
      }
    }
    if (elu) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) af[i][k] = elu1(af[i][k]);
    }
    if (PTTS_PROBE(a) & 1) return;
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][k], bf[j][k], acc[i][j], 0, 0, 0);
  };
  float4 a0[TM][4], b0[TN][4], a1[TM][4], b1[TN][4];
  {
    const int c = cb + wave;
    const int n = c < ce ? (ce - c + 3) / 4 : 0;
    const int clast = c + (n - 1) * 4;
    auto chunk = [&](int i) { return i < n ? c + i * 4 : clast; };
    if (n > 0) {
      load(c, a0, b0);
      int i = 0;
      for (; i + 2 <= n; i += 2) {
        load(chunk(i + 1), a1, b1);
        mma(a0, b0);
        load(chunk(i + 2), a0, b0);
        mma(a1, b1);
      }
      if (i < n) mma(a0, b0);
    }
  }
  // K-split sum over the 4 waves, one 32x32 accumulator at a time through LDS
  const bool ident = gemm_ident(a, MODE, phase);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (i + j > 0) __syncthreads();
#pragma unroll
      for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[i][j][g];
      __syncthreads();
      float vs[4];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int g = wave * 4 + gg;
        float v = red[(0 * 16 + g) * 64 + lane] + red[(1 * 16 + g) * 64 + lane];
        v += red[(2 * 16 + g) * 64 + lane];
        v += red[(3 * 16 + g) * 64 + lane];
        vs[gg] = v;
      }
      if (ident && !a.partial && m0 + 32 * i + 32 <= a.M && n0 + 32 * j + 32 <= a.N) {
        gemm_store_fast<4>(a, vs, wave * 4, m0 + 32 * i, n0 + 32 * j, h, r);
        continue;
      }
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int g = wave * 4 + gg;
        const int row = m0 + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
        const int col = n0 + 32 * j + r;
        if (row >= a.M || col >= a.N) continue;
        if (a.partial) {
          a.partial[((long)z * a.M + row) * a.N + col] = vs[gg];
          continue;
        }
        gemm_store(a, row, col, phase, ident, vs[gg]);
      }
    }
}

// ---------------------------------------------------------------------------------------------
// int8-weight split-K GEMM for the FlowLM step under weight_quant. The weights hold the
// reference's simulated quantization (QuantizedTensor::quantize, quantize.rs:66-90: data =
// clamp(round(x/scale)) * scale, in f32), so the f32 weight is rebuilt per element as
// float(q) * scale[n] - bit-for-bit the value the reference multiplies with - and only the
// int8 code is streamed from HBM: 4x fewer weight bytes on the weight-bound skinny GEMMs.
// Structure of LAYOUT 0: 4 waves on one 32 x (32*TN) tile, the tile's K chunks dealt
// round-robin to the waves (one chunk in flight ahead of the MFMAs), partial tiles summed
// through LDS into split-K slab z. Lane (r, h) reads the 16 codes k0+16h..+15 of row
// n0+32t+r with one 16-byte load; each A fragment feeds TN MFMAs.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float i8_to_f(unsigned d, int b) { return (float)((int)(d << (24 - 8 * b)) >> 24); }

template <int TN>
__global__ __launch_bounds__(256) void k_gemm_w8(GemmArgs a) {
  __shared__ float red[4 * 16 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32 * TN, m0 = blockIdx.y * 32, z = blockIdx.z;
  const int nchunks = a.K >> 5;
  const int cb = (int)((long)nchunks * z / a.S), ce = (int)((long)nchunks * (z + 1) / a.S);
  // rows past M / N are clamped to valid ones: their results are never stored
  const float* xrow = a.X + (long)min(m0 + r, a.M - 1) * a.ldx + 16 * h;
  const int8_t* wrow[TN];
  float sc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = min(n0 + 32 * t + r, a.N - 1);
    wrow[t] = a.Wq + (long)n * a.K + 16 * h;
    sc[t] = a.wscale[n];
  }
  floatx16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[t][g] = 0.f;

  auto load = [&](int cc, float4 (&A)[4], uint4 (&Q)[TN]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) A[i] = *reinterpret_cast<const float4*>(xrow + (cc << 5) + 4 * i);
#pragma unroll
    for (int t = 0; t < TN; ++t) Q[t] = *reinterpret_cast<const uint4*>(wrow[t] + (cc << 5));
  };
  auto mma = [&](float4 (&A)[4], uint4 (&Q)[TN]) {
    float af[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[4 * i + 0] = A[i].x; af[4 * i + 1] = A[i].y; af[4 * i + 2] = A[i].z; af[4 * i + 3] = A[i].w;
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const unsigned d[4] = {Q[t].x, Q[t].y, Q[t].z, Q[t].w};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float w = i8_to_f(d[j >> 2], j & 3) * sc[t];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], w, acc[t], 0, 0, 0);
      }
    }
  };
  float4 a0[4], a1[4];
  uint4 q0[TN], q1[TN];
  const int c = cb + wave;
  const int n = c < ce ? (ce - c + 3) / 4 : 0;
  const int clast = c + (n - 1) * 4;
  auto chunk = [&](int i) { return i < n ? c + i * 4 : clast; };
  if (n > 0) {
    load(c, a0, q0);
    int i = 0;
    for (; i + 2 <= n; i += 2) {
      load(chunk(i + 1), a1, q1);
      mma(a0, q0);
      load(chunk(i + 2), a0, q0);
      mma(a1, q1);
    }
    if (i < n) mma(a0, q0);
  }
#pragma unroll
  for (int t = 0; t < TN; ++t) {
#pragma unroll
    for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[t][g];
    __syncthreads();
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int g = wave * 4 + gg;
      const float v = red[g * 64 + lane] + red[(16 + g) * 64 + lane] + red[(32 + g) * 64 + lane] +
                      red[(48 + g) * 64 + lane];
      const int row = m0 + (g & 3) + 8 * (g >> 2) + 4 * h;
      const int col = n0 + 32 * t + r;
      if (row < a.M && col < a.N) a.partial[((long)z * a.M + row) * a.N + col] = v;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_quant_codes(const float* W, const float* s, int N, int K, int8_t* q,
                                                     int* bad) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * K) return;
  const float sc = s[i / K], w = W[i];
  float c = sc > 0.f ? rintf(w / sc) : 0.f;
  c = fminf(fmaxf(c, -127.f), 127.f);
  q[i] = (int8_t)c;
  if (sc > 0.f && c * sc != w) atomicAdd(bad, 1);
}

void quant_codes(const float* W, const float* s, int N, int K, int8_t* q, int* bad, hipStream_t st) {
  const long n = (long)N * K;
  hipLaunchKernelGGL(k_quant_codes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, W, s, N, K, q, bad);
}

// ---------------------------------------------------------------------------------------------
// fp8 W8A8 split-K GEMM for the FlowLM step (ptts_engine_config.fp8_gemm; BASELINE configs[4]
// "fp8 MFMA GEMM path"). Not a reference numeric: the reference has no fp8 (quantize.rs is a
// simulated int8 grid), so this path is gated on accuracy against the f32 oracle.
//   W: OCP e4m3 codes [N][K], one scale per row (fp8_codes). A: the workgroup's K slice of its
//   32 rows is loaded once, each row's max |a| over the slice sets its scale (max/448), and the
//   e4m3 codes go to LDS. v_mfma_f32_32x32x16_fp8_fp8 then runs the slice: lane (r, h) supplies
//   the 16 bytes at k 32c+16h..+15 of A row r and of W row n as two 8-byte operands (A and B see
//   the same k permutation, so the dot products are unchanged). Products of two e4m3 values are
//   exact in f32; the slab value is acc * sa[row] * sw[col]. 4 waves deal the slice's 32-wide
//   chunks round-robin (W loads one chunk ahead) and are summed through LDS as in k_gemm_w8.
// ---------------------------------------------------------------------------------------------
constexpr int F8_LDA = FP8_KSLICE_MAX + 16;  // LDS row stride (bytes): 16-B skew between rows

template <int TN>
__global__ __launch_bounds__(256) void k_gemm_fp8(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char sa8[32 * F8_LDA];
  __shared__ float sas[32];
  __shared__ float red[4 * 16 * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32 * TN, m0 = blockIdx.y * 32, z = blockIdx.z;
  const int nchunks = a.K >> 5;
  const int cb = (int)((long)nchunks * z / a.S), ce = (int)((long)nchunks * (z + 1) / a.S);
  const int ks = 32 * (ce - cb);  // slice length (<= FP8_KSLICE_MAX, host-checked)
  // ---- A slice: 8 threads per row, float4 j*8 + part; row max over the slice; e4m3 codes to LDS
  {
    const int row = tid >> 3, part = tid & 7;
    const bool live = m0 + row < a.M;
    const float* xr = a.X + (long)min(m0 + row, a.M - 1) * a.ldx + 32 * cb;
    constexpr int NJ = FP8_KSLICE_MAX / 32;
    float4 v[NJ];
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (live && 32 * j < ks) v[j] = *reinterpret_cast<const float4*>(xr + 4 * (8 * j + part));
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[j].x), fabsf(v[j].y)), fmaxf(fabsf(v[j].z), fabsf(v[j].w))));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
    const float inv = mx > 0.f ? 448.f / mx : 0.f;
    if (part == 0) sas[row] = mx / 448.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (32 * j < ks) {
        int q = __builtin_amdgcn_cvt_pk_fp8_f32(v[j].x * inv, v[j].y * inv, 0, false);
        q = __builtin_amdgcn_cvt_pk_fp8_f32(v[j].z * inv, v[j].w * inv, q, true);
        *reinterpret_cast<int*>(&sa8[row * F8_LDA + 4 * (8 * j + part)]) = q;
      }
    }
  }
  __syncthreads();
  const uint8_t* wrow[TN];
  float sc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = min(n0 + 32 * t + r, a.N - 1);
    wrow[t] = a.Wf8 + (long)n * a.K + 16 * h;
    sc[t] = a.wscale[n];
  }
  floatx16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[t][g] = 0.f;
  auto load = [&](int cc, uint4 (&Q)[TN]) {
#pragma unroll
    for (int t = 0; t < TN; ++t) Q[t] = *reinterpret_cast<const uint4*>(wrow[t] + (cc << 5));
  };
  auto mma = [&](int cc, uint4 (&Q)[TN]) {
    const uint4 A = *reinterpret_cast<const uint4*>(&sa8[r * F8_LDA + 32 * (cc - cb) + 16 * h]);
    const long a0 = (long)(((unsigned long)A.y << 32) | A.x), a1 = (long)(((unsigned long)A.w << 32) | A.z);
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const long b0 = (long)(((unsigned long)Q[t].y << 32) | Q[t].x);
      const long b1 = (long)(((unsigned long)Q[t].w << 32) | Q[t].z);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a0, b0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a1, b1, acc[t], 0, 0, 0);
    }
  };
  uint4 q0[TN], q1[TN];
  const int c = cb + wave;
  const int n = c < ce ? (ce - c + 3) / 4 : 0;
  const int clast = c + (n - 1) * 4;
  auto chunk = [&](int i) { return i < n ? c + i * 4 : clast; };
  if (n > 0) {
    load(c, q0);
    int i = 0;
    for (; i + 2 <= n; i += 2) {
      load(chunk(i + 1), q1);
      mma(chunk(i), q0);
      load(chunk(i + 2), q0);
      mma(chunk(i + 1), q1);
    }
    if (i < n) mma(chunk(i), q0);
  }
#pragma unroll
  for (int t = 0; t < TN; ++t) {
#pragma unroll
    for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[t][g];
    __syncthreads();
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int g = wave * 4 + gg;
      const float v = red[g * 64 + lane] + red[(16 + g) * 64 + lane] + red[(32 + g) * 64 + lane] +
                      red[(48 + g) * 64 + lane];
      const int row = (g & 3) + 8 * (g >> 2) + 4 * h;
      const int col = n0 + 32 * t + r;
      if (m0 + row < a.M && col < a.N) a.partial[((long)z * a.M + m0 + row) * a.N + col] = v * sas[row] * sc[t];
    }
    __syncthreads();
  }
}

// One workgroup per weight row: s = max|W[n][:]| / 448 (1 for an all-zero row), codes e4m3(W / s)
__global__ __launch_bounds__(256) void k_fp8_codes(const float* W, int K, uint8_t* q, float* s) {
  __shared__ float sh[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float* w = W + (long)n * K;
  float mx = 0.f;
  for (int k = 4 * tid; k < K; k += 1024) {
    const float4 v = *reinterpret_cast<const float4*>(w + k);
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) sh[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  const float sc = mx > 0.f ? mx / 448.f : 1.f, inv = 1.f / sc;
  if (tid == 0) s[n] = sc;
  for (int k = 4 * tid; k < K; k += 1024) {
    const float4 v = *reinterpret_cast<const float4*>(w + k);
    int c = __builtin_amdgcn_cvt_pk_fp8_f32(v.x * inv, v.y * inv, 0, false);
    c = __builtin_amdgcn_cvt_pk_fp8_f32(v.z * inv, v.w * inv, c, true);
    *reinterpret_cast<int*>(q + (long)n * K + k) = c;
  }
}

void fp8_codes(const float* W, int N, int K, uint8_t* q, float* s, hipStream_t st) {
  hipLaunchKernelGGL(k_fp8_codes, dim3((unsigned)N), dim3(256), 0, st, W, K, q, s);
}

// xcd_pn of a tile grid gx x gy (see xcd_tile): the split of the 8 XCDs over N and M tiles that
// moves the fewest operand bytes through the L2s, (8/pn) * |W| + pn * |A|; 0 when none divides.
static int choose_xcd_pn(const GemmArgs& a, int gx, int gy) {
  if (((long)gx * gy) % 8) return 0;
  const double wb = (double)a.N * a.K;
  const double ab = a.mode == 0 ? (double)a.M * a.K : (double)(a.M / a.Tq) * a.T_in * a.cin;
  int best = 0;
  double bc = 0;
  for (int pn : {8, 4, 2, 1}) {
    const int pm = 8 / pn;
    if (gx % pn || gy % pm) continue;
    const double c = pm * wb + pn * ab;
    if (!best || c < bc) best = pn, bc = c;
  }
  return best;
}
#ifdef PTTS_PROBES
static bool rr4_off() {  // PTTS_NO_RR4: the back part's 512-wide reduces one row per workgroup (A/B)
  static const bool v = getenv("PTTS_NO_RR4") != nullptr;
  return v;
}
static int back_probe() {
  static const int p = getenv("PTTS_BACK_PROBE") ? atoi(getenv("PTTS_BACK_PROBE")) : 0;
  return p;
}
static int front_probe() {  // the same probe on every uncapped launch (front part, prefill, ...)
  static const int p = getenv("PTTS_FRONT_PROBE") ? atoi(getenv("PTTS_FRONT_PROBE")) : 0;
  return p;
}
#else
static constexpr bool rr4_off() { return false; }
#endif
template <typename K>
static void launch_tiled(K kernel, dim3 grid, int threads, hipStream_t s, const GemmArgs& a) {
  GemmArgs b = a;
  b.xcd_pn = choose_xcd_pn(a, (int)grid.x, (int)grid.y);
  b.back_hi = g_back_hi;
#ifdef PTTS_PROBES
  b.probe = g_wg_cap > 0 ? back_probe() : front_probe();  // the cap is set exactly while the back part is captured
#endif
  hipLaunchKernelGGL(kernel, grid, dim3(threads), cap_lds(kernel, std::max(a.max_wg_per_cu, g_wg_cap)), s, b);
}

// Split tail (GemmArgs::tail_S): whole rounds of the CUs' workgroup slots (256 CUs x MINB) run
// whole tiles; the remaining tiles are cut into tail_S K slices that run as the last round.
static constexpr int NUM_CUS = 256;
template <typename K>
static void launch_split_tail(K kernel, int TM, int TN, int minb, hipStream_t s, const GemmArgs& a) {
  GemmArgs b = a;
  b.tiles_n = (a.N + TN - 1) / TN;
  const int tiles_m = (a.M + TM - 1) / TM, tiles = b.tiles_n * tiles_m, slots = NUM_CUS * minb;
  b.tail_full = tiles / slots * slots;
  const int rem = tiles - b.tail_full;
  if (rem == 0) {  // whole rounds: every workgroup takes a whole tile, the ordinary 2-D grid
    b.tail_S = 0;
    launch_tiled(kernel, dim3((unsigned)b.tiles_n, (unsigned)tiles_m, 1), 256, s, b);
    return;
  }
  b.tail_S = std::min(b.tail_S, a.K / 32);
  while (b.tail_S > 1 && (long)rem * b.tail_S * TM * TN > a.tail_cap) --b.tail_S;  // scratch-bound
  if (b.tail_S <= 1) {
    b.tail_S = 0;
    launch_tiled(kernel, dim3((unsigned)b.tiles_n, (unsigned)tiles_m, 1), 256, s, b);
    return;
  }
  if (rem > a.tickets_cap || !a.tail_slab || !a.tickets || a.S != 1)
    throw std::runtime_error("gemm: split tail needs its slab and tickets and S == 1");
  b.xcd_pn = 0;
  hipLaunchKernelGGL(kernel, dim3((unsigned)(b.tail_full + rem * b.tail_S)), dim3(256),
                     cap_lds(kernel, a.max_wg_per_cu), s, b);
}

template <int MODE>
static void gemm_launch(const GemmArgs& a, int grid_z, hipStream_t s) {
  switch (a.layout) {
#define PTTS_GLDS(L, WM_, WN_, BK_, NB_)                                                               \
  case L:                                                                                               \
    launch_tiled((k_gemm_glds<MODE, WM_, WN_, BK_, NB_>),                                              \
                 dim3((a.N + 32 * WN_ - 1) / (32 * WN_), (a.M + 32 * WM_ - 1) / (32 * WM_), grid_z), 256, s, a); \
    return;
    // the product's layouts (engine.cpp: linear_split, back_tile); the rest are compiled only into
    // -DPTTS_PROBES builds (tools/, PTTS_OVR sweeps)
    PTTS_GLDS(6, 2, 2, 32, 2)
    PTTS_GLDS(7, 1, 4, 32, 2)
    PTTS_GLDS(14, 4, 1, 32, 4)
#ifdef PTTS_PROBES
    PTTS_GLDS(8, 2, 2, 64, 2)
    PTTS_GLDS(11, 2, 2, 32, 3)
    PTTS_GLDS(12, 2, 2, 32, 4)
    PTTS_GLDS(13, 1, 4, 32, 4)
    PTTS_GLDS(15, 2, 2, 64, 3)
    PTTS_GLDS(16, 1, 4, 64, 3)
#endif
#undef PTTS_GLDS
#define PTTS_GLRB(L, WM_, WN_, NB_, TMW_, TNW_)                                                       \
  case L:                                                                                             \
    launch_tiled((k_gemm_glds<MODE, WM_, WN_, 32, NB_, TMW_, TNW_>),                                   \
                 dim3((a.N + 32 * WN_ * TNW_ - 1) / (32 * WN_ * TNW_),                                \
                      (a.M + 32 * WM_ * TMW_ - 1) / (32 * WM_ * TMW_), grid_z), 256, s, a);            \
    return;
    // register-blocked LDS-DMA tiles (per-wave TMW x TNW accumulators)
    PTTS_GLRB(23, 2, 2, 3, 2, 1)  // 128 x  64
#ifdef PTTS_PROBES
    PTTS_GLRB(21, 2, 2, 3, 2, 2)  // 128 x 128
    PTTS_GLRB(22, 2, 2, 3, 1, 2)  //  64 x 128
    PTTS_GLRB(24, 4, 1, 3, 2, 1)  // 256 x  32
    PTTS_GLRB(25, 4, 1, 3, 1, 2)  // 128 x  64 (waves stacked in M)
    PTTS_GLRB(26, 2, 2, 4, 2, 2)  // 128 x 128, 4 buffers
    PTTS_GLRB(27, 1, 4, 3, 2, 1)  //  64 x 128 (waves side by side in N)
#endif
#undef PTTS_GLRB
#define PTTS_GLX(L, WM_, WN_, NB_, TMW_, TNW_, MINB_)                                                 \
  case L:                                                                                             \
    if (MODE == 0 && a.tail_S > 0) {                                                                  \
      launch_split_tail((k_gemm_glds<MODE, WM_, WN_, 32, NB_, TMW_, TNW_, MINB_, true>),               \
                        32 * WM_ * TMW_, 32 * WN_ * TNW_, MINB_, s, a);                                \
      return;                                                                                         \
    }                                                                                                 \
    launch_tiled((k_gemm_glds<MODE, WM_, WN_, 32, NB_, TMW_, TNW_, MINB_, true>),                      \
                 dim3((a.N + 32 * WN_ * TNW_ - 1) / (32 * WN_ * TNW_),                                \
                      (a.M + 32 * WM_ * TMW_ - 1) / (32 * WM_ * TMW_), grid_z), 256, s, a);            \
    return;
    // interleaved DMA issue (ILV)
    PTTS_GLX(32, 2, 2, 3, 1, 1, 2)  //  64 x  64, 2 per CU (back part)
    PTTS_GLX(34, 2, 2, 3, 2, 1, 1)  // 128 x  64 (prefill linear1)
    PTTS_GLX(35, 2, 2, 2, 2, 1, 2)  // 128 x  64, 2 per CU (prefill)
#ifdef PTTS_PROBES
    PTTS_GLX(30, 2, 2, 3, 2, 2, 1)  // 128 x 128
    PTTS_GLX(31, 2, 2, 2, 2, 2, 2)  // 128 x 128, 2 per CU
    PTTS_GLX(33, 2, 2, 2, 1, 1, 2)  //  64 x  64, 2 buffers, 2 per CU
    PTTS_GLX(36, 2, 2, 3, 1, 2, 1)  //  64 x 128
    PTTS_GLX(37, 2, 2, 4, 1, 1, 1)  //  64 x  64, 4 buffers
    PTTS_GLX(38, 2, 2, 4, 2, 2, 1)  // 128 x 128, 4 buffers
    PTTS_GLX(39, 2, 2, 3, 1, 2, 2)  //  64 x 128, 2 per CU
#endif
#undef PTTS_GLX
    // bf16 operands (GemmArgs layout + 100; engine back_bf16): the ILV tiles of the back part
#define PTTS_GLB(L, WM_, WN_, NB_, TMW_, TNW_, MINB_)                                                 \
  case 100 + L:                                                                                       \
    launch_tiled((k_gemm_glds<MODE, WM_, WN_, 32, NB_, TMW_, TNW_, MINB_, true, 1>),                   \
                 dim3((a.N + 32 * WN_ * TNW_ - 1) / (32 * WN_ * TNW_),                                \
                      (a.M + 32 * WM_ * TMW_ - 1) / (32 * WM_ * TMW_), grid_z), 256, s, a);            \
    return;
    PTTS_GLB(32, 2, 2, 3, 1, 1, 2)  //  64 x  64, 2 per CU
    PTTS_GLB(35, 2, 2, 2, 2, 1, 2)  // 128 x  64, 2 per CU
    PTTS_GLB(31, 2, 2, 2, 2, 2, 2)  // 128 x 128, 2 per CU
#ifdef PTTS_PROBES
    PTTS_GLB(30, 2, 2, 3, 2, 2, 1)  // 128 x 128
    PTTS_GLB(36, 2, 2, 3, 1, 2, 1)  //  64 x 128
    PTTS_GLB(39, 2, 2, 3, 1, 2, 2)  //  64 x 128, 2 per CU
#endif
#undef PTTS_GLB
    // bf16x6 f32 (GemmArgs layout + 200; engine back_mfma = PTTS_BACK_F32X6): W pre-split (Whm, Wlo)
#define PTTS_GLX6(L, WM_, WN_, NB_, TMW_, TNW_, MINB_)                                                \
  case 200 + L:                                                                                       \
    if (!a.Whm || !a.Wlo) throw std::runtime_error("gemm: bf16x6 layout without its split weights"); \
    launch_tiled((k_gemm_glds<MODE, WM_, WN_, 32, NB_, TMW_, TNW_, MINB_, true, 2>),                   \
                 dim3((a.N + 32 * WN_ * TNW_ - 1) / (32 * WN_ * TNW_),                                \
                      (a.M + 32 * WM_ * TMW_ - 1) / (32 * WM_ * TMW_), grid_z), 256, s, a);            \
    return;
    PTTS_GLX6(32, 2, 2, 3, 1, 1, 2)  //  64 x  64, 2 per CU
    PTTS_GLX6(36, 2, 2, 3, 1, 2, 1)  //  64 x 128
    PTTS_GLX6(39, 2, 2, 3, 1, 2, 2)  //  64 x 128, 2 per CU
    PTTS_GLX6(35, 2, 2, 2, 2, 1, 2)  // 128 x  64, 2 per CU
    PTTS_GLX6(31, 2, 2, 2, 2, 2, 2)  // 128 x 128, 2 per CU
    PTTS_GLX6(30, 2, 2, 3, 2, 2, 1)  // 128 x 128
#undef PTTS_GLX6
    default:
      break;
  }
  switch (a.layout) {
    case 0:
      launch_tiled((k_gemm<MODE, 0>), dim3((a.N + 31) / 32, (a.M + 31) / 32, grid_z), 256, s, a);
      return;
    case 9:
      launch_tiled((k_gemm<MODE, 9>), dim3((a.N + 31) / 32, (a.M + 31) / 32, grid_z), 512, s, a);
      return;
    case 18:
      launch_tiled((k_gemm_rb<MODE, 1, 2>), dim3((a.N + 63) / 64, (a.M + 31) / 32, grid_z), 256, s, a);
      return;
    case 20:
      launch_tiled((k_gemm_rb<MODE, 2, 2>), dim3((a.N + 63) / 64, (a.M + 63) / 64, grid_z), 256, s, a);
      return;
#ifdef PTTS_PROBES
    case 4:
      hipLaunchKernelGGL((k_gemm_lds<MODE, 0>), dim3((a.N + 31) / 32, (a.M + 31) / 32, grid_z), dim3(256), 0, s,
                         a);
      return;
    case 5:
      hipLaunchKernelGGL((k_gemm_lds<MODE, 1>), dim3((a.N + 63) / 64, (a.M + 63) / 64, grid_z), dim3(256), 0, s,
                         a);
      return;
    case 1:
      launch_tiled((k_gemm<MODE, 1>), dim3((a.N + 63) / 64, (a.M + 63) / 64, grid_z), 256, s, a);
      return;
    case 2:
      launch_tiled((k_gemm<MODE, 2>), dim3((a.N + 127) / 128, (a.M + 31) / 32, grid_z), 256, s, a);
      return;
    case 3:
      launch_tiled((k_gemm<MODE, 3>), dim3((a.N + 31) / 32, (a.M + 127) / 128, grid_z), 256, s, a);
      return;
    case 19:
      launch_tiled((k_gemm_rb<MODE, 2, 1>), dim3((a.N + 31) / 32, (a.M + 63) / 64, grid_z), 256, s, a);
      return;
    case 10:
      launch_tiled((k_gemm<MODE, 10>), dim3((a.N + 31) / 32, (a.M + 31) / 32, grid_z), 256, s, a);
      return;
    case 17:
      launch_tiled((k_gemm<MODE, 17>), dim3((a.N + 31) / 32, (a.M + 31) / 32, grid_z), 512, s, a);
      return;
#endif
    default:
      throw std::runtime_error("gemm: tile layout " + std::to_string(a.layout) + " is not in this build");
  }
}

// split3 (kernels.h): round-to-nearest-even pieces, each remainder exact in f32
__global__ __launch_bounds__(256) void k_split3(const float* __restrict__ W, long n, unsigned* __restrict__ hm,
                                                unsigned short* __restrict__ lo) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float x = W[i];
    const __bf16 p0 = (__bf16)x;
    const float r = x - (float)p0;
    const __bf16 p1 = (__bf16)r;
    const __bf16 p2 = (__bf16)(r - (float)p1);
    hm[i] = (unsigned)__builtin_bit_cast(unsigned short, p0) << 16 | __builtin_bit_cast(unsigned short, p1);
    lo[i] = __builtin_bit_cast(unsigned short, p2);
  }
}
void split3(const float* W, long n, unsigned* hm, unsigned short* lo, hipStream_t s) {
  const long blocks = std::min<long>((n + 255) / 256, 4096);
  if (blocks > 0) hipLaunchKernelGGL(k_split3, dim3((unsigned)blocks), dim3(256), 0, s, W, n, hm, lo);
}

void gemm(const GemmArgs& a, int grid_z, hipStream_t s) {
  if (a.Wf8) {  // fp8 W8A8: 32x64 tiles
    hipLaunchKernelGGL((k_gemm_fp8<2>), dim3((a.N + 63) / 64, (a.M + 31) / 32, grid_z), dim3(256), 0, s, a);
    return;
  }
  if (a.Wq) {  // int8 weights: 32x64 tiles
    hipLaunchKernelGGL((k_gemm_w8<2>), dim3((a.N + 63) / 64, (a.M + 31) / 32, grid_z), dim3(256), 0, s, a);
    return;
  }
  // MODE 1 = implicit-GEMM conv, MODE 2 = the same with ELU applied to A on load
  if (a.mode == 0) gemm_launch<0>(a, grid_z, s);
  else if (a.elu_in) gemm_launch<2>(a, grid_z, s);
  else gemm_launch<1>(a, grid_z, s);
}

// =============================================================================================
// Skinny split-K GEMM with register-resident weights (see kernels.h). Packed layout, per
// (tile t, slice z, wave w): NV = kw / 8 groups of 64 float4, group j lane l = W[n][k..k+3] with
//   n = t * 32 * WN + (w % WN) * 32 + (l & 31),  k = z * ks + (w / WN) * kw + (l >> 5) * kw / 2 + 4 j,
// so lane l holds the B operand of v_mfma_f32_32x32x2f32 for the steps s = 0 .. kw/2 - 1 of its
// wave, k = base + (l >> 5) * kw / 2 + s (the two lane halves take the two k of a step from the two
// halves of the wave's k range: the MFMA K order is a permutation of the sum). A (X's slice) is
// read from LDS in the same order: lane l, row l & 31, the same k.
// =============================================================================================
__global__ void k_pack_gemv(const float* __restrict__ W, int N, int K, int wn, int kw, float* __restrict__ P) {
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index into P
  const long total4 = (long)N * K / 4;
  if (i4 >= total4) return;
  const int nv = kw / 8, ks = kw * (4 / wn), S = K / ks;
  const int lane = (int)(i4 & 63);
  long r = i4 >> 6;
  const int j = (int)(r % nv);
  r /= nv;
  const int w = (int)(r & 3);
  r >>= 2;
  const int z = (int)(r % S);
  const int t = (int)(r / S);
  const int n = t * 32 * wn + (w % wn) * 32 + (lane & 31);
  const int k = z * ks + (w / wn) * kw + (lane >> 5) * (kw / 2) + 4 * j;
  reinterpret_cast<float4*>(P)[i4] = *reinterpret_cast<const float4*>(W + (long)n * K + k);
}

// int8 weight codes (engines with weight_quant): code word -> the f32 weight quad float(q) * s
__device__ __forceinline__ float4 q8_quad(unsigned q, float sc) {
  return make_float4((float)(int)(signed char)(q & 0xff) * sc, (float)(int)(signed char)((q >> 8) & 0xff) * sc,
                     (float)(int)(signed char)((q >> 16) & 0xff) * sc, (float)((int)q >> 24) * sc);
}

// fp8 A operand: 8 f32 values * inv -> 8 e4m3 bytes (one MFMA operand)
__device__ __forceinline__ long f8_pack8(const float* v, float inv) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
  return (long)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ long u32x2_long(unsigned lo, unsigned hi) {
  return (long)(((unsigned long)hi << 32) | lo);
}

// WQ: the weight form. 0 f32 fragments; 1 int8 codes of a quantized matrix (weight_quant: widened
// to the same f32 weights in registers); 2 e4m3 codes (fp8_gemm, W8A8: {4, 128} tiles only) - the
// 32 rows of the X slice quantized to e4m3 with one scale per (row, slice) = max |x| / 448 (every
// wave computes the same scales from the LDS slice), v_mfma_f32_32x32x16_fp8_fp8 over the slice
// (lane (r, h) supplies k 64 h + 8 s .. + 7 of step s for A and B alike), slab = acc * sa * sw.
template <int WN, int KW, int WQ = 0>
__global__ __launch_bounds__(256) void k_gemv(const float* __restrict__ X, long ldx, int M, int N,
                                              const float* __restrict__ P, float* __restrict__ partial,
                                              const uint32_t* __restrict__ P8, const float* __restrict__ scale) {
  static_assert(WQ != 2 || (WN == 4 && KW == 128), "fp8 gemv: {4, 128} tiles");
  constexpr bool Q8 = WQ == 1;
  front_prio();
  constexpr int WK = 4 / WN, KS = KW * WK, NV = KW / 8, LDA = KS + 4;  // +4: conflict-free b128 rows
  __shared__ __attribute__((aligned(16))) float sA[32 * LDA];
  __shared__ __attribute__((aligned(16))) float red[WK > 1 ? 4 * 16 * 64 : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = blockIdx.x, z = blockIdx.y, S = gridDim.y, m0 = 32 * blockIdx.z;  // z: K slice; blockIdx.z: 32-row block
  // X's slice first (the LDS fill waits only for these loads), then every weight load
  constexpr int AV = 32 * KS / 4 / 256;  // float4 of X per thread
  float4 av[AV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int e = tid + 256 * i, row = e / (KS / 4), c4 = e % (KS / 4);
    av[i] = m0 + row < M ? *reinterpret_cast<const float4*>(X + (long)(m0 + row) * ldx + (long)z * KS + 4 * c4)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* wp = reinterpret_cast<const f4v*>(P) + (((long)t * S + z) * 4 + wave) * NV * 64 + lane;
  f4v w[WQ ? 1 : NV];
  u32x4 wq[WQ ? NV / 4 : 1];
  const int m = lane & 31, h = lane >> 5, wn = wave % WN, wk = wave / WN;
  const int n = t * 32 * WN + wn * 32 + m;
  if (WQ) {  // codes: NV / 4 16-B loads per lane (pack_q8 order)
    const u32x4* qp = reinterpret_cast<const u32x4*>(P8) + (((long)t * S + z) * 4 + wave) * (NV / 4) * 64 + lane;
#pragma unroll
    for (int j = 0; j < NV / 4; ++j)
      wq[j] = (front_skip() & 1) ? u32x4{0u, 0u, 0u, 0u} : __builtin_nontemporal_load(qp + j * 64);
  } else {
#pragma unroll
    for (int j = 0; j < NV; ++j)
      w[j] = (front_skip() & 1) ? f4v{0.f, 0.f, 0.f, 0.f} : __builtin_nontemporal_load(wp + j * 64);  // once-read
  }
  const float sc = WQ ? scale[n] : 0.f;
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int e = tid + 256 * i, row = e / (KS / 4), c4 = e % (KS / 4);
    *reinterpret_cast<float4*>(&sA[row * LDA + 4 * c4]) = av[i];
  }
  __syncthreads();
  const float* ar = &sA[m * LDA + wk * KW + h * (KW / 2)];
  floatx16 acc;
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;
  if (WQ == 2) {  // ---- fp8 W8A8: this lane's 64 values of row m, the row scale, 8 fp8 MFMAs
    float xv[KW / 2];
#pragma unroll
    for (int j = 0; j < KW / 8; ++j) {
      const float4 a = *reinterpret_cast<const float4*>(ar + 4 * j);
      xv[4 * j] = a.x, xv[4 * j + 1] = a.y, xv[4 * j + 2] = a.z, xv[4 * j + 3] = a.w;
    }
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < KW / 2; ++j) mx = fmaxf(mx, fabsf(xv[j]));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float inv = mx > 0.f ? 448.f / mx : 0.f, sa = mx / 448.f;
#pragma unroll
    for (int st = 0; st < KW / 16; ++st) {
      const long a8 = f8_pack8(&xv[8 * st], inv);
      const u32x4 q = wq[st >> 1];
      const long b8 = (st & 1) ? u32x2_long(q[2], q[3]) : u32x2_long(q[0], q[1]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a8, b8, acc, 0, 0, 0);
    }
    // slab value acc * sa(row) * sw(column): the row of register g is (g & 3) + 8 (g >> 2) + 4 h
    float* out = partial + (long)z * M * N;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int rl = (g & 3) + 8 * (g >> 2) + 4 * h, row = m0 + rl;
      const float sar = __shfl(sa, rl, 64);
      if (row < M) out[(long)row * N + n] = acc[g] * sar * sc;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    if (front_skip() & 2) break;
    const float4 a = *reinterpret_cast<const float4*>(ar + 4 * j);
    float4 b;
    if (Q8) b = q8_quad(wq[j / 4][j % 4], sc);
    else b = make_float4(w[j].x, w[j].y, w[j].z, w[j].w);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
  }
  float* out = partial + (long)z * M * N;
  if (WK == 1) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int row = m0 + (g & 3) + 8 * (g >> 2) + 4 * h;
      if (row < M) out[(long)row * N + n] = acc[g];
    }
    return;
  }
  // WK > 1: the WK waves of column block c (waves c, c + WN, ..) hold partials over their k
  // ranges; the 16 * WN (block, register) outputs are dealt 4 * WN per wave and summed in k order
#pragma unroll
  for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[g];
  __syncthreads();
#pragma unroll
  for (int ff = 0; ff < 4 * WN; ++ff) {
    const int f = wave * 4 * WN + ff, c = f / 16, g = f % 16;
    float v = red[(c * 16 + g) * 64 + lane];
#pragma unroll
    for (int kk = 1; kk < WK; ++kk) v += red[((kk * WN + c) * 16 + g) * 64 + lane];
    const int row = m0 + (g & 3) + 8 * (g >> 2) + 4 * h;
    if (row < M) out[(long)row * N + t * 32 * WN + c * 32 + m] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Whole-K skinny GEMM (kernels.h gemv_fk). Fragment orders, K = 1024, wave w (0..7) covering
// k = 128 w .. 128 w + 127, lane l = 16 g + c (g = l >> 4 the lane group, c = l & 15):
//   A: lane (g, r) of row tile t holds k = 128 w + 32 g + s, s = 0..31, for row 16 t + r, as 8 float4
//      j = s / 4: float4 index ((w * 2 + t) * 8 + j) * 64 + l  (FK_A_FLOATS floats for 32 rows)
//   W: lane (g, c) of column tile n0 / 16 holds k = 128 w + 32 g + s of column n0 + c:
//      float4 index ((n0 / 16 * 8 + w) * 8 + j) * 64 + l
// MFMA step s (16x16x4, lane group g supplies the step's k index g) sums k = 128 w + 32 g + s over
// g for both operands alike: each wave's 128 k are covered once (a permutation of the order).
__device__ __forceinline__ long fk_afrag_index(int row, int k) {  // float index into the A fragment
  const int w = k >> 7, g = (k >> 5) & 3, s = k & 31, t = row >> 4, r = row & 15;
  return ((((long)(w * 2 + t) * 8 + (s >> 2)) * 64 + (g * 16 + r)) << 2) + (s & 3);
}
__global__ void k_pack_gemv_fk(const float* __restrict__ W, int N, int K, float* __restrict__ P) {
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i4 >= (long)N * K / 4) return;
  const int l = (int)(i4 & 63), j = (int)((i4 >> 6) & 7), w = (int)((i4 >> 9) & 7);
  const int ct = (int)(i4 >> 12);
  const int n = ct * 16 + (l & 15), k = w * 128 + (l >> 4) * 32 + 4 * j;
  reinterpret_cast<float4*>(P)[i4] = *reinterpret_cast<const float4*>(W + (long)n * K + k);
}
__global__ __launch_bounds__(512) void k_gemv_fk(const float* __restrict__ A, int M, int N,
                                                 const float* __restrict__ P, const float* __restrict__ bias,
                                                 int act, float* __restrict__ Y, long ldy) {
  front_prio();
  __shared__ __attribute__((aligned(16))) float red[8 * 2 * 4 * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = blockIdx.x;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* wp = reinterpret_cast<const f4v*>(P) + ((long)(ct * 8 + w) * 8) * 64 + lane;
  const f4v* ap = reinterpret_cast<const f4v*>(A) + ((long)(w * 2) * 8) * 64 + lane;
  f4v b[8], a0[8], a1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    b[j] = (front_skip() & 1) ? f4v{0.f, 0.f, 0.f, 0.f} : __builtin_nontemporal_load(wp + j * 64);  // once-read
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a0[j] = ap[j * 64];
    a1[j] = ap[(8 + j) * 64];
  }
  // every load in flight before the first MFMA (the scheduler otherwise sinks them next to their
  // use: a few loads in flight at a time, one round trip each)
  __builtin_amdgcn_sched_barrier(0);
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (front_skip() & 2) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j][e], b[j][e], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j][e], b[j][e], c1, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[((w * 2 + 0) * 4 + i) * 64 + lane] = c0[i];
    red[((w * 2 + 1) * 4 + i) * 64 + lane] = c1[i];
  }
  __syncthreads();
  // thread tid: row tile t, register i, lane ll (C map: column ll & 15, row (ll >> 4) * 4 + i)
  const int t = tid >> 8, i = (tid >> 6) & 3, ll = tid & 63;
  float v = red[((0 * 2 + t) * 4 + i) * 64 + ll];
#pragma unroll
  for (int ww = 1; ww < 8; ++ww) v += red[((ww * 2 + t) * 4 + i) * 64 + ll];
  const int row = 16 * t + (ll >> 4) * 4 + i, col = ct * 16 + (ll & 15);
  if (row < M) {
    if (bias) v += bias[col];
    if (act == ACT_GELU) v = gelu_tanh(v);
    Y[(long)row * ldy + col] = v;
  }
}

bool gemv_fk_supported(int M, int N, int K) { return M >= 1 && M <= 32 && K == FK_K && N % 16 == 0; }

void pack_gemv_fk(const float* W, int N, int K, float* packed, hipStream_t s) {
  if (!gemv_fk_supported(1, N, K)) throw std::runtime_error("pack_gemv_fk: unsupported shape");
  const long total4 = (long)N * K / 4;
  hipLaunchKernelGGL(k_pack_gemv_fk, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, W, N, K, packed);
}

void gemv_fk(const float* Afrag, int M, int N, const float* packed, const float* bias, int act, float* Y, long ldy,
             hipStream_t s) {
  if (!gemv_fk_supported(M, N, FK_K) || (act != ACT_NONE && act != ACT_GELU))
    throw std::runtime_error("gemv_fk: unsupported shape");
  hipLaunchKernelGGL(k_gemv_fk, dim3((unsigned)(N / 16)), dim3(512), cap_lds(k_gemv_fk, g_wg_cap), s, Afrag, M, N,
                     packed, bias, act, Y, ldy);
}

// ---------------------------------------------------------------------------------------------
// Fused FlowLM feed-forward of a step pass (kernels.h ffn_fused). Workgroup L (512 threads) is
// member i of group z, with all 16 members of a group on one XCD when workgroups are dealt to the
// XCDs round-robin (speed only: the hand-off is coherent across XCDs). Linear2 fragments (packed
// by pack_ffn2), float4 index (((z * 16 + i) * 8 + w) * 8 + j) * 64 + l: lane l of wave w holds
// W2[n][k .. k + 3], n = 64 i + 32 (w & 1) + (l & 31), k = 256 z + 64 (w >> 1) + 32 (l >> 5) + 4 j:
// the B operand of v_mfma_f32_32x32x2f32 for the wave's 32 steps (k-half l >> 5 as in k_gemv).
// The hand-off region of group z holds linear1's 32 x 256 outputs in the matching A order: float4
// (q * 8 + j) * 64 + l = U[row l & 31][64 q + 32 (l >> 5) + 4 j .. + 3].
// ---------------------------------------------------------------------------------------------
template <int NG>
__global__ void k_pack_ffn2(const float* __restrict__ W, float* __restrict__ P) {
  constexpr int MB = 256 / NG, CT = 1024 / MB / 32;  // members per group, 32-column tiles per member
  const long f = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index into P
  if (f >= 1024L * 4096 / 4) return;
  const int l = (int)(f & 63), j = (int)((f >> 6) & 7), w = (int)((f >> 9) & 7);
  const long r = f >> 12;
  const int i = (int)(r % MB), z = (int)(r / MB);
  const int n = (1024 / MB) * i + 32 * (w % CT) + (l & 31), k = (4096 / NG) * z + 64 * (w / CT) + 32 * (l >> 5) + 4 * j;
  reinterpret_cast<float4*>(P)[f] = *reinterpret_cast<const float4*>(W + (long)n * 4096 + k);
}

// WQ as k_gemv: 0 f32, 1 int8 codes widened to f32, 2 e4m3 codes W8A8 on the fp8 MFMA - linear1:
// each wave quantizes its two 16-row A tiles over its 128 k (one scale per (row, wave), max |a| /
// 448 over the 4 lane groups of the row) and runs v_mfma_f32_16x16x32_fp8_fp8 (lane group g
// supplies k 128 w + 32 g + 8 s .. + 7 of step s for A and B alike); linear2: each wave its 32 rows
// over its 64-k part (lanes r, r + 32), v_mfma_f32_32x32x16_fp8_fp8; a wave's partial tile is
// scaled by its row scales before the cross-wave sums, the column scale applied after them.
template <int NG, int WQ = 0>
__global__ __launch_bounds__(512) void k_ffn_fused(const float* __restrict__ A, int M, const float* __restrict__ P1,
                                                   const float* __restrict__ P2, float* __restrict__ hand, int set,
                                                   float* __restrict__ P, int* err, const uint32_t* __restrict__ Q1,
                                                   const float* __restrict__ s1, const uint32_t* __restrict__ Q2,
                                                   const float* __restrict__ s2) {
  constexpr int MB = 256 / NG;        // members per group
  constexpr int CT = 1024 / MB / 32;  // linear2 32-column tiles per member
  constexpr int KG = 4096 / NG;       // linear2 K slice of a group = linear1 columns of the group
  front_prio();
  __shared__ __attribute__((aligned(16))) float red[8 * 16 * 64];  // phase 1: 8 x 2 x 4 x 64; phase 2: all
  __shared__ __attribute__((aligned(16))) float sU[32 * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = blockIdx.x;
  int z, i;  // group (linear2 slice), member
  if (NG == 16) {  // a group's 16 members on one XCD (workgroups dealt round-robin; speed only)
    const int x = L & 7, jj = L >> 3;
    z = 2 * x + (jj >> 4);
    i = jj & 15;
  } else {  // contiguous members: progress needs only one group co-resident
    z = L / MB;
    i = L % MB;
  }
  const int ct = MB * z + i;  // linear1 column tile: columns 16 ct .. 16 ct + 15
  typedef float f4v __attribute__((ext_vector_type(4)));
  // every operand that does not depend on the hand-off, requested up front: linear1's weight and
  // A fragments (as k_gemv_fk), then linear2's weight fragment (used after the hand-off)
  const f4v* wp = reinterpret_cast<const f4v*>(P1) + ((long)(ct * 8 + w) * 8) * 64 + lane;
  const f4v* ap = reinterpret_cast<const f4v*>(A) + ((long)(w * 2) * 8) * 64 + lane;
  const f4v* w2p = reinterpret_cast<const f4v*>(P2) + ((long)((z * MB + i) * 8 + w) * 8) * 64 + lane;
  constexpr bool Q8 = WQ != 0;
  f4v b[Q8 ? 1 : 8], a0[8], a1[8], b2[Q8 ? 1 : 8];
  u32x4 q1[Q8 ? 2 : 1], q2[Q8 ? 2 : 1];
  if (Q8) {  // int8 / e4m3 codes (pack_q8 order): two 16-B loads per lane and matrix
    const u32x4* q1p = reinterpret_cast<const u32x4*>(Q1) + ((long)(ct * 8 + w) * 2) * 64 + lane;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      q1[j] = (front_skip() & 1) ? u32x4{0u, 0u, 0u, 0u} : __builtin_nontemporal_load(q1p + j * 64);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      b[j] = (front_skip() & 1) ? f4v{0.f, 0.f, 0.f, 0.f} : __builtin_nontemporal_load(wp + j * 64);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a0[j] = ap[j * 64];
    a1[j] = ap[(8 + j) * 64];
  }
  if (Q8) {
    const u32x4* q2p = reinterpret_cast<const u32x4*>(Q2) + ((long)((z * MB + i) * 8 + w) * 2) * 64 + lane;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      q2[j] = (front_skip() & 1) ? u32x4{0u, 0u, 0u, 0u} : __builtin_nontemporal_load(q2p + j * 64);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      b2[j] = (front_skip() & 1) ? f4v{0.f, 0.f, 0.f, 0.f} : __builtin_nontemporal_load(w2p + j * 64);
  }
  // row scales of this lane's linear1 column and linear2 column (int8 codes)
  const float sc1 = Q8 ? s1[ct * 16 + (lane & 15)] : 0.f;
  const float sc2 = Q8 ? s2[(1024 / MB) * i + 32 * (w % CT) + (lane & 31)] : 0.f;
  __builtin_amdgcn_sched_barrier(0);
  // ---- linear1 + GELU (k_gemv_fk): two 16-row tiles, the 8 waves' partial tiles summed in LDS
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  if (WQ == 2) {
    float x0[32], x1[32];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) x0[4 * j + e] = a0[j][e], x1[4 * j + e] = a1[j][e];
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) m0 = fmaxf(m0, fabsf(x0[j])), m1 = fmaxf(m1, fabsf(x1[j]));
    m0 = fmaxf(m0, __shfl_xor(m0, 16, 64));
    m0 = fmaxf(m0, __shfl_xor(m0, 32, 64));
    m1 = fmaxf(m1, __shfl_xor(m1, 16, 64));
    m1 = fmaxf(m1, __shfl_xor(m1, 32, 64));
    const float i0 = m0 > 0.f ? 448.f / m0 : 0.f, i1 = m1 > 0.f ? 448.f / m1 : 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const u32x4 q = q1[st >> 1];
      const long b8 = (st & 1) ? u32x2_long(q[2], q[3]) : u32x2_long(q[0], q[1]);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(f8_pack8(&x0[8 * st], i0), b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(f8_pack8(&x1[8 * st], i1), b8, c1, 0, 0, 0);
    }
    // C register r of lane l: row (l >> 4) * 4 + r of the tile, whose scale lane that row holds
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = (lane >> 4) * 4 + r;
      c0[r] *= __shfl(m0, rl, 64) / 448.f;
      c1[r] *= __shfl(m1, rl, 64) / 448.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (front_skip() & 2) break;
      float4 bq;
      if (Q8) bq = q8_quad(q1[j / 4][j % 4], sc1);
      else bq = make_float4(b[j][0], b[j][1], b[j][2], b[j][3]);
      const float be[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j][e], be[e], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j][e], be[e], c1, 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[((w * 2 + 0) * 4 + r) * 64 + lane] = c0[r];
    red[((w * 2 + 1) * 4 + r) * 64 + lane] = c1[r];
  }
  __syncthreads();
  {  // thread tid: row tile t, register r, lane ll (C map: column ll & 15, row (ll >> 4) * 4 + r)
    const int t = tid >> 8, r = (tid >> 6) & 3, ll = tid & 63;
    float v = red[((0 * 2 + t) * 4 + r) * 64 + ll];
#pragma unroll
    for (int ww = 1; ww < 8; ++ww) v += red[((ww * 2 + t) * 4 + r) * 64 + ll];
    const int row = 16 * t + (ll >> 4) * 4 + r;
    if (WQ == 2) v *= s1[ct * 16 + (ll & 15)];  // the e4m3 weight column's scale, after the wave sums
    sU[row * 16 + (ll & 15)] = row < M ? gelu_tanh(v) : 0.f;  // rows past M: handed off as 0
  }
  __syncthreads();
  const auto hr = sc1_rsrc(hand + (long)set * FFN_HAND_FLOATS + (long)z * 32 * KG);
  if (tid < 128) {  // publish: row m, columns 4 c4 .. 4 c4 + 3 of this tile = k_local 16 i + 4 c4
    const int m = tid & 31, c4 = tid >> 5;
    const int q = i >> 2, h = (i >> 1) & 1, j = 4 * (i & 1) + c4;
    const float4 v = *reinterpret_cast<const float4*>(&sU[m * 16 + 4 * c4]);
    fh_put(hr, (((q * 8 + j) * 64) + h * 32 + m) * 16, v);
  }
  // ---- linear2, slice z: wave w = (column tile w % CT, 64-k part q = w / CT); its A fragment is
  // linear1's output of the group's members 4 q .. 4 q + 3, swept until none is empty
  const int q = w / CT;
  float4 av[8];
  bool dead = false;
  {
#pragma unroll
    for (int j = 0; j < 8; ++j) av[j] = fh_ld(hr, ((q * 8 + j) * 64 + lane) * 16);
    unsigned spins = 0;
    while (true) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < 8; ++j) ok &= !fh_empty(av[j]);
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (fh_empty(av[j])) av[j] = fh_ld(hr, ((q * 8 + j) * 64 + lane) * 16);
      if (++spins > (1u << 20)) {
        if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
        break;
      }
    }
  }
  (void)dead;
  floatx16 acc;
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;
  if (WQ == 2) {
    float xv[32];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[4 * j] = av[j].x, xv[4 * j + 1] = av[j].y, xv[4 * j + 2] = av[j].z, xv[4 * j + 3] = av[j].w;
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) mx = fmaxf(mx, fabsf(xv[j]));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float inv = mx > 0.f ? 448.f / mx : 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const u32x4 q = q2[st >> 1];
      const long b8 = (st & 1) ? u32x2_long(q[2], q[3]) : u32x2_long(q[0], q[1]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(f8_pack8(&xv[8 * st], inv), b8, acc, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] *= __shfl(mx, (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5), 64) / 448.f;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (front_skip() & 2) break;
      float4 bq;
      if (Q8) bq = q8_quad(q2[j / 4][j % 4], sc2);
      else bq = make_float4(b2[j][0], b2[j][1], b2[j][2], b2[j][3]);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].x, bq.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].y, bq.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].z, bq.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].w, bq.w, acc, 0, 0, 0);
    }
  }
  // the 8 / CT k parts of each column tile summed in k order; slab z of P
#pragma unroll
  for (int g = 0; g < 16; ++g) red[(w * 16 + g) * 64 + lane] = acc[g];
  __syncthreads();
  {
    float* out = P + (long)z * M * 1024;
#pragma unroll
    for (int rr = 0; rr < 2 * CT; ++rr) {
      const int f = tid + 512 * rr;  // (column tile c, register g, lane ll)
      const int c = f >> 10, g = (f >> 6) & 15, ll = f & 63;
      float v = red[((0 * CT + c) * 16 + g) * 64 + ll];
#pragma unroll
      for (int qq = 1; qq < 8 / CT; ++qq) v += red[((qq * CT + c) * 16 + g) * 64 + ll];
      const int row = (g & 3) + 8 * (g >> 2) + 4 * (ll >> 5);
      const int col = (1024 / MB) * i + 32 * c + (ll & 31);
      if (WQ == 2) v *= s2[col];  // the e4m3 weight column's scale, after the k-part sums
      if (row < M) out[(long)row * 1024 + col] = v;
    }
  }
  // empty this workgroup's float4s of the other set for the next launch
  if (tid < 128) {
    const int m = tid & 31, c4 = tid >> 5;
    const int qh = i >> 2, h = (i >> 1) & 1, j = 4 * (i & 1) + c4;
    const auto er = sc1_rsrc(hand + (long)(set ^ 1) * FFN_HAND_FLOATS + (long)z * 32 * KG);
    fh_st(er, (((qh * 8 + j) * 64) + h * 32 + m) * 16,
          make_float4(__uint_as_float(~0u), __uint_as_float(~0u), __uint_as_float(~0u), __uint_as_float(~0u)));
  }
}

bool ffn_fused_supported(int M, int D, int FF) { return M >= 1 && M <= 32 && D == 1024 && FF == 4096; }

void pack_ffn2(const float* W2, int groups, float* packed, hipStream_t s) {
  if (groups == 16) hipLaunchKernelGGL(k_pack_ffn2<16>, dim3(1024 * 4096 / 4 / 256), dim3(256), 0, s, W2, packed);
  else if (groups == 8) hipLaunchKernelGGL(k_pack_ffn2<8>, dim3(1024 * 4096 / 4 / 256), dim3(256), 0, s, W2, packed);
  else throw std::runtime_error("pack_ffn2: 8 or 16 groups");
}

void ffn_fused(const float* Afrag, int M, const float* P1, const float* P2, int groups, float* hand, int set, float* P,
               int* err, hipStream_t s, const uint32_t* Q1, const float* s1, const uint32_t* Q2, const float* s2,
               bool fp8) {
  if (!ffn_fused_supported(M, 1024, 4096) || (set != 0 && set != 1) || (groups != 8 && groups != 16))
    throw std::runtime_error("ffn_fused: bad shape");
  if (!Q1 != !Q2 || (Q1 && (!s1 || !s2))) throw std::runtime_error("ffn_fused: int8 codes of both matrices, with scales");
  if (Q1 && fp8 && groups == 8)
    hipLaunchKernelGGL((k_ffn_fused<8, 2>), dim3(256), dim3(512), cap_lds(k_ffn_fused<8, 2>, g_wg_cap), s, Afrag, M, P1,
                       P2, hand, set, P, err, Q1, s1, Q2, s2);
  else if (Q1 && fp8)
    throw std::runtime_error("ffn_fused: fp8 codes with 8 groups only");
  else if (Q1 && groups == 8)
    hipLaunchKernelGGL((k_ffn_fused<8, 1>), dim3(256), dim3(512), cap_lds(k_ffn_fused<8, 1>, g_wg_cap), s, Afrag, M,
                       P1, P2, hand, set, P, err, Q1, s1, Q2, s2);
  else if (Q1)
    hipLaunchKernelGGL((k_ffn_fused<16, 1>), dim3(256), dim3(512), cap_lds(k_ffn_fused<16, 1>, g_wg_cap), s,
                       Afrag, M, P1, P2, hand, set, P, err, Q1, s1, Q2, s2);
  else if (groups == 16)
    hipLaunchKernelGGL(k_ffn_fused<16>, dim3(256), dim3(512), cap_lds(k_ffn_fused<16>, g_wg_cap), s, Afrag, M, P1, P2,
                       hand, set, P, err, nullptr, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL(k_ffn_fused<8>, dim3(256), dim3(512), cap_lds(k_ffn_fused<8>, g_wg_cap), s, Afrag, M, P1, P2,
                       hand, set, P, err, nullptr, nullptr, nullptr, nullptr);
}

__global__ void k_codes_to_f32(const int8_t* __restrict__ q, long n, float* __restrict__ out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = (float)q[i];
}
void codes_to_f32(const int8_t* q, long n, float* out, hipStream_t s) {
  const long blocks = std::min<long>((n + 255) / 256, 8192);
  if (blocks > 0) hipLaunchKernelGGL(k_codes_to_f32, dim3((unsigned)blocks), dim3(256), 0, s, q, n, out);
}
__global__ void k_codes_u8_to_f32(const uint8_t* __restrict__ q, long n, float* __restrict__ out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = (float)q[i];
}
void codes_u8_to_f32(const uint8_t* q, long n, float* out, hipStream_t s) {
  const long blocks = std::min<long>((n + 255) / 256, 8192);
  if (blocks > 0) hipLaunchKernelGGL(k_codes_u8_to_f32, dim3((unsigned)blocks), dim3(256), 0, s, q, n, out);
}
__global__ void k_pack_q8(const float* __restrict__ pf, long n16, int nj, uint32_t* __restrict__ q8) {
  const long gi = (long)blockIdx.x * 256 + threadIdx.x;  // u32x4 index
  if (gi >= n16) return;
  const int l = (int)(gi & 63);
  const long q = gi >> 6;
  const int J = (int)(q % (nj / 4));
  const long P = q / (nj / 4);
  u32x4 o;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const float4 f = reinterpret_cast<const float4*>(pf)[(P * nj + 4 * J + jj) * 64 + l];
    o[jj] = ((unsigned)(int)f.x & 0xffu) | (((unsigned)(int)f.y & 0xffu) << 8) | (((unsigned)(int)f.z & 0xffu) << 16) |
            ((unsigned)(int)f.w << 24);
  }
  reinterpret_cast<u32x4*>(q8)[gi] = o;
}
void pack_q8(const float* packed_codes, long n4, int nj, uint32_t* q8, hipStream_t s) {
  if (nj % 4 != 0 || n4 % ((long)nj * 64) != 0) throw std::runtime_error("pack_q8: bad shape");
  const long n16 = n4 / 4;
  hipLaunchKernelGGL(k_pack_q8, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, packed_codes, n16, nj, q8);
}

bool gemv_supported(GemvShape g, int N, int K) {
  const bool shape = (g.wn == 4 && g.kw == 128) || (g.wn == 1 && g.kw == 32) || (g.wn == 1 && g.kw == 64) ||
                     (g.wn == 2 && g.kw == 64);
  return shape && N % (32 * g.wn) == 0 && K % g.ks() == 0 && K / g.ks() <= 16;
}

void pack_gemv(const float* W, int N, int K, GemvShape g, float* packed, hipStream_t s) {
  if (!gemv_supported(g, N, K)) throw std::runtime_error("pack_gemv: unsupported shape");
  const long total4 = (long)N * K / 4;
  hipLaunchKernelGGL(k_pack_gemv, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, W, N, K, g.wn, g.kw,
                     packed);
}

void gemv_splitk(const float* X, long ldx, int M, int N, int K, const float* packed, GemvShape g, float* partial,
                 hipStream_t s, const uint32_t* q8, const float* scale, bool fp8) {
  if (M < 1 || M > 64 || !gemv_supported(g, N, K)) throw std::runtime_error("gemv_splitk: unsupported shape");
  if (q8 && (!scale || g.kw % 32 != 0)) throw std::runtime_error("gemv_splitk: int8 codes need scales, kw % 32 == 0");
  const dim3 grid((unsigned)(N / (32 * g.wn)), (unsigned)(K / g.ks()), (unsigned)((M + 31) / 32));
#define PTTS_GEMV(WN_, KW_)                                                                              \
  if (g.wn == WN_ && g.kw == KW_) {                                                                      \
    if (q8 && fp8 && WN_ == 4 && KW_ == 128)                                                             \
      hipLaunchKernelGGL((k_gemv<4, 128, 2>), grid, dim3(256), cap_lds(k_gemv<4, 128, 2>, g_wg_cap), s, X, ldx, M, \
                         N, packed, partial, q8, scale);                                                 \
    else if (q8 && !fp8)                                                                                 \
      hipLaunchKernelGGL((k_gemv<WN_, KW_, 1>), grid, dim3(256), cap_lds(k_gemv<WN_, KW_, 1>, g_wg_cap), s, X, \
                         ldx, M, N, packed, partial, q8, scale);                                         \
    else if (q8)                                                                                         \
      throw std::runtime_error("gemv_splitk: fp8 codes on {4, 128} tiles only");                        \
    else                                                                                                 \
      hipLaunchKernelGGL((k_gemv<WN_, KW_>), grid, dim3(256), cap_lds(k_gemv<WN_, KW_>, g_wg_cap), s, X, ldx, M, \
                         N, packed, partial, nullptr, nullptr);                                          \
    return;                                                                                              \
  }
  PTTS_GEMV(4, 128)
  PTTS_GEMV(2, 64)
  PTTS_GEMV(1, 64)
  PTTS_GEMV(1, 32)
#undef PTTS_GEMV
}

// =============================================================================================
// Row reduce + epilogue + LayerNorm/modulate. One workgroup per row.
// =============================================================================================

// One workgroup per (row, 1024-column block); each thread owns 4 consecutive columns (float4).
// The S partial slabs are summed in z order (deterministic) with 4 independent loads in flight.
__device__ __forceinline__ float act1(float x, int act) {
  return act == ACT_GELU ? gelu_tanh(x) : (act == ACT_SILU ? silu(x) : (act == ACT_ELU ? elu1(x) : x));
}

// Every load of a thread (its S slab float4s and the bias / gate / residual operands) is issued
// before the first add: one memory round trip. Absent operands are read from a valid stand-in
// address and dropped by a select (no branches around loads).
template <int SMAX>
__device__ __forceinline__ float4 rr_value(const RowReduceArgs& a, int m, int n) {
  const float* p = a.P + (long)m * a.N + n;
  const long zs = (long)a.M * a.N;
  float4 pz[SMAX];
#pragma unroll
  for (int z = 0; z < SMAX; ++z) pz[z] = *reinterpret_cast<const float4*>(p + (long)min(z, a.S - 1) * zs);
  const float4 bi = *reinterpret_cast<const float4*>((a.bias ? a.bias + n : p));
  const float4 ga = *reinterpret_cast<const float4*>((a.gate ? a.gate + (long)m * a.ldg + n : p));
  const float4 rr = *reinterpret_cast<const float4*>((a.R ? a.R + (long)m * a.ldr + n : p));
  float4 v = pz[0];
#pragma unroll
  for (int z = 1; z < SMAX; ++z)
    if (z < a.S) v = f4add(v, pz[z]);
  if (a.bias) v = f4add(v, bi);
  if (a.act != ACT_NONE) v = make_float4(act1(v.x, a.act), act1(v.y, a.act), act1(v.z, a.act), act1(v.w, a.act));
  if (a.gate) v = f4mul(v, ga);
  if (a.R) v = f4add(v, rr);
  return v;
}
__device__ __forceinline__ void rr_store(const RowReduceArgs& a, int m, int n, float4 v) {
  if (a.Y) *reinterpret_cast<float4*>(a.Y + (long)m * a.ldy + n) = v;
  if (a.fhm) {  // adaLN columns [shift | scale | gate] x 6 ResBlocks, then [shift | scale] (final)
    const int st = m / a.fhm_B, b = m - st * a.fhm_B, RG = (a.fhm_B + 15) / 16;
    const int i = min(n / (3 * FH_D), FH_DEPTH), rem = n - i * 3 * FH_D;
    const int t = rem / FH_D, k = rem - t * FH_D;
    if (t < 2) {
      const long idx = (((((long)(st * RG + b / 16) * (FH_DEPTH + 1) + i) * 2 + t) * 8 + (k >> 6)) * 4 + ((k >> 4) & 3)) * 64 +
                       (b & 15) + 16 * ((k >> 2) & 3);
      reinterpret_cast<float4*>(a.fhm)[idx] = v;
    }
  }
  if (a.Y2) *reinterpret_cast<float4*>(a.Y2 + (long)m * a.ldy + n) = make_float4(elu1(v.x), elu1(v.y), elu1(v.z), elu1(v.w));
  if (a.euler) {
    float4* e = reinterpret_cast<float4*>(a.euler + (long)m * 32 + n);
    const float sc = a.euler_scale;
    float4 c = *e;
    *e = make_float4(c.x + v.x * sc, c.y + v.y * sc, c.z + v.z * sc, c.w + v.w * sc);
  }
}
// LayerNorm (+affine) (+modulate) of one row value quad, given the row mean and 1/den
__device__ __forceinline__ float4 rr_ln(const RowReduceArgs& a, int m, int n, float4 d, float den) {
  float4 hh = make_float4(d.x / den, d.y / den, d.z / den, d.w / den);
  if (a.ln_w)
    hh = f4add(f4mul(hh, *reinterpret_cast<const float4*>(a.ln_w + n)), *reinterpret_cast<const float4*>(a.ln_b + n));
  if (a.mshift) {
    const float4 sc = *reinterpret_cast<const float4*>(a.mscale + (long)m * a.ldm + n);
    const float4 sf = *reinterpret_cast<const float4*>(a.mshift + (long)m * a.ldm + n);
    hh = make_float4(hh.x * (1.0f + sc.x) + sf.x, hh.y * (1.0f + sc.y) + sf.y, hh.z * (1.0f + sc.z) + sf.z,
                     hh.w * (1.0f + sc.w) + sf.w);
  }
  return hh;
}

// Flow-head input projection of 4 columns n..n+3 of one row (cv: the row's 32 latent values),
// in one summation order for both of its callers (k_row_reduce's x0 side job, k_flow_head's
// later Euler steps); a NaN result is stored canonical (never the hand-off's empty pattern).
__device__ __forceinline__ float fh_dot4(float4 c, float4 w) { return (c.x * w.x + c.y * w.y) + (c.z * w.z + c.w * w.w); }
__device__ __forceinline__ float4 fh_inproj4(const float4 (&cv)[8], const float* in_w, const float* in_b, int n) {
  float acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float* w = in_w + (long)(n + q) * FH_L;
    float t = in_b[n + q];
#pragma unroll
    for (int j = 0; j < 8; ++j) t += fh_dot4(cv[j], *reinterpret_cast<const float4*>(w + 4 * j));
    acc[q] = t;
  }
  return make_float4(acc[0], acc[1], acc[2], acc[3]);
}

// x0 of Euler step 0 into hand-off region 0 ([RG][32][16][16] tiles; plain stores, read by the
// next launch), one output per thread i0, i0 + nthr, ...; the weight is read transposed (w_t
// [32][512], made at finalize) so each load instruction of a wave is one contiguous 256-B run
__device__ __forceinline__ void fh_x0_job(const float* cur, const float* w_t, const float* bias, float* hx, int B,
                                          long i0, long nthr) {
  for (long i = i0; i < (long)B * FH_D; i += nthr) {
    const int b = (int)(i / FH_D), n = (int)(i % FH_D);
    float t = bias[n];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 c = *reinterpret_cast<const float4*>(cur + (long)b * FH_L + 4 * j);
      const float* w = w_t + (long)(4 * j) * FH_D + n;
      t += fh_dot4(c, make_float4(w[0], w[FH_D], w[2 * FH_D], w[3 * FH_D]));
    }
    if (t != t) t = __uint_as_float(0x7FC00000u);  // never the hand-off's empty pattern
    hx[((long)((b >> 4) * 32 + (n >> 4))) * 256 + (b & 15) * 16 + (n & 15)] = t;
  }
}
__global__ void k_fh_x0(const float* cur, const float* w, const float* bias, float* hx, int B) {
  fh_x0_job(cur, w, bias, hx, B, (long)blockIdx.x * 256 + threadIdx.x, (long)gridDim.x * 256);
}
void flow_head_x0(const float* cur, const float* w_t, const float* bias, float* hx, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_fh_x0, dim3((B * FH_D + 255) / 256), dim3(256), 0, s, cur, w_t, bias, hx, B);
}

template <int SMAX>
__global__ __launch_bounds__(256) void k_row_reduce(RowReduceArgs a) {
  if (a.front) front_prio();
  __shared__ float sh[4];
  if (a.fill) {
    const long nthr = (long)gridDim.x * gridDim.y * 256;
    for (long i = ((long)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x; i < a.fill_n4; i += nthr)
      reinterpret_cast<uint4*>(a.fill)[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
  }
  if (a.x0_hx)
    fh_x0_job(a.x0_cur, a.x0_w, a.x0_b, a.x0_hx, a.x0_B, ((long)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x,
              (long)gridDim.x * gridDim.y * 256);
  const int m = blockIdx.x;
  const int n0 = blockIdx.y * 1024 + 4 * threadIdx.x;
  const bool ok = n0 < a.N;
  const int n = ok ? n0 : 0;
  const float4 v = rr_value<SMAX>(a, m, n);
  if (ok) rr_store(a, m, n, v);
  if (!a.ln) return;  // LN rows are <= 1024 wide: gridDim.y == 1 (host-checked)
  const float s = ok ? (v.x + v.y) + (v.z + v.w) : 0.f;
  const float mean = block_sum(s, sh) / (float)a.N;
  const float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
  const float q = ok ? (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w) : 0.f;
  const float den = sqrtf(block_sum(q, sh) / (float)a.N + a.eps);
  if (!ok) return;
  const float4 hv = rr_ln(a, m, n, d, den);
  *reinterpret_cast<float4*>(a.Hout + (long)m * a.ldh + n) = hv;
  if (a.Hfrag) *reinterpret_cast<float4*>(a.Hfrag + fk_afrag_index(m, n)) = hv;  // n % 4 == 0: one float4
}

// The same for the back part's 512-wide rows (Mimi d_model, SEANet conv0): FOUR rows per 512-thread
// workgroup, 128 threads per row, so a pass's 16 B rows fill the chip's one capped workgroup per
// CU in a single round instead of four (the one-row form left half of its 256 threads idle). A
// row's sums are its two waves' DPP sums, combined in LDS: the values, their order and every
// rounding are those of k_row_reduce (whose other two waves add zeros).
template <int SMAX>
__global__ __launch_bounds__(512) void k_row_reduce4(RowReduceArgs a) {
  if (a.front) front_prio();
  __shared__ float sh[2][8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = tid >> 7;
  if (!a.ln) {  // no row statistics: elementwise over the 4 rows
    const int q = a.N >> 2;  // float4 per row
    for (int e = tid; e < 4 * q; e += 512) {
      const int mm = blockIdx.x * 4 + e / q, nn = 4 * (e % q);
      if (mm < a.M) rr_store(a, mm, nn, rr_value<SMAX>(a, mm, nn));
    }
    return;
  }
  const int m = blockIdx.x * 4 + r, n = 4 * (tid & 127);
  const bool ok = m < a.M;
  const float4 v = rr_value<SMAX>(a, ok ? m : a.M - 1, n);
  if (ok) rr_store(a, m, n, v);
  const float s = wave_sum(ok ? (v.x + v.y) + (v.z + v.w) : 0.f);
  if (lane == 0) sh[0][wave] = s;
  __syncthreads();
  const float mean = (sh[0][2 * r] + sh[0][2 * r + 1]) / 512.f;
  const float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
  const float q = wave_sum(ok ? (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w) : 0.f);
  if (lane == 0) sh[1][wave] = q;
  __syncthreads();
  const float den = sqrtf((sh[1][2 * r] + sh[1][2 * r + 1]) / 512.f + a.eps);
  if (!ok) return;
  const float4 hv = rr_ln(a, m, n, d, den);
  *reinterpret_cast<float4*>(a.Hout + (long)m * a.ldh + n) = hv;
}

void row_reduce(const RowReduceArgs& a, hipStream_t s) {
  // (N = 512 only: the 2,048-wide reduce as 4 rows per workgroup, 4 float4 per thread, measured
  // slower than its one-row form, profiles/r04/row_reduce4_ab.txt)
  if (!a.front && a.N == 512 && !a.fill && !a.x0_hx && !a.fhm && !a.Hfrag && !rr4_off()) {
    const dim3 g4((a.M + 3) / 4);
    if (a.S <= 1) hipLaunchKernelGGL(k_row_reduce4<1>, g4, dim3(512), cap_lds(k_row_reduce4<1>, g_wg_cap), s, a);
    else if (a.S <= 2) hipLaunchKernelGGL(k_row_reduce4<2>, g4, dim3(512), cap_lds(k_row_reduce4<2>, g_wg_cap), s, a);
    else if (a.S <= 4) hipLaunchKernelGGL(k_row_reduce4<4>, g4, dim3(512), cap_lds(k_row_reduce4<4>, g_wg_cap), s, a);
    else if (a.S <= 8) hipLaunchKernelGGL(k_row_reduce4<8>, g4, dim3(512), cap_lds(k_row_reduce4<8>, g_wg_cap), s, a);
    else hipLaunchKernelGGL(k_row_reduce4<16>, g4, dim3(512), cap_lds(k_row_reduce4<16>, g_wg_cap), s, a);
    return;
  }
  dim3 grid(a.M, (a.N + 1023) / 1024);
  if (a.S <= 1) hipLaunchKernelGGL(k_row_reduce<1>, grid, dim3(256), cap_lds(k_row_reduce<1>, g_wg_cap), s, a);
  else if (a.S <= 2) hipLaunchKernelGGL(k_row_reduce<2>, grid, dim3(256), cap_lds(k_row_reduce<2>, g_wg_cap), s, a);
  else if (a.S <= 4) hipLaunchKernelGGL(k_row_reduce<4>, grid, dim3(256), cap_lds(k_row_reduce<4>, g_wg_cap), s, a);
  else if (a.S <= 8) hipLaunchKernelGGL(k_row_reduce<8>, grid, dim3(256), cap_lds(k_row_reduce<8>, g_wg_cap), s, a);
  else hipLaunchKernelGGL(k_row_reduce<16>, grid, dim3(256), cap_lds(k_row_reduce<16>, g_wg_cap), s, a);
}

// LayerNorm, one wave per row (N <= 1024, multiple of 64).
__global__ __launch_bounds__(256) void k_layernorm(const float* x, long ldx, float* y, long ldy, int M, int N,
                                                   const float* w, const float* b, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long)row * ldx;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = lane + 64 * i;
    v[i] = n < N ? xr[n] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float d = v[i] - mean;
    q += (lane + 64 * i < N) ? d * d : 0.f;
  }
  const float den = sqrtf(wave_sum(q) / (float)N + eps);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = lane + 64 * i;
    if (n < N) y[(long)row * ldy + n] = (v[i] - mean) / den * w[n] + b[n];
  }
}
void layernorm(const float* x, long ldx, float* y, long ldy, int M, int N, const float* w, const float* b,
               float eps, hipStream_t s) {
  hipLaunchKernelGGL(k_layernorm, dim3((M + 3) / 4), dim3(256), cap_lds(k_layernorm, g_wg_cap), s, x, ldx, y, ldy, M, N, w, b, eps);
}

// =============================================================================================
// QKV (+ split-K reduce) -> RoPE -> KV append. One thread per (row, head, rotation pair).
// =============================================================================================

__global__ __launch_bounds__(256) void k_qkv_rope(const float* P, int S, const float* dense, int M, int nh,
                                                  RowMap mp, KvStore kv, float* Q) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int per_row = nh * 32;
  if (idx >= M * per_row) return;
  const int row = idx / per_row;
  const int rem = idx - row * per_row;
  const int hh = rem >> 5, i = rem & 31;
  const int d = nh * 64, ld = 3 * d;
  const int c = hh * 64 + 2 * i;
  float q0, q1, k0, k1, v0, v1;
  if (dense) {
    const float* pr = dense + (long)row * ld;
    q0 = pr[c]; q1 = pr[c + 1]; k0 = pr[d + c]; k1 = pr[d + c + 1]; v0 = pr[2 * d + c]; v1 = pr[2 * d + c + 1];
  } else {
    q0 = q1 = k0 = k1 = v0 = v1 = 0.f;
    for (int z = 0; z < S; ++z) {
      const float* pr = P + ((long)z * M + row) * ld;
      q0 += pr[c]; q1 += pr[c + 1]; k0 += pr[d + c]; k1 += pr[d + c + 1]; v0 += pr[2 * d + c]; v1 += pr[2 * d + c + 1];
    }
  }
  int slot, pos;
  row_slot_pos(mp, row, slot, pos);
  // rope.rs:9-16 inv_freq = exp(-ln(max_period) * 2i / head_dim); ts = offset + t
  const float freq = expf((float)i * (-logf(10000.0f) * 2.0f / 64.0f));
  const float ang = (float)pos * freq;
  const float cs = cosf(ang), sn = sinf(ang);
  const long qr = mp.qrow ? mp.qrow[row] : row;  // compact admission: the query's padded row
  Q[qr * d + c] = q0 * cs - q1 * sn;
  Q[qr * d + c + 1] = q0 * sn + q1 * cs;
  if (slot < 0) return;  // padding row of a batched admission
  float* kb = kv.base + (long)slot * kv.slot_stride + ((long)hh * kv.cap + (pos % kv.cap)) * 64 + 2 * i;
  float* vb = kv.base + (long)slot * kv.slot_stride + ((long)(nh + hh) * kv.cap + (pos % kv.cap)) * 64 + 2 * i;
  kb[0] = k0 * cs - k1 * sn;
  kb[1] = k0 * sn + k1 * cs;
  vb[0] = v0;
  vb[1] = v1;
}

void qkv_rope_append(const float* P, int S, const float* dense, int M, int nh, RowMap map, KvStore kv, float* Q,
                     hipStream_t s) {
  const int total = M * nh * 32;
  hipLaunchKernelGGL(k_qkv_rope, dim3((total + 255) / 256), dim3(256), cap_lds(k_qkv_rope, g_wg_cap), s, P, S, dense, M, nh, map, kv, Q);
}

// =============================================================================================
// Attention: one workgroup per (group of <= 16 query rows of one slot, head). Keys in tiles of
// 64 are staged in LDS (K padded to 65 floats per row: conflict-free ds_read_b32 column reads),
// online softmax per row; wave w owns rows w, w+4, w+8, w+12 in both the score and PV phases.
// Mask (sdpa.rs:128-171): key kp visible to query qp iff kp <= qp and (no window or qp-kp < window).
// =============================================================================================
__global__ __launch_bounds__(256) void k_attention(const float* Q, int M, int nh, RowMap mp, KvStore kv, int window,
                                                   int qg, float* O) {
  __shared__ float sQ[16 * 64];
  __shared__ float sK[64 * 65];
  __shared__ float sV[64 * 64];
  __shared__ float sP[16 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int head = blockIdx.y;
  const int row0 = blockIdx.x * qg;
  const int nrows = min(qg, M - row0);
  int slot, qpos0, slot_l, qposl;
  row_slot_pos(mp, row0, slot, qpos0);
  row_slot_pos(mp, row0 + nrows - 1, slot_l, qposl);
  const int d = nh * 64;
  const int kmax = qposl;
  const int kmin = window > 0 ? max(0, qpos0 - window + 1) : 0;
  const float* kbase = kv.base + (long)slot * kv.slot_stride + (long)head * kv.cap * 64;
  const float* vbase = kv.base + (long)slot * kv.slot_stride + (long)(nh + head) * kv.cap * 64;

  for (int e = tid; e < 16 * 64; e += 256) {
    const int i = e >> 6, dd = e & 63;
    sQ[e] = i < nrows ? Q[(long)(row0 + i) * d + head * 64 + dd] : 0.f;
  }
  float m_run[4], l_run[4], o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m_run[r] = -INFINITY;
    l_run[r] = 0.f;
    o[r] = 0.f;
  }
  for (int kt = kmin; kt <= kmax; kt += 64) {
    __syncthreads();
    // stage K and V tiles: 64 keys x 16 float4 each
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      const int idx = tid + 256 * e4;
      const int j = idx >> 4, c4 = idx & 15;
      const int kp = kt + j;
      float4 kk = make_float4(0.f, 0.f, 0.f, 0.f), vv = kk;
      if (kp <= kmax) {
        const long off = (long)(kp % kv.cap) * 64 + c4 * 4;
        kk = *reinterpret_cast<const float4*>(kbase + off);
        vv = *reinterpret_cast<const float4*>(vbase + off);
      }
      sK[j * 65 + c4 * 4 + 0] = kk.x;
      sK[j * 65 + c4 * 4 + 1] = kk.y;
      sK[j * 65 + c4 * 4 + 2] = kk.z;
      sK[j * 65 + c4 * 4 + 3] = kk.w;
      *reinterpret_cast<float4*>(&sV[j * 64 + c4 * 4]) = vv;
    }
    __syncthreads();
    const int kp = kt + lane;
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = wave + 4 * r;
      alpha[r] = 1.f;
      if (i >= nrows) continue;  // wave-uniform
      float sc = 0.f;
#pragma unroll 16
      for (int dd = 0; dd < 64; ++dd) sc += sQ[i * 64 + dd] * sK[lane * 65 + dd];
      sc *= 0.125f;  // 1/sqrt(64) (attention.rs:191,229)
      const int qp = qpos0 + i;
      const bool ok = kp <= qp && kp <= kmax && (window <= 0 || qp - kp < window);
      sc = ok ? sc : -INFINITY;
      const float mt = wave_max(sc);
      const float mn = fmaxf(m_run[r], mt);
      float p = 0.f;
      if (mn != -INFINITY) {
        alpha[r] = (m_run[r] == -INFINITY) ? 0.f : expf(m_run[r] - mn);
        p = ok ? expf(sc - mn) : 0.f;
      }
      l_run[r] = l_run[r] * alpha[r] + wave_sum(p);
      m_run[r] = mn;
      sP[i * 64 + lane] = p;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = wave + 4 * r;
      if (i >= nrows) continue;
      float acc = 0.f;
#pragma unroll 16
      for (int j = 0; j < 64; ++j) acc += sP[i * 64 + j] * sV[j * 64 + lane];
      o[r] = o[r] * alpha[r] + acc;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = wave + 4 * r;
    if (i < nrows) O[(long)(row0 + i) * d + head * 64 + lane] = o[r] / l_run[r];
  }
}

// ---------------------------------------------------------------------------------------------
// Decode attention, one query per (row, head) (FlowLM step, attention.rs:104-283 with the
// single-query mask skip of sdpa.rs:3-18): one 256-thread workgroup per (row, head), the keys
// dealt to the 4 waves 64 at a time. Lane j owns key j of its 64-key block: the whole K row
// (16 float4) and, for P.V, lane d owns output dim d and reads V[j][d] for the block's 64 keys
// (coalesced 256-B rows) - all loads of a block are issued before any arithmetic, so each wave
// pays one memory round trip per block. p_j is broadcast with v_readlane. Waves combine their
// (max, sum, o) through LDS. Positions never wrap (max_ctx covers voice + text + frames).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_attn_decode(const float* __restrict__ Q, int nh, RowMap mp, KvStore kv,
                                                     float* __restrict__ O) {
  __shared__ float s_m[4], s_l[4], s_o[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row = blockIdx.x, head = blockIdx.y;
  int slot, qp;
  row_slot_pos(mp, row, slot, qp);
  const int d = nh * 64;
  const float* kbase = kv.base + (long)slot * kv.slot_stride + (long)head * kv.cap * 64;
  const float* vbase = kv.base + (long)slot * kv.slot_stride + (long)(nh + head) * kv.cap * 64;
  const float4* q4 = reinterpret_cast<const float4*>(Q + (long)row * d + head * 64);
  float4 q[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) q[i] = q4[i];
  float m = -INFINITY, l = 0.f, o = 0.f;
  for (int base = 64 * wave; base <= qp; base += 256) {
    const int j = base + lane;
    const bool valid = j <= qp;
    const float4* kr = reinterpret_cast<const float4*>(kbase + (long)(valid ? j : qp) * 64);
    float4 k[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) k[i] = kr[i];
    float v[64];
#pragma unroll
    for (int jj = 0; jj < 64; ++jj) v[jj] = vbase[(long)min(base + jj, qp) * 64 + lane];
    float sc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) sc += q[i].x * k[i].x + q[i].y * k[i].y + q[i].z * k[i].z + q[i].w * k[i].w;
    sc = valid ? sc * 0.125f : -INFINITY;  // 1/sqrt(64) (attention.rs:191,229)
    const float mn = fmaxf(m, wave_max(sc));  // finite: key `base` <= qp is valid
    const float alpha = expf(m - mn);         // m = -inf -> 0
    const float p = valid ? expf(sc - mn) : 0.f;
    l = l * alpha + wave_sum(p);
    o *= alpha;
    const int pb = __builtin_bit_cast(int, p);
#pragma unroll
    for (int jj = 0; jj < 64; ++jj) o += __builtin_bit_cast(float, __builtin_amdgcn_readlane(pb, jj)) * v[jj];
    m = mn;
  }
  if (lane == 0) {
    s_m[wave] = m;
    s_l[wave] = l;
  }
  s_o[wave][lane] = o;
  __syncthreads();
  if (wave == 0) {
    const float M = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float e = s_m[w] == -INFINITY ? 0.f : expf(s_m[w] - M);
      num += s_o[w][lane] * e;
      den += s_l[w] * e;
    }
    O[(long)row * d + head * 64 + lane] = num / den;
  }
}

// ---------------------------------------------------------------------------------------------
// 16-query attention on MFMA (Mimi decoder ring window: 16 upsampled positions per row, and the
// prefill / encoder groups): one workgroup per (16 consecutive rows of one slot, head), 16-key
// tiles dealt to 8 waves, online softmax per wave, waves merged through LDS.
// v_mfma_f32_16x16x4_f32 fragments (lane l, c = l & 15, G = l >> 4):
//   A[i][k] lane i + 16k, B[k][j] lane j + 16k, D reg g -> row 4G + g, col c.
// S^T = K Q^T: A = K (key c, dims 16G+s at step s), B = Q^T (query c, same dims) -> lane holds
// S[query c][key 4G+g]. O += P V: A = P (query c, key 4G+s at step s: the lane's own S^T regs,
// no transpose), B = V (key 4G+s, dim 4c+dt for output tile dt: one float4 per key) -> lane holds
// O[query 4G+g][dim 4c+dt]. The dot-product / key order permutations only reorder sums.
// ---------------------------------------------------------------------------------------------
typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr int A16_WAVES = 8;

// rope.rs:9-16: inv_freq = exp(-ln(max_period) * 2i / head_dim), angle = position * inv_freq
// (the same expressions as k_qkv_rope, so both paths rotate identically)
__device__ __forceinline__ void rope_cs(int pos, int i, float& cs, float& sn) {
  const float freq = expf((float)i * (-logf(10000.0f) * 2.0f / 64.0f));
  const float ang = (float)pos * freq;
  cs = cosf(ang);
  sn = sinf(ang);
}

// FUSE: Q is the dense QKV projection [M][3d] (Mimi decoder step) instead of rotated queries:
// the workgroup rotates its 16 rows' q and k (RoPE), appends k and v at their positions in the
// ring, and attends over the ring after a workgroup barrier (replaces the k_qkv_rope launch; the
// ring holds window + 16 positions, so the appended rows never evict a key inside the window).
template <bool RING, bool FUSE = false>
__global__ __launch_bounds__(64 * A16_WAVES) void k_attn16(const float* __restrict__ Q, int M, int nh, RowMap mp,
                                                          KvStore kv, int window, float* __restrict__ O) {
  __shared__ float s_m[A16_WAVES][16], s_l[A16_WAVES][16];
  __shared__ float s_o[A16_WAVES][16][65];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, G = lane >> 4;
  const int row0 = blockIdx.x * 16, head = blockIdx.y;
  int nrows = min(16, M - row0);
  if (mp.tab) {  // a slot's rows come first in its 16-row groups, padding rows after them
    int n = 0;
    for (int i = 0; i < nrows; ++i) n += mp.tab[row0 + i] >= 0;
    nrows = n;
  }
  if (nrows <= 0) return;  // whole group of padding (uniform over the workgroup)
  int slot, qpos0;
  row_slot_pos(mp, row0, slot, qpos0);
  const int kmax = qpos0 + nrows - 1;
  const int kmin = window > 0 ? max(0, qpos0 - window + 1) : 0;
  const int d = nh * 64;
  const KvHead kh = kv_head(kv, slot, nh, head);
  const float* kbase = kh.kb;
  const float* vbase = kh.vb;
  const int cmask = kv.cap - 1;
  auto kidx = [&](int kp) { return RING ? (kp & cmask) : kp; };
  // FlowLM prefill: keys below F come from the shared voice prefix (never in a wrapped ring)
  auto kaddr = [&](int kp) { return (FUSE || kp >= kh.F ? kbase + (long)kidx(kp) * 64 : kh.pk + (long)kp * 64); };
  auto vaddr = [&](int kp) { return (FUSE || kp >= kh.F ? vbase + (long)kidx(kp) * 64 : kh.pv + (long)kp * 64); };
  const int ntiles = (kmax - kmin + 16) / 16;
  float4 kf[4], vf[4];
  auto load = [&](int t) {
    const int kt = kmin + 16 * t;
    const float4* kr = reinterpret_cast<const float4*>(kaddr(min(kt + c, kmax)) + 16 * G);
#pragma unroll
    for (int i = 0; i < 4; ++i) kf[i] = kr[i];
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx)
      vf[sidx] = *reinterpret_cast<const float4*>(vaddr(min(kt + 4 * G + sidx, kmax)) + 4 * c);
  };
  // a wave whose first key tile holds only keys older than this step's appended rows issues its
  // loads now, so their latency overlaps the append below (the append never evicts a key of the
  // window: the ring holds window + 16 positions)
  const bool early = FUSE && wave < ntiles && kmin + 16 * wave + 15 < qpos0;
  if (early) load(wave);
  // Q^T fragment: query c (rows past nrows reuse the last row; never stored), dims 16G..16G+15
  float qf[16];
  if (FUSE) {
    const int ld = 3 * d;
    {  // append: thread (row r, rotation pair i) of the 16 x 32 (A16_WAVES = 8: 512 threads)
      const int r = threadIdx.x >> 5, i = threadIdx.x & 31;
      if (r < nrows) {
        const float* pr = Q + (long)(row0 + r) * ld + head * 64 + 2 * i;
        const float k0 = pr[d], k1 = pr[d + 1], v0 = pr[2 * d], v1 = pr[2 * d + 1];
        float cs, sn;
        rope_cs(qpos0 + r, i, cs, sn);
        float* kb = kv.base + (long)slot * kv.slot_stride + ((long)head * kv.cap + kidx(qpos0 + r)) * 64 + 2 * i;
        float* vb = kv.base + (long)slot * kv.slot_stride + ((long)(nh + head) * kv.cap + kidx(qpos0 + r)) * 64 + 2 * i;
        *reinterpret_cast<float2*>(kb) = make_float2(k0 * cs - k1 * sn, k0 * sn + k1 * cs);
        *reinterpret_cast<float2*>(vb) = make_float2(v0, v1);
      }
    }
    const int rq = min(c, nrows - 1);
    const float4* q4 = reinterpret_cast<const float4*>(Q + (long)(row0 + rq) * ld + head * 64 + 16 * G);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 t = q4[i];
      float cs, sn;
      rope_cs(qpos0 + rq, 8 * G + 2 * i, cs, sn);
      qf[4 * i] = t.x * cs - t.y * sn;
      qf[4 * i + 1] = t.x * sn + t.y * cs;
      rope_cs(qpos0 + rq, 8 * G + 2 * i + 1, cs, sn);
      qf[4 * i + 2] = t.z * cs - t.w * sn;
      qf[4 * i + 3] = t.z * sn + t.w * cs;
    }
    __syncthreads();  // the appended keys / values are read back by every wave below
  } else {
    const float4* q4 = reinterpret_cast<const float4*>(Q + (long)(row0 + min(c, nrows - 1)) * d + head * 64 + 16 * G);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 t = q4[i];
      qf[4 * i] = t.x; qf[4 * i + 1] = t.y; qf[4 * i + 2] = t.z; qf[4 * i + 3] = t.w;
    }
  }
  const int qp = qpos0 + c;  // this lane's query position (softmax side)
  float m = -INFINITY, l = 0.f;
  floatx4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (wave < ntiles && !early) load(wave);
  for (int t = wave; t < ntiles; t += A16_WAVES) {
    const int kt = kmin + 16 * t;
    float ka[16];
    float4 vc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ka[4 * i] = kf[i].x; ka[4 * i + 1] = kf[i].y; ka[4 * i + 2] = kf[i].z; ka[4 * i + 3] = kf[i].w;
      vc[i] = vf[i];
    }
    if (t + A16_WAVES < ntiles) load(t + A16_WAVES);  // next tile in flight during this one
    floatx4 st = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sidx = 0; sidx < 16; ++sidx) st = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[sidx], qf[sidx], st, 0, 0, 0);
    float sc[4];
    float mt = -INFINITY;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int kp = kt + 4 * G + g;
      const bool ok = kp <= kmax && kp <= qp && (window <= 0 || qp - kp < window);
      sc[g] = ok ? st[g] * 0.125f : -INFINITY;  // 1/sqrt(64) (attention.rs:191,229)
      mt = fmaxf(mt, sc[g]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = mn == -INFINITY ? 1.f : expf(m - mn);
    float p[4], ps = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      p[g] = sc[g] == -INFINITY ? 0.f : expf(sc[g] - mn);
      ps += p[g];
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = mn;
    // O rows are queries 4G+g: their rescale factors live in lanes 4G+g
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float a = __shfl(alpha, 4 * G + g, 64);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][g] *= a;
    }
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      o[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(p[sidx], vc[sidx].x, o[0], 0, 0, 0);
      o[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(p[sidx], vc[sidx].y, o[1], 0, 0, 0);
      o[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(p[sidx], vc[sidx].z, o[2], 0, 0, 0);
      o[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(p[sidx], vc[sidx].w, o[3], 0, 0, 0);
    }
  }
  if (G == 0) {
    s_m[wave][c] = m;
    s_l[wave][c] = l;
  }
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) s_o[wave][4 * G + g][4 * c + dt] = o[dt][g];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * 64; e += 64 * A16_WAVES) {
    const int qi = e >> 6, dd = e & 63;
    if (qi >= nrows) continue;
    float M_ = -INFINITY;
#pragma unroll
    for (int w = 0; w < A16_WAVES; ++w) M_ = fmaxf(M_, s_m[w][qi]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < A16_WAVES; ++w) {
      const float ew = s_m[w][qi] == -INFINITY ? 0.f : expf(s_m[w][qi] - M_);
      num += s_o[w][qi][dd] * ew;
      den += s_l[w][qi] * ew;
    }
    const int orow = mp.orow ? mp.orow[row0 + qi] : row0 + qi;  // compact admission: the token's row
    if (orow >= 0) O[(long)orow * d + head * 64 + dd] = num / den;
  }
}

// ---------------------------------------------------------------------------------------------
// FlowLM step attention with the QKV split-K sum, RoPE and KV append fused in front (replaces
// qkv_rope_append + k_attn_decode for the one-query-per-row step): the workgroup of (row, head)
// sums its 192 q|k|v columns over the S slabs, rotates q and k (rope.rs:18-60), appends k, v at
// the row's position and attends over the cached keys 0..pos-1 plus the new key from LDS.
// ---------------------------------------------------------------------------------------------

// Decode attention of the FlowLM step fused with the QKV slab sum, RoPE and KV append
// (attention.rs:104-283 with the single-query mask skip of sdpa.rs:3-18). One 256-thread
// workgroup per (row, head); the cached keys are dealt to the 4 waves 64 at a time.
// A 64-key block of K (and of V) is 16 KB contiguous, read with 16 fully coalesced 1-KB wave
// loads: load i gives lane l the 4 dims 4(l%16).. of key 4i + l/16. Scores: a 4-term dot with
// the matching q dims, summed over the 16-lane row with DPP, so lane l holds the score of key
// 4i + l/16 - exactly the key whose V dims it holds from V load i, so P.V needs no broadcast.
// The rows (l/16) are combined once per wave at the end. Each wave issues its first block's
// loads before the QKV/RoPE phase: the cached keys do not depend on this step's token.
template <int NW, int KQ, bool NT = false>
__global__ __launch_bounds__(64 * NW) void k_attn_decode_qkv(const float* __restrict__ P, int S, int M, int nh, RowMap mp,
                                                         KvStore kv, const float* __restrict__ rope,
                                                         float* __restrict__ O) {
  front_prio();
  constexpr int BLK = 4 * KQ * NW;  // keys per round: NW waves x KQ loads of 4 keys
  __shared__ float s_m[NW], s_l[NW];
  __shared__ __attribute__((aligned(16))) float s_o[NW][64];
  __shared__ __attribute__((aligned(16))) float s_qkv[3][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c4 = (lane & 15) * 4;  // key row within a load, first of my 4 dims
  const int row = blockIdx.x, head = blockIdx.y;
  int slot, qp;
  row_slot_pos(mp, row, slot, qp);
  // a finished row is still stepped (its frame is discarded): once it has filled the cache
  // (qp == cap) its key/value must not be appended, or position cap would spill into the next
  // head's (or, for the slot's last head, the next slot's) position 0
  const bool append = qp < kv.cap;
  qp = min(qp, kv.cap - 1);
  const int d = nh * 64, ld = 3 * d;
  const KvHead kh = kv_head(kv, slot, nh, head);
  float* kbase = kh.kb;
  float* vbase = kh.vb;
  const int last = qp - 1;
  float4 k[KQ], v[KQ];
  auto load_block = [&](int base) {
    if (front_skip() & 4) {
#pragma unroll
      for (int i = 0; i < KQ; ++i) k[i] = v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      return;
    }
    if (base < kh.F) {  // (part of) the block in the shared voice prefix: cached loads, since
                        // every row of the voice reads these lines (wave-uniform branch)
#pragma unroll
      for (int i = 0; i < KQ; ++i) {
        const int j = min(base + 4 * i + g, last);
        const long off = (long)j * 64 + c4;
        k[i] = *reinterpret_cast<const float4*>((j < kh.F ? kh.pk : kbase) + off);
        v[i] = *reinterpret_cast<const float4*>((j < kh.F ? kh.pv : vbase) + off);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < KQ; ++i) {
      const long off = (long)min(base + 4 * i + g, last) * 64 + c4;
      if (NT) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v kk = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(kbase + off));
        const f4v vv = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(vbase + off));
        k[i] = make_float4(kk.x, kk.y, kk.z, kk.w);
        v[i] = make_float4(vv.x, vv.y, vv.z, vv.w);
      } else {
        k[i] = *reinterpret_cast<const float4*>(kbase + off);
        v[i] = *reinterpret_cast<const float4*>(vbase + off);
      }
    }
  };
  int base = 4 * KQ * wave;
  if (base < qp) load_block(base);
  if (tid < 192) {  // q | k | v column of this head, summed over the slabs in z order
    const int part = tid >> 6;
    const float* pr = P + (long)row * ld + part * d + head * 64 + lane;
    s_qkv[part][lane] = slab_sum(pr, (long)M * ld, S);
  }
  __syncthreads();
  if (tid < 64) {  // rotate the (2i, 2i+1) pairs of q (tid < 32) and k (tid >= 32)
    const int i = tid & 31, part = tid >> 5;
    const float2 cssn = *reinterpret_cast<const float2*>(rope + (long)qp * 64 + 2 * i);  // table of rope_table()
    const float cs = cssn.x, sn = cssn.y;
    const float x0 = s_qkv[part][2 * i], x1 = s_qkv[part][2 * i + 1];
    const float y0 = x0 * cs - x1 * sn, y1 = x0 * sn + x1 * cs;  // one wave: all reads precede the writes
    s_qkv[part][2 * i] = y0;
    s_qkv[part][2 * i + 1] = y1;
    if (part == 1 && append) {
      kbase[(long)qp * 64 + 2 * i] = y0;
      kbase[(long)qp * 64 + 2 * i + 1] = y1;
    }
  } else if (tid < 128 && append) {
    vbase[(long)qp * 64 + lane] = s_qkv[2][lane];
  }
  __syncthreads();
  const float4 q = *reinterpret_cast<const float4*>(&s_qkv[0][c4]);
  float m = -INFINITY, l = 0.f;
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  for (; base < qp; base += BLK) {  // cached keys 0 .. qp-1, block `base` already in registers
    float sc[KQ];
    float bm = -INFINITY;
#pragma unroll
    for (int i = 0; i < KQ; ++i) {
      const float part = q.x * k[i].x + q.y * k[i].y + q.z * k[i].z + q.w * k[i].w;
      const float t = row16_sum(part) * 0.125f;  // 1/sqrt(64) (attention.rs:191,229)
      sc[i] = base + 4 * i + g <= last ? t : -INFINITY;
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
    l = l * alpha + ps;
    m = mn;
    if (base + BLK < qp) load_block(base + BLK);
  }
  // combine the 4 key rows (lanes l, l^16, l^32, l^48 hold the same dims)
  o.x += __shfl_xor(o.x, 16, 64); o.y += __shfl_xor(o.y, 16, 64);
  o.z += __shfl_xor(o.z, 16, 64); o.w += __shfl_xor(o.w, 16, 64);
  o.x += __shfl_xor(o.x, 32, 64); o.y += __shfl_xor(o.y, 32, 64);
  o.z += __shfl_xor(o.z, 32, 64); o.w += __shfl_xor(o.w, 32, 64);
  if (wave == 0) {  // the new key (position qp) from LDS
    const float sc = wave_sum(s_qkv[0][lane] * s_qkv[1][lane]) * 0.125f;
    const float mn = fmaxf(m, sc);
    const float alpha = expf(m - mn);
    const float p = expf(sc - mn);
    l = l * alpha + p;
    const float4 vn = *reinterpret_cast<const float4*>(&s_qkv[2][c4]);
    o.x = o.x * alpha + p * vn.x; o.y = o.y * alpha + p * vn.y;
    o.z = o.z * alpha + p * vn.z; o.w = o.w * alpha + p * vn.w;
    m = mn;
  }
  if (lane == 0) {
    s_m[wave] = m;
    s_l[wave] = l;
  }
  if (lane < 16) *reinterpret_cast<float4*>(&s_o[wave][c4]) = o;
  __syncthreads();
  if (wave == 0) {
    float Mx = s_m[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) Mx = fmaxf(Mx, s_m[w]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float e = s_m[w] == -INFINITY ? 0.f : expf(s_m[w] - Mx);
      num += s_o[w][lane] * e;
      den += s_l[w] * e;
    }
    O[(long)row * d + head * 64 + lane] = num / den;
  }
}

void attention_step_qkv(const float* P, int S, int M, int nh, RowMap map, KvStore kv, const float* rope, float* O,
                        hipStream_t s) {
  // 4 waves x 32 keys (128 keys per round, 133 VGPRs): in the pipelined step the front part's
  // attention shares each CU with a back-part workgroup, and this register budget keeps two of
  // its workgroups resident beside it. Steady step 0.690 -> 0.673 ms against 4 x 64 keys
  // (238 VGPRs, faster alone); 8 x 32, 4 x 48, 4 x 16, 2 x 64, 8 x 48 measured in between
  // (tools/sweep_env.sh). KV blocks are read once per step: non-temporal loads (-1.1 % step).
  hipLaunchKernelGGL((k_attn_decode_qkv<4, 8, true>), dim3(M, nh), dim3(256), 0, s, P, S, M, nh, map, kv, rope, O);
}

__global__ __launch_bounds__(256) void k_rope_table(float* tab, int npos) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)npos * 32) return;
  const int pos = (int)(idx >> 5), i = (int)(idx & 31);
  const float freq = expf((float)i * (-logf(10000.0f) * 2.0f / 64.0f));
  const float ang = (float)pos * freq;
  tab[(long)pos * 64 + 2 * i] = cosf(ang);
  tab[(long)pos * 64 + 2 * i + 1] = sinf(ang);
}

void rope_table(float* tab, int npos, hipStream_t s) {
  hipLaunchKernelGGL(k_rope_table, dim3((unsigned)((npos * 32L + 255) / 256)), dim3(256), 0, s, tab, npos);
}

void attention16_qkv(const float* qkv, int M, int nh, RowMap map, KvStore kv, int window, float* O, hipStream_t s) {
  if (map.tab != nullptr || map.rps != 16) throw std::runtime_error("attention16_qkv: needs 16 rows per slot");
  if ((kv.cap & (kv.cap - 1)) != 0 || kv.cap < window + 16)
    throw std::runtime_error("attention16_qkv: ring too small for the fused append");
  const dim3 grid((M + 15) / 16, nh);
  hipLaunchKernelGGL((k_attn16<true, true>), grid, dim3(64 * A16_WAVES), cap_lds(k_attn16<true, true>, g_wg_cap), s,
                     qkv, M, nh, map, kv, window, O);
}

void attention(const float* Q, int M, int nh, RowMap map, KvStore kv, int window, int qg, float* O, hipStream_t s) {
  if (kv.pre != nullptr && (qg != 16 || window > 0))
    throw std::runtime_error("attention: shared voice prefixes need the 16-row causal kernel");
  if (qg == 1 && window <= 0) {
    hipLaunchKernelGGL(k_attn_decode, dim3(M, nh), dim3(256), cap_lds(k_attn_decode, g_wg_cap), s, Q, nh, map, kv, O);
  } else if (qg == 16) {
    // 16-row groups never straddle slots (rows-per-slot is 16 or the whole group)
    const dim3 grid((M + 15) / 16, nh);
    if ((kv.cap & (kv.cap - 1)) == 0)
      hipLaunchKernelGGL(k_attn16<true>, grid, dim3(64 * A16_WAVES), cap_lds(k_attn16<true>, g_wg_cap), s, Q, M, nh, map, kv, window, O);
    else
      hipLaunchKernelGGL(k_attn16<false>, grid, dim3(64 * A16_WAVES), cap_lds(k_attn16<false>, g_wg_cap), s, Q, M, nh, map, kv, window, O);
  } else {
    dim3 grid((M + qg - 1) / qg, nh);
    hipLaunchKernelGGL(k_attention, grid, dim3(256), cap_lds(k_attention, g_wg_cap), s, Q, M, nh, map, kv, window, qg, O);
  }
}

// =============================================================================================
// Flow head prologue: cond_embed | out_eos reduce, EOS bookkeeping, adaLN inputs, x0 noise.
// =============================================================================================
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Standard normal for (seed, step, k, attempt): Box-Muller over two 24-bit uniforms.
__device__ float normal_at(unsigned long long seed, int step, int k, int attempt) {
  const unsigned long long base =
      mix64(seed * 0x9E3779B97F4A7C15ull + (unsigned long long)step * 0xD1B54A32D192ED03ull +
            (unsigned long long)(k * 64 + attempt) * 0x8CB92BA72F3D8DD7ull);
  const float u1 = ((float)(base >> 41) + 0.5f) * (1.0f / 8388608.0f);  // (0,1), exact in fp32
  const float u2 = (float)(mix64(base ^ 0x5851F42D4C957F2Dull) >> 40) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

__global__ __launch_bounds__(256) void k_flow_cond(const float* P, int S, int B, const float* bias, const float* temb,
                                                   int lsd, const SlotState* st, float* ysilu, float* cur,
                                                   float* eos_out) {
  front_prio();
  const int b = blockIdx.x, tid = threadIdx.x;
  const int NC = 513;  // cond_embed (512) | out_eos (1)
  // every load of the thread first (its two columns' slabs, thread 0's EOS slabs, the slot
  // state of the noise lanes), then the arithmetic: one memory round trip, not four
  const long zs = (long)B * NC;
  const float* p0 = P + (long)b * NC + tid;
  float v0[16], v1[16], ve[16];
#pragma unroll
  for (int z = 0; z < 16; ++z) {
    v0[z] = z < S ? p0[z * zs] : 0.f;
    v1[z] = z < S ? p0[z * zs + 256] : 0.f;
    ve[z] = (z < S && tid == 0) ? P[(long)b * NC + 512 + z * zs] : 0.f;
  }
  const SlotState& ss = st[b];
  const float temp = ss.temp, clamp = ss.noise_clamp;
  const unsigned long long seed = ss.seed;
  const int step = ss.step;
  const float b0 = bias[tid], b1 = bias[tid + 256], be = bias[512];
  float c0 = 0.f, c1 = 0.f, e = 0.f;
#pragma unroll
  for (int z = 0; z < 16; ++z)
    if (z < S) {
      c0 += v0[z];
      c1 += v1[z];
      e += ve[z];
    }
  c0 += b0;
  c1 += b1;
  for (int s = 0; s < lsd; ++s) {
    ysilu[((long)s * B + b) * 512 + tid] = silu(temb[s * 512 + tid] + c0);
    ysilu[((long)s * B + b) * 512 + tid + 256] = silu(temb[s * 512 + tid + 256] + c1);
  }
  if (tid == 0) eos_out[b] = e + be;  // out_eos logit (flow_lm.rs:139-145); the EOS rule runs in front_commit
  if (tid < 32) {
    float x0 = 0.f;
    if (temp > 0.f) {  // flow_lm.rs:39-65: N(0, sqrt(temp)), optionally truncated to |x| <= clamp
      const float sd = sqrtf(temp);
      x0 = sd * normal_at(seed, step, tid, 0);
      if (clamp > 0.f) {
        int att = 1;
        while (fabsf(x0) > clamp && att < 64) x0 = sd * normal_at(seed, step, tid, att++);
        x0 = fminf(fmaxf(x0, -clamp), clamp);
      }
    }
    cur[b * 32 + tid] = x0;
  }
}

void flow_cond(const float* P, int S, int B, const float* bias, const float* temb, int lsd_steps,
               const SlotState* st, float* ysilu, float* cur, float* eos_out, hipStream_t s) {
  if (S < 1 || S > FLOW_COND_MAX_SLABS) throw std::runtime_error("flow_cond: 1..16 split-K slabs");
  hipLaunchKernelGGL(k_flow_cond, dim3(B), dim3(256), 0, s, P, S, B, bias, temb, lsd_steps, st, ysilu, cur, eos_out);
}

// =============================================================================================
// Mimi front: denorm -> 1x1 quantizer -> depthwise ConvTrUpsample1d (k=32, s=16) -> LN.
// The transposed conv's overlap-add `partial` (conv.rs:202-267) equals qprev * W[:, 16 + r],
// so the kernel keeps the previous frame's quantized vector instead.
// =============================================================================================
// Denorm + quantizer 1x1 conv (mimi.rs:8-37) + depthwise ConvTrUpsample1d k32 s16
// (conv.rs:315-346: frame row r = q*w[r] + qprev*w[16+r], the overlap-add of the previous frame's
// tail) + norm1 of Mimi layer 0. One workgroup per (row b, 4 of the 16 output rows): 4x the
// workgroups of a per-row kernel, each loading only its rows' upsample taps, one LayerNorm row
// per wave. The pass's quantizer outputs go to a scratch (qprev_out [B][NFR_MAX][512]) and the commit
// moves the last valid frame's into the history, so the four workgroups of a row never race on
// it, and a row without a frame in the pass (or outside it) keeps its history unchanged.
struct QuantUpArgs {
  const float* latent[NFR_MAX];
  const FrameFlags* fl[NFR_MAX];
  int nfr;
  const float *emb_std, *emb_mean, *wq, *wup, *qprev_in;
  float* qprev_out;
  float *x, *h;
  const float *ln_w, *ln_b;
};
// grid (B, 4 nfr): rows 4 (y % 4).. of frame y / 4 of row b
__global__ __launch_bounds__(256) void k_quant_upsample(QuantUpArgs a) {
  __shared__ float sz[NFR_MAX][32];
  __shared__ float sx[4 * 512];
  const int b = blockIdx.x, f = blockIdx.y >> 2, r0 = (blockIdx.y & 3) * 4, tid = threadIdx.x;
  const int T = 16 * a.nfr;
  // every operand load of the thread's two channels is issued before the arithmetic
  float4 wqr[2][8], wur[2][2];
  float qpv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u;
#pragma unroll
    for (int i = 0; i < 8; ++i) wqr[u][i] = *reinterpret_cast<const float4*>(a.wq + c * 32 + 4 * i);
    wur[u][0] = *reinterpret_cast<const float4*>(a.wup + c * 32 + r0);
    wur[u][1] = *reinterpret_cast<const float4*>(a.wup + c * 32 + 16 + r0);
    qpv[u] = a.qprev_in[(long)b * 512 + c];
  }
  if (tid < 32 * a.nfr) {
    const int g = tid >> 5, k = tid & 31;
    sz[g][k] = a.latent[g][b * 32 + k] * a.emb_std[k] + a.emb_mean[k];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u;
    const float* wqf = reinterpret_cast<const float*>(wqr[u]);
    const float* w0 = reinterpret_cast<const float*>(&wur[u][0]);
    const float* w1 = reinterpret_cast<const float*>(&wur[u][1]);
    float q[NFR_MAX] = {};
#pragma unroll
    for (int g = 0; g < NFR_MAX; ++g)
      if (g < a.nfr) {
#pragma unroll
        for (int k = 0; k < 32; ++k) q[g] += wqf[k] * sz[g][k];
      }
    // frame f overlaps frame f - 1 (frame 0 the history); selects, no dynamic register indexing
    float cur = q[0], prev = qpv[u];
#pragma unroll
    for (int g = 1; g < NFR_MAX; ++g)
      if (f == g) cur = q[g], prev = q[g - 1];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = cur * w0[r] + prev * w1[r];
      sx[r * 512 + c] = v;
      a.x[((long)b * T + 16 * f + r0 + r) * 512 + c] = v;
    }
    if (blockIdx.y == 0) {
#pragma unroll
      for (int g = 0; g < NFR_MAX; ++g)
        if (g < a.nfr) a.qprev_out[((long)b * NFR_MAX + g) * 512 + c] = q[g];
    }
  }
  __syncthreads();
  const int lane = tid & 63, r = tid >> 6;  // one row per wave
  float v[8], sm = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = sx[r * 512 + lane + 64 * i];
    sm += v[i];
  }
  const float mean = wave_sum(sm) / 512.f;
  float qq = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) qq += (v[i] - mean) * (v[i] - mean);
  const float den = sqrtf(wave_sum(qq) / 512.f + 1e-5f);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = lane + 64 * i;
    a.h[((long)b * T + 16 * f + r0 + r) * 512 + n] = (v[i] - mean) / den * a.ln_w[n] + a.ln_b[n];
  }
}

void quant_upsample(const float* const latent[NFR_MAX], const FrameFlags* const fl[NFR_MAX], int nfr, int B, const float* emb_std,
                    const float* emb_mean, const float* wq, const float* wup, const float* qprev_in, float* qprev_out,
                    float* x, float* h, const float* ln_w, const float* ln_b, hipStream_t s) {
  if (nfr < 1 || nfr > NFR_MAX) throw std::runtime_error("quant_upsample: 1 to NFR_MAX frames");
  QuantUpArgs a{};
  for (int g = 0; g < NFR_MAX; ++g) {
    a.latent[g] = latent[g < nfr ? g : 0];
    a.fl[g] = fl[g < nfr ? g : 0];
  }
  a.nfr = nfr;
  a.emb_std = emb_std;
  a.emb_mean = emb_mean;
  a.wq = wq;
  a.wup = wup;
  a.qprev_in = qprev_in;
  a.qprev_out = qprev_out;
  a.x = x;
  a.h = h;
  a.ln_w = ln_w;
  a.ln_b = ln_b;
  hipLaunchKernelGGL(k_quant_upsample, dim3(B, 4 * nfr), dim3(256), cap_lds(k_quant_upsample, g_wg_cap), s, a);
}

// =============================================================================================
// Step commit: conv histories (last P input rows per slot), counters, next backbone input.
// =============================================================================================
// One workgroup per row: every history of the row (P x C floats each, C % 4 == 0) and its
// quantizer output, as float4 copies (the launch is one capped round: 32 workgroups, where a
// workgroup per (history, row) took two rounds of scalar copies).
__global__ __launch_bounds__(256) void k_commit(CommitArgs a) {
  const int b = blockIdx.x;
  if (a.fin_side) {  // every row (as the final conv computes every row): tile-boundary shares
    const int nx = a.fin_T / RESBLOCK_FIN_TT;
    for (int e = 2 + threadIdx.x; e < 2 * nx; e += 256)
      a.fin_pcm[(long)b * (a.fin_ld ? a.fin_ld : a.fin_T) + (e >> 1) * RESBLOCK_FIN_TT + (e & 1)] +=
          a.fin_side[(long)b * 2 * nx + e];
  }
  int nv = 0;  // valid frames: a prefix
  while (nv < a.nfr && a.flags[nv][b].valid) ++nv;
  if (nv == 0) return;
  for (int i = 0; i < a.nh; ++i) {
    const HistDesc& hd = a.h[i];
    const long n4 = (long)hd.P * hd.C / 4;
    const int tv = hd.T / a.nfr * nv;  // rows through the last valid frame
    const float4* src = reinterpret_cast<const float4*>(hd.src + ((long)b * hd.T + (tv - hd.P)) * hd.C);
    float4* dst = reinterpret_cast<float4*>(hd.dst + (long)b * hd.P * hd.C);
    if (hd.elu) {
      for (long e = threadIdx.x; e < n4; e += 256) {
        const float4 v = src[e];
        dst[e] = make_float4(elu1(v.x), elu1(v.y), elu1(v.z), elu1(v.w));
      }
    } else {
      for (long e = threadIdx.x; e < n4; e += 256) dst[e] = src[e];
    }
  }
  // the overlap-add history of the next pass: the last valid frame's quantizer output
  if (threadIdx.x < 128)
    reinterpret_cast<float4*>(a.qprev + (long)b * 512)[threadIdx.x] =
        reinterpret_cast<const float4*>(a.qcur + ((long)b * NFR_MAX + nv - 1) * 512)[threadIdx.x];
  if (threadIdx.x == 0) a.mpos[b] += 16 * nv;
}

// x[m] = lat[m] W^T (K = 32) for the 4 columns n.. of this thread, and h[m] = LN(x[m]) (eps 1e-5)
// over the 256 threads of the workgroup (one row): flow_lm.rs:117 input_linear +
// transformer.rs:66-90 norm1 of layer 0. The weight arrives transposed, Wt [32][1024], so the 64
// lanes of a wave read one contiguous 1-KB run of Wt[k] per load. lat: the row's 32 inputs.
__device__ __forceinline__ void input_ln_row(const float* lat, const float* __restrict__ Wt,
                                             const float* __restrict__ lnw, const float* __restrict__ lnb,
                                             float* __restrict__ xr, float* __restrict__ hr, float* sh) {
  const int n = 4 * threadIdx.x;  // N = 1024
  float4 lv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) lv[j] = *reinterpret_cast<const float4*>(lat + 4 * j);
  float4 wv[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) wv[k] = *reinterpret_cast<const float4*>(Wt + (long)k * 1024 + n);
  float acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // same summation order as the row-major form: ((k0 k1) + (k2 k3)) per float4
      const float a0 = lv[j].x * (&wv[4 * j].x)[q], a1 = lv[j].y * (&wv[4 * j + 1].x)[q];
      const float a2 = lv[j].z * (&wv[4 * j + 2].x)[q], a3 = lv[j].w * (&wv[4 * j + 3].x)[q];
      t += (a0 + a1) + (a2 + a3);
    }
    acc[q] = t;
  }
  const float4 v = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(xr + n) = v;
  const float mean = block_sum((v.x + v.y) + (v.z + v.w), sh) / 1024.f;
  const float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
  const float den = sqrtf(block_sum((d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w), sh) / 1024.f + 1e-5f);
  const float4 w4 = *reinterpret_cast<const float4*>(lnw + n), b4 = *reinterpret_cast<const float4*>(lnb + n);
  *reinterpret_cast<float4*>(hr + n) =
      make_float4(d.x / den * w4.x + b4.x, d.y / den * w4.y + b4.y, d.z / den * w4.z + b4.z, d.w / den * w4.w + b4.w);
}

// one 256-thread block per row: the EOS rule and frame flags (lane 0), the frame's latent, then
// the next step's x / h rows from the updated backbone input (the step's first launch, folded in)
__global__ __launch_bounds__(256) void k_front_commit(FrontCommitArgs a) {
  front_prio();
  __shared__ float s_lat[32];
  __shared__ float sh[4];
  const int b = blockIdx.x, t = threadIdx.x;
  SlotState& ss = a.st[b];
  const int valid = ss.active;
  const float e = a.eos[b];                       // loaded with `active`: one round trip
  const float cv = t < 32 ? a.cur[b * 32 + t] : 0.f;
  const float li = t < 32 ? a.lat_in[b * 32 + t] : 0.f;
  __syncthreads();  // every lane has read `active` before lane 0 updates the state
  if (t == 0) {
    FrameFlags f{0, 0};
    if (valid) {  // tts_model.rs:1055-1063 + map_while over 0..max_gen_len
      if (e > ss.eos_threshold && ss.eos_step < 0) ss.eos_step = ss.step;
      const bool tail = ss.eos_step >= 0 && ss.step >= ss.eos_step + ss.frames_after_eos;
      f.valid = 1;
      f.last = (tail || ss.step + 1 >= ss.max_frames) ? 1 : 0;
      ss.step += 1;
      a.fpos[b] += 1;
      if (f.last) ss.active = 0;
    }
    a.flags[b] = f;
    a.eos_out[b] = e;
    if (b == 0 && a.err_host)
      __hip_atomic_store(a.err_host, __hip_atomic_load(a.err_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (b == 0)
    for (int r = t; r < a.n_zero; r += 256) a.flags[a.B + r] = FrameFlags{0, 0};
  if (t < 32) {
    a.lat_out[b * 32 + t] = cv;
    if (valid) a.lat_in[b * 32 + t] = cv;
    s_lat[t] = valid ? cv : li;
  }
  if (!a.Wt) return;  // uniform
  __syncthreads();
  input_ln_row(s_lat, a.Wt, a.lnw, a.lnb, a.x + (long)b * 1024, a.h + (long)b * 1024, sh);
}

void front_commit(const FrontCommitArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_front_commit, dim3(a.B), dim3(256), 0, s, a);
}

void step_commit(const CommitArgs& a, hipStream_t s) {
  for (int i = 0; i < a.nh; ++i)
    if (a.h[i].C % 4) throw std::runtime_error("step_commit: history channels must be a multiple of 4");
  hipLaunchKernelGGL(k_commit, dim3(a.B), dim3(256), cap_lds(k_commit, g_wg_cap), s, a);
}

__global__ __launch_bounds__(256) void k_slot_reset(ResetArgs a) {
  const int i = blockIdx.x, b = blockIdx.y;
  const int slot = a.slots[i];
  if (b < a.nb) {
    float* p = a.buf[b] + (long)slot * a.per_slot[b];
    for (long e = threadIdx.x; e < a.per_slot[b]; e += 256) p[e] = 0.f;
    return;
  }
  if (threadIdx.x < 32) a.lat_in[slot * 32 + threadIdx.x] = a.bos[threadIdx.x];
  if (threadIdx.x == 0) {
    a.st[slot] = a.st_src[i];
    a.fpos[slot] = a.fpos_src[i];
    a.mpos[slot] = 0;
    for (int q = 0; q < NHB_MAX; ++q)
      if (a.flags[q]) a.flags[q][slot] = FrameFlags{0, 0};
  }
}

void slot_reset(const ResetArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_slot_reset, dim3(a.n, a.nb + 1), dim3(256), 0, s, a);
}

struct GatherArgs {
  const float* lat;
  const FrameFlags* flags;
  float* lat_out;
  FrameFlags* flags_out;
  int n;
  int idx[GATHER_MAX];
};

__global__ __launch_bounds__(64) void k_gather_preview(GatherArgs a) {
  const int i = blockIdx.x, t = threadIdx.x;
  const bool on = i < a.n;
  const int r = on ? a.idx[i] : 0;
  if (t < 32) a.lat_out[i * 32 + t] = on ? a.lat[(long)r * 32 + t] : 0.f;
  if (t == 32) a.flags_out[i] = on ? a.flags[r] : FrameFlags{0, 0};
}

void gather_preview(const float* lat, const FrameFlags* flags, const int* idx, int n, int P, float* lat_out,
                    FrameFlags* flags_out, hipStream_t s) {
  if (n < 0 || n > P || P < 1 || P > GATHER_MAX) throw std::runtime_error("gather_preview: 0 <= n <= P <= 8");
  GatherArgs a{lat, flags, lat_out, flags_out, n, {}};
  for (int i = 0; i < n; ++i) a.idx[i] = idx[i];
  hipLaunchKernelGGL(k_gather_preview, dim3(P), dim3(64), 0, s, a);
}

// =============================================================================================
// Time embeddings (once per engine / lsd_decode_steps): grid (step, embedder).
// =============================================================================================
__global__ __launch_bounds__(256) void k_time_embed(TimeEmbedWeights w, int n, float* tmp) {
  __shared__ float emb[256];
  __shared__ float h1[512];
  __shared__ float sh[4];
  const int i = blockIdx.x, e = blockIdx.y, tid = threadIdx.x;
  const float tau = (float)((double)(e == 0 ? i : i + 1) / (double)n);  // s = i/N, t = (i+1)/N
  if (tid < 128) {
    const float f = expf(-logf(10000.0f) * (float)tid / 128.0f);
    emb[tid] = cosf(tau * f);
    emb[128 + tid] = sinf(tau * f);
  }
  __syncthreads();
  for (int o = tid; o < 512; o += 256) {
    float acc = 0.f;
    for (int k = 0; k < 256; ++k) acc += w.l1w[e][o * 256 + k] * emb[k];
    h1[o] = silu(acc + w.l1b[e][o]);
  }
  __syncthreads();
  float v[2];
  for (int q = 0; q < 2; ++q) {
    const int o = tid + 256 * q;
    float acc = 0.f;
    for (int k = 0; k < 512; ++k) acc += w.l2w[e][o * 512 + k] * h1[k];
    v[q] = acc + w.l2b[e][o];
  }
  const float mean = block_sum(v[0] + v[1], sh) / 512.f;
  const float var = block_sum((v[0] - mean) * (v[0] - mean) + (v[1] - mean) * (v[1] - mean), sh) / 511.f;
  const float inv = 1.0f / sqrtf(var + 1e-5f);  // RMSNorm on unbiased variance (mlp.rs:18-26)
  for (int q = 0; q < 2; ++q) {
    const int o = tid + 256 * q;
    tmp[((long)e * n + i) * 512 + o] = v[q] * inv * w.alpha[e][o];
  }
}
__global__ void k_time_avg(const float* tmp, int n, float* out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < n * 512) out[idx] = (tmp[idx] + tmp[n * 512 + idx]) / 2.0f;
}
void time_embeddings(const TimeEmbedWeights& w, int n, float* tmp, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_time_embed, dim3(n, 2), dim3(256), 0, s, w, n, tmp);
  hipLaunchKernelGGL(k_time_avg, dim3((n * 512 + 255) / 256), dim3(256), 0, s, tmp, n, out);
}

// =============================================================================================
// Small helpers.
// =============================================================================================
__global__ void k_embed(const int* ids, int n, const float* table, int dim, float* out) {
  const int i = blockIdx.x;
  const float* src = table + (long)ids[i] * dim;
  for (int c = threadIdx.x; c < dim; c += blockDim.x) out[(long)i * dim + c] = src[c];
}
void embed_gather(const int* ids, int n, const float* table, int dim, float* out, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_embed, dim3(n), dim3(256), 0, s, ids, n, table, dim, out);
}

__global__ void k_copy2d(const float* src, long lds, float* dst, long ldd, int rows, int cols) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)rows * cols) return;
  const int r = (int)(idx / cols), c = (int)(idx % cols);
  dst[(long)r * ldd + c] = src[(long)r * lds + c];
}
void copy2d(const float* src, long lds, float* dst, long ldd, int rows, int cols, hipStream_t s) {
  const long total = (long)rows * cols;
  if (total > 0) hipLaunchKernelGGL(k_copy2d, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, src, lds, dst, ldd, rows, cols);
}

// Final SEANet conv (64 -> 1, k=3) with ELU'd input and 2-row history: one thread per sample.
// One wave per (batch row, 64 consecutive outputs): lane c owns input channel c (cin == 64) and
// loads its channel of the 64 + k - 1 input rows with coalesced 256-B row reads (history rows for
// t < 0), applies ELU once per element, and the k-tap dot products are reduced across the wave.
// One wave per (batch row, 64 consecutive outputs). The 64 + k - 1 input rows (cin == 64; history
// rows for t < 0) are read with coalesced 256-B row loads, ELU'd once per element and transposed
// through a padded LDS tile (row stride 65: conflict-free column reads); lane t then forms output
// t as a plain k x cin dot product (weights broadcast from LDS).
// =============================================================================================
// Fused SEANet residual block of one decoder stage (seanet.rs:43-89; SEANetResnetBlock with one
// residual layer, kernel sizes [3, 1], true skip): per (utterance, time tile of TT rows)
//   v = elu(b3 + conv_k3(E))          E = elu(convtr output), the stage's k3 conv input; its two
//                                       rows before the frame come from the conv history HE
//   Y = elu(R + b1 + conv_k1(v))       R = the raw convtr output (skip); Y = the next stage's
//                                       (or the final conv's) ELU'd input
// The intermediate v never leaves the CU: it goes from the first GEMM's accumulators to LDS and
// is the second GEMM's A operand. Both GEMMs run on v_mfma_f32_32x32x2_f32 with A fragments read
// from LDS (rows padded by 16 B: conflict-free ds_read_b128) and W fragments straight from global
// memory (L2-resident; each lane one 64-B piece of a weight row), one K chunk ahead.
// Shapes (B = 32): stage 0 C 256 / H 128 / T 96, stage 1 128 / 64 / 480, stage 2 64 / 32 / 1920.
// =============================================================================================
template <int C, int H, int TT>
__global__ __launch_bounds__(256) void k_resblock(ResBlockArgs a) {
  if (a.back_hi) back_prio();
  constexpr int LDE = C + 4, LDV = H + 4;
  __shared__ __attribute__((aligned(16))) float sm[(TT + 2) * LDE + TT * LDV];
  float* sE = sm;
  float* sV = sm + (TT + 2) * LDE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.y, t0 = blockIdx.x * TT;
  // ---- E rows t0-2 .. t0+TT-1 (history rows for t < 0) into LDS: every load of the thread is
  // issued before the first LDS store (one memory round trip, not one per 256-thread sweep)
  constexpr int C4 = C / 4, NE = ((TT + 2) * C4 + 255) / 256;
  float4 ev[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int e = min(tid + 256 * i, (TT + 2) * C4 - 1);  // a clamped duplicate, never stored
    const int row = e / C4, c4 = e - row * C4;
    const int t = t0 - 2 + row;
    const float* src = t >= 0 ? a.E + ((long)b * a.T + t) * C : a.HE + ((long)b * 2 + (t + 2)) * C;
    ev[i] = *reinterpret_cast<const float4*>(src + 4 * c4);
  }
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int e = tid + 256 * i;
    if (e >= (TT + 2) * C4) break;
    const int row = e / C4, c4 = e - row * C4;
    float4 v = ev[i];
    if (a.e_raw && t0 - 2 + row >= 0) v = make_float4(elu1(v.x), elu1(v.y), elu1(v.z), elu1(v.w));
    *reinterpret_cast<float4*>(sE + row * LDE + 4 * c4) = v;
  }
  __syncthreads();
  // ---- GEMM 1: v[TT][H] = E3[TT][3C] . W3[H][3C]^T, k = tap * C + c reads sE[i + tap][c]
  constexpr int MB = TT / 32, NB1 = H / 32, K1 = 3 * C / 32;
  for (int blk = wave; blk < MB * NB1; blk += 4) {
    const int mi = blk / NB1, ni = blk - mi * NB1;
    const float* wrow = a.W3 + (long)(32 * ni + r) * (3 * C) + 16 * h;
    floatx16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
    // W fragments three chunks ahead (an L2 / MALL round trip is several chunks of MFMAs): a ring
    // of three register sets with fixed roles per unrolled step
    float4 w0[4], w1[4], w2[4];
    auto wload = [&](int kc, float4 (&w)[4]) {
      const int k = kc < K1 ? kc : K1 - 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = *reinterpret_cast<const float4*>(wrow + 32 * k + 4 * q);
    };
    auto step = [&](int kc, const float4 (&w)[4]) {
      const int k0 = 32 * kc + 16 * h, tap = k0 / C, c = k0 - tap * C;
      const float* ap = sE + (32 * mi + r + tap) * LDE + c;
      float af[16], bf[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(ap + 4 * q);
        af[4 * q] = x.x; af[4 * q + 1] = x.y; af[4 * q + 2] = x.z; af[4 * q + 3] = x.w;
        bf[4 * q] = w[q].x; bf[4 * q + 1] = w[q].y; bf[4 * q + 2] = w[q].z; bf[4 * q + 3] = w[q].w;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], acc, 0, 0, 0);
    };
    static_assert(K1 % 3 == 0, "K1 = 3C/32 chunks: a multiple of 3 (the ring)");
    wload(0, w0);
    wload(1, w1);
    for (int kc = 0; kc < K1; kc += 3) {
      wload(kc + 2, w2);
      step(kc, w0);
      wload(kc + 3, w0);
      step(kc + 1, w1);
      wload(kc + 4, w1);
      step(kc + 2, w2);
    }
    const int col = 32 * ni + r;
    const float bias = a.b3[col];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int row = 32 * mi + (g & 3) + 8 * (g >> 2) + 4 * h;
      sV[row * LDV + col] = elu1(acc[g] + bias);
    }
  }
  __syncthreads();
  // ---- GEMM 2: Y[TT][C] = elu(R + b1 + v . W1[C][H]^T)
  constexpr int NB2 = C / 32, K2 = H / 32;
  for (int blk = wave; blk < MB * NB2; blk += 4) {
    const int mi = blk / NB2, ni = blk - mi * NB2;
    const float* wrow = a.W1 + (long)(32 * ni + r) * H + 16 * h;
    const int col = 32 * ni + r;
    const long base = ((long)b * a.T + t0) * C + col;
    float rv[16];  // the skip rows, requested ahead of the MFMAs that they do not depend on
#pragma unroll
    for (int g = 0; g < 16; ++g) rv[g] = a.R[base + (long)(32 * mi + (g & 3) + 8 * (g >> 2) + 4 * h) * C];
    floatx16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
#pragma unroll
    for (int kc = 0; kc < K2; ++kc) {
      const float* ap = sV + (32 * mi + r) * LDV + 32 * kc + 16 * h;
      float af[16], bf[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(ap + 4 * q);
        const float4 y = *reinterpret_cast<const float4*>(wrow + 32 * kc + 4 * q);
        af[4 * q] = x.x; af[4 * q + 1] = x.y; af[4 * q + 2] = x.z; af[4 * q + 3] = x.w;
        bf[4 * q] = y.x; bf[4 * q + 1] = y.y; bf[4 * q + 2] = y.z; bf[4 * q + 3] = y.w;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], acc, 0, 0, 0);
    }
    const float bias = a.b1[col];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int row = 32 * mi + (g & 3) + 8 * (g >> 2) + 4 * h;
      const float y = elu1(acc[g] + bias + rv[g]);
      a.Y[base + (long)row * C] = y;
      if (C == 64 && a.fw) sE[row * LDE + col] = y;  // (sE is free: GEMM 1 is behind the barrier)
    }
  }
  if constexpr (C == 64) {
    if (!a.fw) return;  // uniform
    // ---- final conv (64 -> 1, k = 3) of this tile: out[t] = b + d0[t-2] + d1[t-1] + d2[t],
    // d_j[r] = w[j] . Y[r]. Rows -2, -1 (the utterance's first tile only) are the conv history.
    static_assert(TT == RESBLOCK_FIN_TT, "the side buffer is laid out for 128-row tiles");
    float* sD = sV;  // [3][TT + 2] (row r at index r + 2); sV is free once GEMM 2 is done
    __syncthreads();
    for (int e = tid; e < 2 * (TT + 2); e += 256) {
      const int r = e / 2 - 2, half = e & 1;  // two threads per row (adjacent lanes), 32 channels each
      const bool live = r >= 0 || t0 == 0;
      const float* yr = r >= 0 ? sE + r * LDE + 32 * half : a.fH + ((long)b * 2 + (live ? r + 2 : 0)) * 64 + 32 * half;
      float d[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 y = *reinterpret_cast<const float4*>(yr + 4 * q);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const float4 w = *reinterpret_cast<const float4*>(a.fw + j * 64 + 32 * half + 4 * q);
          d[j] += (y.x * w.x + y.y * w.y) + (y.z * w.z + y.w * w.w);
        }
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        d[j] += __shfl_xor(d[j], 1, 64);
        if (half == 0) sD[j * (TT + 2) + r + 2] = live ? d[j] : 0.f;
      }
    }
    __syncthreads();
    const float fb = a.fb[0];
    const int nx = a.T / TT, x = blockIdx.x;
    if (tid < TT) {
      const int r = tid;
      const float d0 = sD[r], d1 = sD[(TT + 2) + r + 1], d2 = sD[2 * (TT + 2) + r + 2];
      // rows 0, 1 of a later tile: the terms from this tile's rows only (the rest via the side buffer)
      const float v = r >= 2 || t0 == 0 ? ((d0 + d1) + d2) + fb : (r == 0 ? d2 : d1 + d2) + fb;
      a.fout[(long)b * (a.fld ? a.fld : a.T) + t0 + r] = v;
    } else if (tid < TT + 2 && x + 1 < nx) {  // this tile's share of the next tile's rows 0, 1
      const int k = tid - TT;
      const float v = k == 0 ? sD[TT] + sD[(TT + 2) + TT + 1]  // d0[TT-2] + d1[TT-1]
                             : sD[TT + 1];                     // d0[TT-1]
      a.fside[((long)b * nx + x + 1) * 2 + k] = v;
    }
  }
}

void resblock(const ResBlockArgs& ra, hipStream_t s) {
  ResBlockArgs a = ra;
  a.back_hi = g_back_hi;
  // time tiles: stage 0 32 rows (96 workgroups), stage 1 96 (160), stage 2 128 (480) at B = 32
  if (a.C == 256 && a.T % 32 == 0)
    hipLaunchKernelGGL((k_resblock<256, 128, 32>), dim3(a.T / 32, a.B), dim3(256),
                       cap_lds(k_resblock<256, 128, 32>, g_wg_cap), s, a);
  else if (a.C == 128 && a.T % 96 == 0)
    hipLaunchKernelGGL((k_resblock<128, 64, 96>), dim3(a.T / 96, a.B), dim3(256),
                       cap_lds(k_resblock<128, 64, 96>, g_wg_cap), s, a);
  else if (a.C == 64 && a.T % 128 == 0 && (!a.fw || (a.fb && a.fH && a.fout && a.fside)))
    hipLaunchKernelGGL((k_resblock<64, 32, 128>), dim3(a.T / 128, a.B), dim3(256),
                       cap_lds(k_resblock<64, 32, 128>, g_wg_cap), s, a);
  else
    throw std::runtime_error("resblock: unsupported stage shape");
}

template <int KT>
__global__ __launch_bounds__(256) void k_conv_cout1(const float* X, const float* H, int B, int T, int cin,
                                                    const float* w, const float* bias, float* Y, int elu_in,
                                                    long ldy) {
  constexpr int P = KT - 1, ROWS = 64 + P;
  __shared__ float tile[4][ROWS][65];
  __shared__ float sw[KT * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < KT * 64; i += 256) sw[i] = w[i];
  const int blk = blockIdx.x * 4 + wave;
  const int nblk = (T + 63) / 64;
  const bool live = blk < B * nblk;
  const int b = live ? blk / nblk : 0, t0 = live ? (blk - b * nblk) * 64 : 0;
  const float* xb = X + (long)b * T * cin + lane;
  const float* hb = H + ((long)b * P + P) * cin + lane;
  float e[ROWS];
#pragma unroll
  for (int i = 0; i < ROWS; ++i) {  // unconditional loads: rows past T re-read row T-1
    const int tt = min(t0 + i - P, T - 1);
    e[i] = tt >= 0 ? xb[(long)tt * cin] : hb[(long)tt * cin];
  }
#pragma unroll
  for (int i = 0; i < ROWS; ++i) tile[wave][i][lane] = elu_in ? elu1(e[i]) : e[i];
  __syncthreads();
  float acc = 0.f;
#pragma unroll 8
  for (int c = 0; c < 64; ++c)
#pragma unroll
    for (int j = 0; j < KT; ++j) acc += sw[j * 64 + c] * tile[wave][lane + j][c];
  if (live && t0 + lane < T) Y[(long)b * ldy + t0 + lane] = acc + bias[0];
}

void conv_cout1(const float* X, const float* H, int B, int T, int cin, int k, const float* w, const float* bias,
                float* Y, int elu_in, hipStream_t s, long ldy) {
  const long waves = (long)B * ((T + 63) / 64);  // one lane per input channel: cin == 64, k == 3
  (void)k;
  hipLaunchKernelGGL(k_conv_cout1<3>, dim3((unsigned)((waves + 3) / 4)), dim3(256), cap_lds(k_conv_cout1<3>, g_wg_cap), s, X, H, B, T, cin, w, bias,
                     Y, elu_in, ldy > 0 ? ldy : (long)T);
}

// Encoder first conv (1 -> cout, k taps, zero history of k-1 samples): one thread per output.
__global__ __launch_bounds__(256) void k_conv_cin1(const float* X, int T, int cout, int k, const float* w,
                                                   const float* bias, float* Y) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)T * cout) return;
  const int t = (int)(idx / cout), co = (int)(idx % cout);
  float acc = 0.f;
  for (int j = 0; j < k; ++j) {
    const int tt = t + j - (k - 1);
    acc += (tt >= 0 ? X[tt] : 0.f) * w[co * k + j];
  }
  Y[idx] = acc + bias[co];
}
void conv_cin1(const float* X, int T, int cout, int k, const float* w, const float* bias, float* Y, hipStream_t s) {
  const long total = (long)T * cout;
  hipLaunchKernelGGL(k_conv_cin1, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, X, T, cout, k, w, bias, Y);
}

// ---------------------------------------------------------------------------------------------
// Polyphase resampler (see kernels.h). One lane per output sample: lanes of a wave walk
// consecutive outputs, so their input windows overlap and the x reads coalesce in L1/L2; the
// taps (L floats, <= 64 KB) are staged once per workgroup in LDS. Each output touches only the
// ~L/up taps of its phase, accumulated in f64 (scipy's f32 upfirdn differs by f32 rounding only).
__global__ __launch_bounds__(256) void k_resample(const float* __restrict__ x, int n_in,
                                                  const float* __restrict__ taps, int L, int up, int down,
                                                  int half, int n_out, int n_pad, int use_lds, float* y) {
  extern __shared__ float sh_taps[];
  if (use_lds) {
    for (int i = threadIdx.x; i < L; i += blockDim.x) sh_taps[i] = taps[i];
    __syncthreads();
  }
  const float* h = use_lds ? sh_taps : taps;
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_pad) return;
  if (m >= n_out) {
    y[m] = 0.f;
    return;
  }
  const long a = m * down + half;  // h index of x[0]; x[j] pairs with h[a - j*up]
  const long jhi = min(a / up, (long)n_in - 1);
  const long lo = a - (L - 1);
  const long jlo = lo <= 0 ? 0 : (lo + up - 1) / up;
  double acc = 0.0;
  for (long j = jlo; j <= jhi; ++j) acc += (double)x[j] * (double)h[a - j * up];
  y[m] = (float)acc;
}

namespace {
int gcd_int(int a, int b) {
  while (b) {
    const int t = a % b;
    a = b;
    b = t;
  }
  return a;
}
double bessel_i0(double x) {  // power series; converges in a few dozen terms for beta = 5
  double s = 1.0, t = 1.0;
  const double q = 0.25 * x * x;
  for (int k = 1; k < 500; ++k) {
    t *= q / ((double)k * k);
    s += t;
    if (t < 1e-17 * s) break;
  }
  return s;
}
}  // namespace

ResamplePlan resample_plan(int sr_from, int sr_to) {
  ResamplePlan p;
  const int g = gcd_int(sr_from, sr_to);
  p.up = sr_to / g;
  p.down = sr_from / g;
  p.half = 10 * std::max(p.up, p.down);  // resample_poly: half_len = 10 * max_rate
  p.L = 2 * p.half + 1;
  return p;
}

// firwin(L, 1/max_rate, window=("kaiser", 5.0)): windowed sinc normalised to unit DC gain,
// then cast to f32 and multiplied by `up` in f32, as resample_poly does for f32 input.
std::vector<float> resample_taps(const ResamplePlan& p) {
  std::vector<double> hd(p.L);
  const double fc = 1.0 / std::max(p.up, p.down), alpha = 0.5 * (p.L - 1), i0b = bessel_i0(5.0);
  double sum = 0.0;
  for (int i = 0; i < p.L; ++i) {
    const double v = fc * (i - alpha), r = (i - alpha) / alpha;
    const double sinc = v == 0.0 ? 1.0 : std::sin(M_PI * v) / (M_PI * v);
    hd[i] = fc * sinc * (bessel_i0(5.0 * std::sqrt(std::max(0.0, 1.0 - r * r))) / i0b);
    sum += hd[i];
  }
  std::vector<float> h(p.L);
  for (int i = 0; i < p.L; ++i) h[i] = (float)(hd[i] / sum) * (float)p.up;
  return h;
}

void resample(const float* x, int n_in, const float* taps, const ResamplePlan& p, int n_out, int n_pad, float* y,
              hipStream_t s) {
  if (n_pad <= 0) return;
  const int use_lds = p.L <= 16384 ? 1 : 0;
  const size_t lds = use_lds ? sizeof(float) * (size_t)p.L : 0;
  hipLaunchKernelGGL(k_resample, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), lds, s, x, n_in, taps, p.L, p.up,
                     p.down, p.half, n_out, n_pad, use_lds, y);
}

// ---------------------------------------------------------------------------------------------
// rubato FastFixedIn / Septic (see kernels.h): the Lagrange weights of nodes -3..4 at frac as
// prefix x suffix products of (frac - node), each times 1 / prod_{m != j} (j - m) =
// (-1)^(7-j) / (j! (7-j)!); the sum over the 8 taps in tap order. The oracle's orc_resample_septic
// performs the same f32 operations in the same order (contraction off on both sides), so the two
// agree bit for bit; lanes of a wave read overlapping 8-sample windows (L1/L2 hits).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float septic_eval(const float* __restrict__ x, int n_in, int s, float f) {
#pragma clang fp contract(off)
  constexpr float inv_den[8] = {-1.f / 5040.f, 1.f / 720.f, -1.f / 240.f, 1.f / 144.f,
                                -1.f / 144.f,  1.f / 240.f, -1.f / 720.f, 1.f / 5040.f};
  float d[8], pre[8], suf[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) d[m] = f - (float)(m - 3);
  pre[0] = 1.f;
#pragma unroll
  for (int m = 1; m < 8; ++m) pre[m] = pre[m - 1] * d[m - 1];
  suf[7] = 1.f;
#pragma unroll
  for (int m = 6; m >= 0; --m) suf[m] = suf[m + 1] * d[m + 1];
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int i = s - 3 + j;
    const float v = (i >= 0 && i < n_in) ? x[i] : 0.f;
    acc = acc + v * ((pre[j] * suf[j]) * inv_den[j]);
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_resample_septic(const float* __restrict__ x, int n_in,
                                                         const int* __restrict__ start,
                                                         const float* __restrict__ frac, int n_out, int n_pad,
                                                         float* __restrict__ y) {
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_pad) return;
  y[m] = m < n_out ? septic_eval(x, n_in, start[m], frac[m]) : 0.f;
}

long septic_schedule(long n, int sr_from, int sr_to, std::vector<int>* start, std::vector<float>* frac) {
  if (n <= 0 || sr_from <= 0 || sr_to <= 0) return 0;
  const double ratio = (double)sr_to / (double)sr_from;  // audio.rs:213
  const double t = 1.0 / ratio;                          // dt_ratio is 0 at a fixed ratio
  const double end = (double)(n - 9);                    // chunk_size - (POLYNOMIAL_LEN + 1)
  double idx = -4.0;                                     // last_index = -(POLYNOMIAL_LEN / 2)
  long cnt = 0;
  if (start) start->clear();
  if (frac) frac->clear();
  while (idx < end) {
    idx += t;
    const double fl = std::floor(idx);
    if (start) start->push_back((int)fl);
    if (frac) frac->push_back((float)(idx - fl));
    ++cnt;
  }
  return cnt;
}

void resample_septic(const float* x, int n_in, const int* start, const float* frac, int n_out, int n_pad, float* y,
                     hipStream_t s) {
  if (n_pad <= 0) return;
  hipLaunchKernelGGL(k_resample_septic, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), 0, s, x, n_in, start, frac,
                     n_out, n_pad, y);
}

// =============================================================================================
// Flow-head chain in ONE persistent launch (mlp.rs:146-213, 370-383; flow_lm.rs:7-22): for every
// lsd Euler step, input projection -> 6 ResBlocks -> FinalLayer -> x += v / N. As separate
// launches this is 28 GEMM + row-reduce kernels of M = B rows x 512 (each ~1 MB of weights), a
// chain of launch gaps and HBM round trips. Here a grid of ceil(B/16) row groups x 32 column
// groups (16 rows x 16 output columns per workgroup, 8 waves splitting K = 512) runs the chain
// with in-launch hand-offs in which the data is its own flag (the tag-free form of the granule
// hand-off, cdna_hip_programming.md Guideline 16 R2):
//   every hand-off has its own region, filled with 0xFFFFFFFF (a NaN no arithmetic produces) by
//   the launch just ahead (k_row_reduce's side job in the adaLN reduce);
//   producer: the storing wave writes its 16x16 tile with sc1 (write-through) 16-B buffer stores
//             and moves on (no drain, no counter);
//   consumer: each wave sweeps its 16 rows x 64 columns with sc1 buffer loads and re-reads every
//             float4 that still holds the empty pattern (bounded spin) - a 4-byte word is read
//             either empty or final, so a word that is not empty is the producer's value.
// Each workgroup keeps its 16x16 tile of the residual stream x in registers for the whole chain;
// consumers rebuild the full rows (LayerNorm statistics need all 512 columns) from the published
// copy. Weights, LayerNorm affines and adaLN modulations do not depend on the chain and are
// loaded before each wait. The latent `cur` between Euler steps (lsd > 1) is handed off with a
// counter (sc1 stores, drain, agent-scope add); counters are zeroed at allocation and re-armed by
// the last workgroup to finish.
// v_mfma_f32_16x16x4_f32 fragments as in k_attn16: lane (c = l & 15, G = l >> 4) supplies
// A[row c][k] and B[k][col c] for k = 64*wave + FH_KJ*(s/4) + 4*G + s%4 at step s (FH_KJ below); D reg g -> row 4G+g, col c.
// =============================================================================================
constexpr int FH_WAVES = 8;  // FH_D, FH_L, FH_DEPTH: kernels.h
// k layout of a lane's 16 values: float4 j of lane group G holds k = 64 wave + FH_KJ j + 4 G ..+3,
// so the 4 lane groups of a row read 64 contiguous bytes per load instruction (16 rows x 64 B
// per instruction instead of 16 rows x four 16-B pieces 64 B apart). A and B use the same k
// order, so the MFMA sum is over the same products.
constexpr int FH_KJ = 16;
// consumer offsets of float4 j in a hand-off region: the 16 columns of j sit in the next column
// group's 16x16 tile, 1 KB on
constexpr int FH_SJ = 16 * 16 * 4;

__device__ __forceinline__ float4 f4ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
// consumer: this lane's 16 values of a region (byte offset `off`), re-read until none is empty.
// The loop condition is wave-uniform; a timeout sets *err and stops waiting for the rest of the
// launch (the frame is poisoned, fetch() reports it).
__device__ __forceinline__ void fh_sweep(__amdgpu_buffer_rsrc_t r, int off, float4 (&v)[4], int* err, bool& dead) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = fh_ld(r, off + FH_SJ * j);
  unsigned spins = 0;
  while (!dead) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) ok &= !fh_empty(v[j]);
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (fh_empty(v[j])) v[j] = fh_ld(r, off + FH_SJ * j);
    if (++spins > (1u << 20)) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dead = true;
    }
  }
}

// LayerNorm (eps 1e-6, optional affine) + adaLN modulate (mlp.rs:29-58,135-137) of this lane's
// 16 values of row c. Row statistics in ONE workgroup barrier: each wave contributes its 64
// values' sum and squared deviations about their own mean, combined as M2 = sum_w [M2_w +
// 64 (mean_w - mean)^2] (Chan et al.'s pairwise update; the same two-pass variance, summed in a
// different order), in a fixed wave order.
// The affines (lnw, lnb: LDS, this lane's k range; nullptr for none) are read after the barrier,
// so the prologue's LDS fill needs no barrier of its own.
__device__ __forceinline__ void fh_ln(float4 (&v)[4], float (*s_st)[FH_WAVES][16], int wave, int c, int G,
                                      const float* lnw, const float* lnb, const float4 (&sc)[4],
                                      const float4 (&sf)[4]) {
  float s1 = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s1 += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  const float mw = s1 * (1.0f / 64.0f);
  float m2 = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = v[j].x - mw, b = v[j].y - mw, d = v[j].z - mw, e = v[j].w - mw;
    m2 += (a * a + b * b) + (d * d + e * e);
  }
  m2 += __shfl_xor(m2, 16, 64);
  m2 += __shfl_xor(m2, 32, 64);
  if (G == 0) {
    s_st[0][wave][c] = s1;
    s_st[1][wave][c] = m2;
  }
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < FH_WAVES; ++w) tot += s_st[0][w][c];
  const float mean = tot / (float)FH_D;
  float q = 0.f;
#pragma unroll
  for (int w = 0; w < FH_WAVES; ++w) {
    const float dm = s_st[0][w][c] * (1.0f / 64.0f) - mean;
    q += s_st[1][w][c] + 64.0f * dm * dm;
  }
  const float rden = 1.0f / sqrtf(q / (float)FH_D + 1e-6f);  // one divide, then multiplies (<= 1 ulp apart)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float4 h = make_float4((v[j].x - mean) * rden, (v[j].y - mean) * rden, (v[j].z - mean) * rden,
                           (v[j].w - mean) * rden);
    if (lnw) h = f4add(f4mul(h, f4ld(lnw + FH_KJ * j)), f4ld(lnb + FH_KJ * j));
    v[j] = make_float4(h.x * (1.0f + sc[j].x) + sf[j].x, h.y * (1.0f + sc[j].y) + sf[j].y,
                       h.z * (1.0f + sc[j].z) + sf[j].z, h.w * (1.0f + sc[j].w) + sf[j].w);
  }
}
// 16 MFMA steps over this lane's k range, then the 8 wave partials summed in wave order; wave 0
// lane t returns the 16x16 tile's row t/4, columns 4(t%4)..+3
// (consecutive GEMMs alternate between two s_red buffers: no barrier is needed between wave 0's
// reads of one and the other waves' writes of the next)
__device__ __forceinline__ float4 fh_gemm(const float4 (&a)[4], const float4 (&b)[4], float (*s_red)[16][16],
                                          int wave, int c, int G, int lane) {
  // four independent accumulator chains (one per float4 of the lane's k range), summed after:
  // the dependent chain of 16 MFMAs was the phase's longest serial step
  floatx4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].x, b[j].x, floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].y, b[j].y, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].z, b[j].z, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].w, b[j].w, acc[j], 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) s_red[wave][4 * G + g][c] = (acc[0][g] + acc[1][g]) + (acc[2][g] + acc[3][g]);
  __syncthreads();
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (wave == 0) {
#pragma unroll
    for (int w = 0; w < FH_WAVES; ++w) r = f4add(r, f4ld(&s_red[w][lane >> 2][4 * (lane & 3)]));
  }
  return r;
}

// Operands of one phase, loaded a phase ahead of their use (non-publishing waves right after the
// current phase's payload loads, the publishing wave 0 right after its publish, so that neither
// the payload wait nor the publish drain waits for them): the lane's 16-k slice of one weight
// row, and for LayerNorm phases the adaLN scale / shift of the lane's row.
struct FhOps {
  float4 w[4], sc[4], sf[4];
  float4 e0, e1;  // wave 0 epilogue: bias | gate, bias
};

__global__ __launch_bounds__(64 * FH_WAVES) void k_flow_head(FlowHeadArgs a) {
  front_prio();
  __shared__ float s_st[2][FH_WAVES][16];
  __shared__ __attribute__((aligned(16))) float s_red2[2][FH_WAVES][16][16];
  __shared__ __attribute__((aligned(16))) float s_ln[FH_DEPTH][2][FH_D];  // ResBlock LayerNorm affines
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, G = lane >> 4;
  const int RG = (a.B + 15) / 16;
  // XCD-aware placement (speed only: blocks b and b + 8 are observed to share an XCD's L2): the
  // RG row groups of a column group sit on one XCD, so each weight fragment is fetched into that
  // L2 once and read by all RG of them (column groups 4x .. 4x+3 on XCD slot x)
  const int xs = blockIdx.x & 7, xr = blockIdx.x >> 3;
  const int rg = xr % RG, cg = 4 * xs + xr / RG;
  const int col0 = 16 * cg;
  const int arow = min(16 * rg + c, a.B - 1);  // A-operand row of this lane (clamped; rows >= B unused)
  const int k0 = 64 * wave + 4 * G;            // this lane's 16 k: k0 + FH_KJ j + 0..3, j < 4
  const int orow = 16 * rg + (lane >> 2);      // epilogue (wave 0): row, columns ocol..ocol+3
  const int ocol = col0 + 4 * (lane & 3);
  const int crow = min(orow, a.B - 1);
  const bool ostore = orow < a.B;
  const bool fin = cg < FH_L / 16;  // column groups 0 and 1 own the 32 latent columns
  const __amdgpu_buffer_rsrc_t hr = fh_rsrc(a.hx), cr = fh_rsrc(a.cur);
  int* cc = a.ctr + 4 * rg + 2;  // cur published (lsd > 1)
  const int rstride = RG * 16 * FH_D * 4;  // bytes per hand-off region
  // sweep / store byte offsets in a hand-off region ([RG][32][16][16]: tile (rg, cg) is one KB):
  // lane (c, G) of wave w reads row c, columns 16 (4w + j) + 4G..+3 of its row group; wave 0 lane
  // t stores its tile's row t/4, columns 4(t%4)..+3 at tile offset 16 t bytes
  const int aoff = (((rg * 32 + 4 * wave) * 16 + (arow - 16 * rg)) * 16 + 4 * G) * 4;
  const int ooff = ((rg * 32 + cg) * 256 + 4 * lane) * 4;
  int q = 0;   // next hand-off region
  int gi = 0;  // GEMMs done (s_red buffer parity)
  bool dead = false;
  float4 xo = make_float4(0.f, 0.f, 0.f, 0.f);  // wave 0: residual tile x[orow][ocol..+3]
  int sk = 0;
#ifdef PTTS_PROBES  // s_memrealtime stamps of workgroups 0-3 (tools/head_stamps.py)
#define FH_STAMP()                                                                     \
  if (a.dbg && tid == 0 && blockIdx.x < 4 && sk < 120) a.dbg[blockIdx.x * 128 + sk++] = __builtin_amdgcn_s_memrealtime()
#else
#define FH_STAMP() (void)sk
#endif
  // probe layout: [entry, x0 published, 6 x 8 ResBlock stamps, final: swept, done]
  FH_STAMP();

  // operand loaders (i: ResBlock, or FH_DEPTH for the FinalLayer)
  // fragment-packed matrix m (2i: w0 of ResBlock i, 2i + 1: its w2, 12: fin_w), this lane's float4 j
  const float* wpl = a.wp + ((long)cg * FH_WAVES + wave) * 4 * 256 + 4 * lane;
  auto wfrag = [&](int m, int j) { return f4ld(wpl + (long)m * (32 * FH_WAVES * 4 * 256) + j * 256); };
  auto load_ln_ops = [&](FhOps& o, const float* mods, int i, int stp) {
    if (i == FH_DEPTH && !fin) return;
    const float* mp = a.fhm + (((((long)(stp * RG + rg) * (FH_DEPTH + 1) + i) * 2) * 8 + wave) * 4 * 64 + lane) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o.w[j] = wfrag(2 * i, j);
      o.sf[j] = f4ld(mp + j * 256);
      o.sc[j] = f4ld(mp + 8 * 4 * 256 + j * 256);
    }
    if (wave == 0) o.e0 = f4ld((i < FH_DEPTH ? a.b0 + (long)i * a.blk : a.fin_b) + ocol);
  };
  auto load_mlp2_ops = [&](FhOps& o, const float* mods, int i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o.w[j] = wfrag(2 * i + 1, j);
    if (wave == 0) {
      o.e0 = f4ld(mods + (long)crow * a.ldm + (long)i * 3 * FH_D + 2 * FH_D + ocol);  // gate
      o.e1 = f4ld(a.b2 + (long)i * a.blk + ocol);
    }
  };
  FhOps p0, p2;  // operands of the next LayerNorm phase and the next mlp2 phase

  for (int st = 0; st < a.lsd; ++st) {
    const float* mods = a.mods + (long)st * a.B * a.ldm;
    // ---- input projection x = cur W_in^T + b_in (K = 32), one wave. At st = 0 it comes first:
    // its hand-off starts the chain, so its loads are not queued behind the prologue's
    // At st = 0 with x0_ready the launch ahead (the adaLN reduce) has stored x0 already: wave 0
    // only reads its residual tile back (the chain's prologue was 3.5-3.9 us of cold loads).
    if (st > 0) fh_wait(cc, 2 * st, a.err, dead);
    if (wave == 0 && st == 0 && a.x0_ready) {
      xo = fh_ld(hr, ooff);
    } else if (wave == 0) {
      float4 cv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) cv[j] = fh_ld(cr, (crow * FH_L + 4 * j) * 4);
      xo = fh_inproj4(cv, a.in_w, a.in_b, ocol);
      if (ostore) fh_put(hr, q * rstride + ooff, xo);
    }
    ++q;
    FH_STAMP();
    if (st == 0) {
      // the first phases' operands, then the ResBlock LayerNorm affines into LDS (first read
      // after the first LayerNorm's barrier)
      load_ln_ops(p0, mods, 0, st);
      load_mlp2_ops(p2, mods, 0);
#pragma unroll
      for (int i = 0; i < FH_DEPTH; ++i)
        if (tid < FH_D / 2) {  // threads 0..255: float4 (tid & 127) of lnw (tid < 128) or lnb
          const float* src = (tid < FH_D / 4 ? a.lnw : a.lnb) + (long)i * a.blk;
          reinterpret_cast<float4*>(&s_ln[i][tid < FH_D / 4 ? 0 : 1][0])[tid & (FH_D / 4 - 1)] =
              f4ld(src + 4 * (tid & (FH_D / 4 - 1)));
        }
    }
#pragma unroll 1
    for (int i = 0; i < FH_DEPTH; ++i) {
      // ---- h = modulate(LN(x)), u = silu(h W0^T + b0)
      float4 v[4];
      FH_STAMP();
      fh_sweep(hr, (q - 1) * rstride + aoff, v, a.err, dead);
      FH_STAMP();
      fh_ln(v, s_st, wave, c, G, &s_ln[i][0][k0], &s_ln[i][1][k0], p0.sc, p0.sf);
      FH_STAMP();
      float4 r = fh_gemm(v, p0.w, s_red2[gi++ & 1], wave, c, G, lane);
      FH_STAMP();
      if (wave != 0) load_ln_ops(p0, mods, i + 1, st);
      if (wave == 0) {
        const float4 bb = p0.e0;
        const float4 u = make_float4(silu(r.x + bb.x), silu(r.y + bb.y), silu(r.z + bb.z), silu(r.w + bb.w));
        if (ostore) fh_put(hr, q * rstride + ooff, u);
        load_ln_ops(p0, mods, i + 1, st);
      }
      FH_STAMP();
      ++q;
      // ---- x += gate * (u W2^T + b2)
      fh_sweep(hr, (q - 1) * rstride + aoff, v, a.err, dead);
      FH_STAMP();
      r = fh_gemm(v, p2.w, s_red2[gi++ & 1], wave, c, G, lane);
      FH_STAMP();
      if (wave != 0 && i + 1 < FH_DEPTH) load_mlp2_ops(p2, mods, i + 1);
      if (wave == 0) {
        xo = f4add(xo, f4mul(p2.e0, f4add(r, p2.e1)));
        if (ostore) fh_put(hr, q * rstride + ooff, xo);
        if (i + 1 < FH_DEPTH) load_mlp2_ops(p2, mods, i + 1);
      }
      FH_STAMP();
      ++q;
    }
    // ---- FinalLayer (mlp.rs:182-213): modulate(LN_noaffine(x)) W_f^T + b_f, Euler x += v / N
    const float* nmods = mods + (long)a.B * a.ldm;  // next Euler step's modulations
    const bool more = st + 1 < a.lsd;
    if (fin) {
      const int off = (crow * FH_L + ocol) * 4;
      float4 cv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (wave == 0) cv = fh_ld(cr, off);  // latent before this Euler step (read ahead of the sweep)
      float4 v[4];
      fh_sweep(hr, (q - 1) * rstride + aoff, v, a.err, dead);
      FH_STAMP();
      if (wave != 0 && more) load_mlp2_ops(p2, nmods, 0);
      fh_ln(v, s_st, wave, c, G, nullptr, nullptr, p0.sc, p0.sf);
      const float4 r = fh_gemm(v, p0.w, s_red2[gi++ & 1], wave, c, G, lane);
      if (wave != 0 && more) load_ln_ops(p0, nmods, 0, st + 1);
      if (wave == 0) {
        const float e = a.euler_scale;
        const float4 o = f4add(r, p0.e0);
        if (ostore) fh_st(cr, off, make_float4(cv.x + o.x * e, cv.y + o.y * e, cv.z + o.z * e, cv.w + o.w * e));
        if (more) fh_publish(cc);
        FH_STAMP();
        if (more) {
          load_ln_ops(p0, nmods, 0, st + 1);
          load_mlp2_ops(p2, nmods, 0);
        }
      }
    } else if (more) {
      load_ln_ops(p0, nmods, 0, st + 1);
      load_mlp2_ops(p2, nmods, 0);
    }
  }
  // re-arm: the last workgroup to finish zeroes every counter (all waits are behind it); with one
  // Euler step no counter is used
  if (a.lsd > 1 && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* done = a.ctr + 4 * RG;
    if (__hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      for (int g = 0; g < 4 * RG; ++g) __hip_atomic_store(a.ctr + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// FlowLM input projection + the first layer's norm1 in one launch (flow_lm.rs:117 input_linear,
// transformer.rs:66-90 norm1): x[m] = lat[m] W^T (K = 32, no bias), h[m] = LN(x[m]) (eps 1e-5).
// One workgroup per row (input_ln_row). The step graphs fold this into k_front_commit of the step
// before; this launch refreshes every row after anything else wrote x / h or lat_in.
__global__ __launch_bounds__(256) void k_input_ln(const float* __restrict__ lat, const float* __restrict__ Wt,
                                                  const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                  float* __restrict__ x, float* __restrict__ h) {
  front_prio();
  __shared__ float sh[4];
  const int m = blockIdx.x;
  input_ln_row(lat + (long)m * 32, Wt, lnw, lnb, x + (long)m * 1024, h + (long)m * 1024, sh);
}

void input_ln(const float* lat, const float* Wt, const float* lnw, const float* lnb, float* x, float* h, int M,
              hipStream_t s) {
  hipLaunchKernelGGL(k_input_ln, dim3(M), dim3(256), 0, s, lat, Wt, lnw, lnb, x, h);
}

__global__ void k_transpose(const float* src, int rows, int cols, float* dst) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i % cols);
  dst[(long)c * rows + r] = src[i];
}

void transpose(const float* src, int rows, int cols, float* dst, hipStream_t s) {
  const long n = (long)rows * cols;
  hipLaunchKernelGGL(k_transpose, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, rows, cols, dst);
}


bool flow_head_fits(int B) { return B >= 1 && B <= 128; }

size_t flow_head_packed_floats() { return (size_t)2 * FH_DEPTH * FH_D * FH_D + (size_t)FH_L * FH_D; }

// dst float4 (((m * 32 + cg) * 8 + w) * 4 + j) * 64 + l = W_m[16 cg + (l & 15)][64 w + FH_KJ j +
// 4 (l >> 4) ..+3], W_m = w0 / w2 of ResBlock m / 2, or fin_w (m = 12, column groups 0-1)
__global__ void k_pack_flow_head(const float* w0, const float* w2, long blk, const float* fin_w, float4* dst,
                                 long n4) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n4) return;
  const int l = (int)(e & 63), j = (int)((e >> 6) & 3), w = (int)((e >> 8) & 7), cg = (int)((e >> 11) & 31);
  const int m = (int)(e >> 16);
  const float* W = m == 2 * FH_DEPTH ? fin_w : (m & 1 ? w2 : w0) + (long)(m >> 1) * blk;
  dst[e] = *reinterpret_cast<const float4*>(W + (long)(16 * cg + (l & 15)) * FH_D + 64 * w + FH_KJ * j + 4 * (l >> 4));
}

void pack_flow_head(const float* w0, const float* w2, long blk, const float* fin_w, float* dst, hipStream_t s) {
  const long n4 = (long)flow_head_packed_floats() / 4;
  hipLaunchKernelGGL(k_pack_flow_head, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, w0, w2, blk, fin_w,
                     reinterpret_cast<float4*>(dst), n4);
}

int flow_head_grid(int B) { return (B + 15) / 16 * (FH_D / 16); }

int flow_head_max_resident(int dev) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_flow_head, 64 * FH_WAVES, 0) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return per_cu * cus;
}

void flow_head(const FlowHeadArgs& a, hipStream_t s) {
  if (!flow_head_fits(a.B)) throw std::runtime_error("flow_head: B out of range");
  hipLaunchKernelGGL(k_flow_head, dim3(flow_head_grid(a.B)), dim3(64 * FH_WAVES), 0, s, a);
}

#ifdef PTTS_PROBES
__global__ void k_stamp(unsigned long long* ring, unsigned* ctr, unsigned tag) {
  const unsigned i = atomicAdd(ctr, 1u);
  if (i < STAMP_CAP) {
    ring[2 * i] = tag;
    ring[2 * i + 1] = wall_clock64();
  }
}

void stamp(unsigned long long* ring, unsigned* ctr, unsigned tag, hipStream_t s) {
  hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, s, ring, ctr, tag);
}
#endif

}  // namespace ptts
