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

namespace ptts {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float gelu_tanh(float x) {
  // candle Tensor::gelu (tanh approximation), transformer.rs:85
  return 0.5f * x * (1.0f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float elu1(float x) { return x >= 0.f ? x : expf(x) - 1.0f; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
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
template <int MODE>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs a) {
  __shared__ float red[4 * 16 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32, z = blockIdx.z;
  const int nchunks = a.K >> 5;
  int cb = 0, ce = nchunks, phase = 0;
  if (MODE == 0) {
    cb = (int)((long)nchunks * z / a.S);
    ce = (int)((long)nchunks * (z + 1) / a.S);
  } else {
    phase = z;
  }
  const float* wrow = a.W + (long)phase * a.w_phase_stride + (long)(n0 + r) * a.K + 16 * h;
  const int m = m0 + r;
  const bool mvalid = m < a.M;
  const float* xrow = nullptr;
  int bq = 0, qq = 0;
  if (MODE == 0) {
    xrow = a.X + (long)(mvalid ? m : 0) * a.ldx + 16 * h;
  } else if (mvalid) {
    bq = m / a.Tq;
    qq = m - bq * a.Tq;
  }

  auto a_ptr = [&](int k0) -> const float* {
    if (MODE == 0) return xrow + k0;
    const int j = k0 / a.cin;
    const int ci = k0 - j * a.cin + 16 * h;
    const int t = qq * a.stride_in + j - a.P;
    if (t >= 0) return a.X + ((long)bq * a.T_in + t) * a.ldx + ci;
    return a.H + ((long)bq * a.P + (a.P + t)) * a.cin + ci;
  };

  floatx16 acc;
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;

  float4 av[4], bv[4], an[4], bn[4];
  int c = cb + wave;
  if (c < ce) {
    const float* ap = a_ptr(c << 5);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bv[i] = *reinterpret_cast<const float4*>(wrow + (c << 5) + 4 * i);
      av[i] = mvalid ? *reinterpret_cast<const float4*>(ap + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  for (; c < ce; c += 4) {
    const int cn = c + 4;
    if (cn < ce) {  // prefetch the wave's next chunk while this one is multiplied
      const float* ap = a_ptr(cn << 5);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bn[i] = *reinterpret_cast<const float4*>(wrow + (cn << 5) + 4 * i);
        an[i] = mvalid ? *reinterpret_cast<const float4*>(ap + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    float af[16], bf[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[4 * i + 0] = av[i].x; af[4 * i + 1] = av[i].y; af[4 * i + 2] = av[i].z; af[4 * i + 3] = av[i].w;
      bf[4 * i + 0] = bv[i].x; bf[4 * i + 1] = bv[i].y; bf[4 * i + 2] = bv[i].z; bf[4 * i + 3] = bv[i].w;
    }
    if (MODE == 1 && a.elu_in) {
#pragma unroll
      for (int j = 0; j < 16; ++j) af[j] = elu1(af[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      av[i] = an[i];
      bv[i] = bn[i];
    }
  }

#pragma unroll
  for (int g = 0; g < 16; ++g) red[(wave * 16 + g) * 64 + lane] = acc[g];
  __syncthreads();
#pragma unroll
  for (int gg = 0; gg < 4; ++gg) {
    const int g = wave * 4 + gg;
    float v = red[(0 * 16 + g) * 64 + lane] + red[(1 * 16 + g) * 64 + lane];
    v += red[(2 * 16 + g) * 64 + lane];
    v += red[(3 * 16 + g) * 64 + lane];
    const int row = m0 + (g & 3) + 8 * (g >> 2) + 4 * h;
    const int col = n0 + r;
    if (row >= a.M || col >= a.N) continue;
    if (a.partial) {
      a.partial[((long)z * a.M + row) * a.N + col] = v;
      continue;
    }
    if (a.bias) v += a.bias[col];
    if (a.act == ACT_GELU) v = gelu_tanh(v);
    else if (a.act == ACT_SILU) v = silu(v);
    long yrow = row;
    if (MODE == 1) {
      const int b2 = row / a.Tq;
      const int q2 = row - b2 * a.Tq;
      yrow = (long)b2 * a.T_out + (long)q2 * a.out_tstride + phase;
    }
    if (a.rscale) v *= a.rscale[col];
    if (a.R) v += a.R[yrow * a.ldr + col];
    a.Y[yrow * a.ldy + col] = v;
  }
}

void gemm(const GemmArgs& a, int grid_z, hipStream_t s) {
  dim3 grid((a.N + 31) / 32, (a.M + 31) / 32, grid_z);
  if (a.mode == 0) hipLaunchKernelGGL(k_gemm<0>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_gemm<1>, grid, dim3(256), 0, s, a);
}

// =============================================================================================
// Row reduce + epilogue + LayerNorm/modulate. One workgroup per row.
// =============================================================================================
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

template <int NPT>
__global__ __launch_bounds__(256) void k_row_reduce(RowReduceArgs a) {
  __shared__ float sh[4];
  const int m = blockIdx.x;
  const int tid = threadIdx.x;
  float v[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int n = tid + i * 256;
    float x = 0.f;
    if (n < a.N) {
      for (int z = 0; z < a.S; ++z) x += a.P[((long)z * a.M + m) * a.N + n];
      if (a.bias) x += a.bias[n];
      if (a.act == ACT_GELU) x = gelu_tanh(x);
      else if (a.act == ACT_SILU) x = silu(x);
      if (a.gate) x *= a.gate[(long)m * a.ldg + n];
      if (a.R) x += a.R[(long)m * a.ldr + n];
      if (a.Y) a.Y[(long)m * a.ldy + n] = x;
      if (a.euler) a.euler[(long)m * 32 + n] += x * a.euler_scale;
    }
    v[i] = x;
  }
  if (!a.ln) return;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) s += (tid + i * 256 < a.N) ? v[i] : 0.f;
  const float mean = block_sum(s, sh) / (float)a.N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const float d = v[i] - mean;
    q += (tid + i * 256 < a.N) ? d * d : 0.f;
  }
  const float var = block_sum(q, sh) / (float)a.N;
  const float den = sqrtf(var + a.eps);
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int n = tid + i * 256;
    if (n >= a.N) continue;
    float hh = (v[i] - mean) / den;
    if (a.ln_w) hh = hh * a.ln_w[n] + a.ln_b[n];
    if (a.mshift) hh = hh * (1.0f + a.mscale[(long)m * a.ldm + n]) + a.mshift[(long)m * a.ldm + n];
    a.Hout[(long)m * a.ldh + n] = hh;
  }
}

void row_reduce(const RowReduceArgs& a, hipStream_t s) {
  dim3 grid(a.M);
  if (a.N <= 1024) hipLaunchKernelGGL(k_row_reduce<4>, grid, dim3(256), 0, s, a);
  else if (a.N <= 4096) hipLaunchKernelGGL(k_row_reduce<16>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_row_reduce<40>, grid, dim3(256), 0, s, a);
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
  hipLaunchKernelGGL(k_layernorm, dim3((M + 3) / 4), dim3(256), 0, s, x, ldx, y, ldy, M, N, w, b, eps);
}

// =============================================================================================
// QKV (+ split-K reduce) -> RoPE -> KV append. One thread per (row, head, rotation pair).
// =============================================================================================
__device__ __forceinline__ void row_slot_pos(const RowMap& mp, int row, int& slot, int& pos) {
  slot = mp.slot0 + row / mp.rps;
  pos = (mp.pos_arr ? mp.pos_arr[slot] : mp.p0) + row % mp.rps;
}

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
  Q[(long)row * d + c] = q0 * cs - q1 * sn;
  Q[(long)row * d + c + 1] = q0 * sn + q1 * cs;
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
  hipLaunchKernelGGL(k_qkv_rope, dim3((total + 255) / 256), dim3(256), 0, s, P, S, dense, M, nh, map, kv, Q);
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

void attention(const float* Q, int M, int nh, RowMap map, KvStore kv, int window, int qg, float* O, hipStream_t s) {
  dim3 grid((M + qg - 1) / qg, nh);
  hipLaunchKernelGGL(k_attention, grid, dim3(256), 0, s, Q, M, nh, map, kv, window, qg, O);
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
                                                   int lsd, SlotState* st, float* ysilu, float* cur, float* eos_out) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int NC = 513;  // cond_embed (512) | out_eos (1)
  for (int n = tid; n < 512; n += 256) {
    float c = 0.f;
    for (int z = 0; z < S; ++z) c += P[((long)z * B + b) * NC + n];
    c += bias[n];
    for (int s = 0; s < lsd; ++s) ysilu[((long)s * B + b) * 512 + n] = silu(temb[s * 512 + n] + c);
  }
  SlotState& ss = st[b];
  if (tid == 0) {
    float e = 0.f;
    for (int z = 0; z < S; ++z) e += P[((long)z * B + b) * NC + 512];
    e += bias[512];
    eos_out[b] = e;
    ss.valid = ss.active;
    ss.last = 0;
    if (ss.active) {  // tts_model.rs:1055-1063 + map_while over 0..max_gen_len
      if (e > ss.eos_threshold && ss.eos_step < 0) ss.eos_step = ss.step;
      const bool tail = ss.eos_step >= 0 && ss.step >= ss.eos_step + ss.frames_after_eos;
      ss.last = (tail || ss.step + 1 >= ss.max_frames) ? 1 : 0;
    }
  }
  if (tid < 32) {
    float x0 = 0.f;
    const float temp = ss.temp;
    if (temp > 0.f) {  // flow_lm.rs:39-65: N(0, sqrt(temp)), optionally truncated to |x| <= clamp
      const float sd = sqrtf(temp);
      x0 = sd * normal_at(ss.seed, ss.step, tid, 0);
      if (ss.noise_clamp > 0.f) {
        int att = 1;
        while (fabsf(x0) > ss.noise_clamp && att < 64) x0 = sd * normal_at(ss.seed, ss.step, tid, att++);
        x0 = fminf(fmaxf(x0, -ss.noise_clamp), ss.noise_clamp);
      }
    }
    cur[b * 32 + tid] = x0;
  }
}

void flow_cond(const float* P, int S, int B, const float* bias, const float* temb, int lsd_steps, SlotState* st,
               float* ysilu, float* cur, float* eos_out, hipStream_t s) {
  hipLaunchKernelGGL(k_flow_cond, dim3(B), dim3(256), 0, s, P, S, B, bias, temb, lsd_steps, st, ysilu, cur, eos_out);
}

// =============================================================================================
// Mimi front: denorm -> 1x1 quantizer -> depthwise ConvTrUpsample1d (k=32, s=16) -> LN.
// The transposed conv's overlap-add `partial` (conv.rs:202-267) equals qprev * W[:, 16 + r],
// so the kernel keeps the previous frame's quantized vector instead.
// =============================================================================================
__global__ __launch_bounds__(256) void k_quant_upsample(const float* latent, const float* emb_std,
                                                        const float* emb_mean, const float* wq, const float* wup,
                                                        float* qprev, const SlotState* st, float* x, float* h,
                                                        const float* ln_w, const float* ln_b) {
  __shared__ float sz[32];
  __shared__ float sx[16 * 512];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid < 32) sz[tid] = latent[b * 32 + tid] * emb_std[tid] + emb_mean[tid];
  __syncthreads();
  const bool upd = st[b].valid != 0;
  for (int c = tid; c < 512; c += 256) {
    float q = 0.f;
    for (int k = 0; k < 32; ++k) q += wq[c * 32 + k] * sz[k];
    const float qp = qprev[(long)b * 512 + c];
    for (int r = 0; r < 16; ++r) {
      const float v = q * wup[c * 32 + r] + qp * wup[c * 32 + 16 + r];
      sx[r * 512 + c] = v;
      x[((long)b * 16 + r) * 512 + c] = v;
    }
    if (upd) qprev[(long)b * 512 + c] = q;
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  for (int r = wave; r < 16; r += 4) {
    float v[8], s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[i] = sx[r * 512 + lane + 64 * i];
      s += v[i];
    }
    const float mean = wave_sum(s) / 512.f;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) q += (v[i] - mean) * (v[i] - mean);
    const float den = sqrtf(wave_sum(q) / 512.f + 1e-5f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = lane + 64 * i;
      h[((long)b * 16 + r) * 512 + n] = (v[i] - mean) / den * ln_w[n] + ln_b[n];
    }
  }
}

void quant_upsample(const float* latent, int B, const float* emb_std, const float* emb_mean, const float* wq,
                    const float* wup, float* qprev, const SlotState* st, float* x, float* h, const float* ln_w,
                    const float* ln_b, hipStream_t s) {
  hipLaunchKernelGGL(k_quant_upsample, dim3(B), dim3(256), 0, s, latent, emb_std, emb_mean, wq, wup, qprev, st, x,
                     h, ln_w, ln_b);
}

// =============================================================================================
// Step commit: conv histories (last P input rows per slot), counters, next backbone input.
// =============================================================================================
__global__ __launch_bounds__(256) void k_commit(CommitArgs a) {
  const int b = blockIdx.y;
  SlotState& ss = a.st[b];
  if (!ss.valid) return;
  if ((int)blockIdx.x < a.nh) {
    const HistDesc& hd = a.h[blockIdx.x];
    const long n = (long)hd.P * hd.C;
    const float* src = hd.src + ((long)b * hd.T + (hd.T - hd.P)) * hd.C;
    float* dst = hd.dst + (long)b * n;
    for (long e = threadIdx.x; e < n; e += 256) dst[e] = src[e];
    return;
  }
  if (threadIdx.x < 32) a.latent_next[b * 32 + threadIdx.x] = a.latent[b * 32 + threadIdx.x];
  if (threadIdx.x == 0) {
    ss.step += 1;
    a.fpos[b] += 1;
    a.mpos[b] += 16;
    if (ss.last) ss.active = 0;
  }
}

void step_commit(const CommitArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_commit, dim3(a.nh + 1, a.B), dim3(256), 0, s, a);
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
__global__ __launch_bounds__(256) void k_conv_cout1(const float* X, const float* H, int B, int T, int cin, int k,
                                                    const float* w, const float* bias, float* Y) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * T) return;
  const int b = (int)(idx / T), t = (int)(idx % T);
  const int P = k - 1;
  float acc = 0.f;
  for (int j = 0; j < k; ++j) {
    const int tt = t + j - P;
    const float* src = tt >= 0 ? X + ((long)b * T + tt) * cin : H + ((long)b * P + (P + tt)) * cin;
    const float* wr = w + j * cin;
    for (int c = 0; c < cin; c += 4) {
      const float4 xv = *reinterpret_cast<const float4*>(src + c);
      const float4 wv = *reinterpret_cast<const float4*>(wr + c);
      acc += elu1(xv.x) * wv.x + elu1(xv.y) * wv.y + elu1(xv.z) * wv.z + elu1(xv.w) * wv.w;
    }
  }
  Y[idx] = acc + bias[0];
}
void conv_cout1(const float* X, const float* H, int B, int T, int cin, int k, const float* w, const float* bias,
                float* Y, hipStream_t s) {
  const long total = (long)B * T;
  hipLaunchKernelGGL(k_conv_cout1, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, X, H, B, T, cin, k, w,
                     bias, Y);
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

}  // namespace ptts
