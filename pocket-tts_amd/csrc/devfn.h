// Device helpers of the kernel file (kernels.hip): activations, wave
// reductions, float4 arithmetic, the row -> (slot, position) map and the sc1 (agent-coherent)
// buffer loads / stores of the in-launch hand-offs.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ptts {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Issue priority of a front-part wave (s_setprio) where front (FlowLM / flow-head) and back (Mimi
// decode) waves share a SIMD: probe builds only (PTTS_FRONT_PRIO, set_front_prio; s_setprio
// takes an immediate). Measured: with frame pairs, priority 3 took the steady
// step from 0.602 to 0.580 ms, but with one frame per pass (the back part bounds the step) it
// cost 5 % (0.583 -> 0.613 ms), and pairs + priority beat the product's one-frame passes by
// 0.5 % only (same-box A/B, alternating rounds): not adopted.
#ifdef PTTS_PROBES
extern __device__ int g_front_prio;
__device__ __forceinline__ void front_prio() {
  const int p = __builtin_amdgcn_readfirstlane(g_front_prio);
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
}
// the back part's GEMM / conv tile waves: product builds issue at priority 3 (back_prio below);
// probe builds take the level from PTTS_BACK_PRIO (set_back_prio, default 3, 0 = off)
extern __device__ int g_back_prio;
__device__ __forceinline__ void back_prio() {
  const int p = __builtin_amdgcn_readfirstlane(g_back_prio);
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
}
// front-part skip probe (PTTS_FRONT_SKIP, results wrong): bit 0 the skinny GEMMs' weight loads,
// bit 1 their MFMAs, bit 2 the step attention's cached K / V loads
extern __device__ int g_front_skip;
__device__ __forceinline__ int front_skip() { return __builtin_amdgcn_readfirstlane(g_front_skip); }
#else
__device__ __forceinline__ void front_prio() {}
// Issue priority 3 for the back part's GEMM / conv tile waves (k_gemm_glds launches outside the
// front part, k_gemm_rb, k_resblock): where a back wave and a front wave are both ready on a SIMD,
// the back wave issues first. In the frame-pair step the back stream runs end to end (graph stamps,
// tools/stamps.py); steady step 0.5569 -> 0.5513 and 0.5674 -> 0.5631 ms on two boxes
// (profiles/r04/interference_probes.txt, interleaved repeats). Re-measured in round 5 with the
// front part bounding the step: level 0 in a product build 0.5533 against 0.5496 ms for 3
// (profiles/r05/prio_product_ab.txt; the probe build's knob read 0.5578 vs 0.5775 there,
// profiles/r05/prio_probe_ab.txt, but a probe build's per-launch priority load slows every launch
// and does not transfer): 3 stays.
__device__ __forceinline__ void back_prio() { __builtin_amdgcn_s_setprio(3); }
__device__ __forceinline__ constexpr int front_skip() { return 0; }
#endif

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

// Sum over each 16-lane row of the wave with DPP (quad_perm xor 1, xor 2, row_half_mirror,
// row_mirror); every lane of the row ends with the row's sum.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
  return v;
}

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4mul(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}

__device__ __forceinline__ void row_slot_pos(const RowMap& mp, int row, int& slot, int& pos) {
  if (mp.tab) {
    const int v = mp.tab[row];
    slot = v < 0 ? -1 : v >> 16;
    pos = v < 0 ? 0 : v & 0xFFFF;
    return;
  }
  slot = mp.slot0 + row / mp.rps;
  pos = (mp.pos_arr ? mp.pos_arr[slot] : mp.p0) + row % mp.rps;
}

// K / V of (slot, head): the slot's own rows (kb, vb; appends go there) and, under a shared voice
// prefix, the voice's rows (pk, pv) that hold positions < F (KvStore::pre)
struct KvHead {
  float *kb, *vb;
  const float *pk, *pv;
  int F;
};
__device__ __forceinline__ KvHead kv_head(const KvStore& kv, int slot, int nh, int head) {
  KvHead h;
  h.kb = kv.base + (long)slot * kv.slot_stride + (long)head * kv.cap * 64;
  h.vb = kv.base + (long)slot * kv.slot_stride + (long)(nh + head) * kv.cap * 64;
  h.pk = h.kb;
  h.pv = h.vb;
  h.F = 0;
  if (kv.pre != nullptr && slot >= 0) {
    const int F = kv.pre_len[slot];
    if (F > 0) {
      const float* p = kv.pre[slot] + ((long)kv.layer * 2 * nh + head) * F * 64;
      h.pk = p;
      h.pv = p + (long)nh * F * 64;
      h.F = F;
    }
  }
  return h;
}

// Buffer resource over a whole allocation, and 16-B loads / stores with the sc1 cache policy
// (agent scope: a store writes through to the point of coherence of all XCDs, a load does not hit
// a line another XCD's L2 may hold stale): the hand-off traffic of the persistent launches.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fh_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 fh_ld(__amdgpu_buffer_rsrc_t r, int byte_off) {  // sc1 load
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ void fh_st(__amdgpu_buffer_rsrc_t r, int byte_off, float4 f) {  // sc1 store
  const u32x4 v = {__float_as_uint(f.x), __float_as_uint(f.y), __float_as_uint(f.z), __float_as_uint(f.w)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, 16);
}
__device__ __forceinline__ void fh_st1(__amdgpu_buffer_rsrc_t r, int byte_off, float f) {  // sc1 store, 4 B
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f), r, byte_off, 0, 16);
}

// a handed-off value never carries the empty pattern: a NaN is stored as the canonical quiet NaN
// (the result stays NaN, as in the reference, and no consumer waits for it)
__device__ __forceinline__ float fh_canon(float x) { return x != x ? __uint_as_float(0x7FC00000u) : x; }
__device__ __forceinline__ void fh_put(__amdgpu_buffer_rsrc_t r, int byte_off, float4 f) {
  fh_st(r, byte_off, make_float4(fh_canon(f.x), fh_canon(f.y), fh_canon(f.z), fh_canon(f.w)));
}
__device__ __forceinline__ bool fh_empty(float4 v) {
  return ((int)(__float_as_uint(v.x) == ~0u) | (int)(__float_as_uint(v.y) == ~0u) |
          (int)(__float_as_uint(v.z) == ~0u) | (int)(__float_as_uint(v.w) == ~0u)) != 0;
}
__device__ __forceinline__ void fh_put1(__amdgpu_buffer_rsrc_t r, int byte_off, float f) {
  fh_st1(r, byte_off, fh_canon(f));
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// storing wave: drain its sc1 stores, then one lane signals
__device__ __forceinline__ void fh_publish(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// whole workgroup: thread 0 polls until ctr >= target (bounded: a timeout sets *err and stops
// waiting for the rest of the launch), then the barrier releases every wave's sc1 loads
__device__ __forceinline__ void fh_wait(int* ctr, int target, int* err, bool& dead) {
  if (threadIdx.x == 0 && !dead) {
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 20)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
}

}  // namespace ptts
