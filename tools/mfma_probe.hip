// Calibration: sustained v_mfma_f32_32x32x2_f32 throughput (operands in registers, no memory)
// for 1/2/4 independent accumulators and 1..8 waves per SIMD, plus the in-kernel clock.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void k_probe(float* out, int iters, float seed, unsigned long long* clk) {
  floatx16 acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[q][g] = 0.f;
  float a = seed + threadIdx.x * 1e-3f, b = seed - threadIdx.x * 1e-3f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16 / NACC; ++j)
#pragma unroll
      for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[q], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int g = 0; g < 16; ++g) s += acc[q][g];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

int main() {
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, sizeof(float) * 256 * 8192);
  hipMalloc(&clk, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  for (int nacc : {1, 2, 4}) {
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: blocks of 256 threads = 1 wave per SIMD each
      const int blocks = 256 * wps;
      auto launch = [&]() {
        if (nacc == 1) hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f, clk);
        if (nacc == 2) hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f, clk);
        if (nacc == 4) hipLaunchKernelGGL(k_probe<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f, clk);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[2];
      hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
      const double flops = 5.0 * blocks * 4.0 * iters * 16 * 4096.0;  // 5 launches, 4096 flop per MFMA
      const double ghz = (double)h[0] / ((double)h[1] / 100.0) / 1000.0;
      printf("acc %d waves/SIMD %d : %.3f ms  %.1f TF/s  clock %.2f GHz\n", nacc, wps, ms, flops / (ms * 1e-3) / 1e12,
             ghz);
    }
  }
  return 0;
}
