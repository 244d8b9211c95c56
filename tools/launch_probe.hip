// Calibration: wall time per kernel of a hipGraph of N dependent tiny kernels, by grid size and
// kernel-argument size (the engine's GemmArgs is ~250 bytes), to price kernel boundaries.
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big {
  float* p;
  int pad[60];
};

__global__ __launch_bounds__(256) void k_small(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}
__global__ __launch_bounds__(256) void k_big(Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) b.p[0] += (float)b.pad[7];
}

int main() {
  float* d;
  (void)hipMalloc(&d, 4096);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int big = 0; big < 2; ++big) {
    for (int grid : {1, 32, 256, 1024}) {
      const int N = 100;
      hipGraph_t g;
      hipGraphExec_t ge;
      (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
      Big b{};
      b.p = d;
      for (int i = 0; i < N; ++i) {
        if (big) hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, b);
        else hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, d);
      }
      (void)hipStreamEndCapture(s, &g);
      (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
      (void)hipStreamSynchronize(s);
      const int R = 20;
      (void)hipEventRecord(e0, s);
      for (int r = 0; r < R; ++r) (void)hipGraphLaunch(ge, s);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("graph of %d kernels, grid %4d, %s args: %.2f us per kernel\n", N, grid, big ? "252-byte" : "8-byte",
             1000.0 * ms / (R * N));
      // eager launches of the same
      (void)hipEventRecord(e0, s);
      for (int r = 0; r < R; ++r)
        for (int i = 0; i < N; ++i) {
          if (big) hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, b);
          else hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, d);
        }
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("   eager: %.2f us per kernel\n", 1000.0 * ms / (R * N));
      (void)hipGraphExecDestroy(ge);
      (void)hipGraphDestroy(g);
    }
  }
  return 0;
}
