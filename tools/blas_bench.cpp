// Calibration: rocBLAS fp32 GEMM on the hot-path dense shapes (Y[M][N] = X[M][K] W[N][K]^T),
// as the library ceiling to compare tools/gemm_bench.hip against.
// Build: hipcc -O3 -std=c++17 tools/blas_bench.cpp -lrocblas -o tools/bin/blas_bench
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <vector>

int main() {
  rocblas_handle h;
  rocblas_create_handle(&h);
  hipStream_t st;
  (void)hipStreamCreate(&st);
  rocblas_set_stream(h, st);
  struct S {
    const char* name;
    int M, N, K;
  };
  std::vector<S> shapes = {{"flow.qkv", 32, 3072, 1024},   {"flow.out", 32, 1024, 1024},
                           {"flow.ff1", 32, 4096, 1024},   {"flow.ff2", 32, 1024, 4096},
                           {"head.ada", 32, 10240, 512},   {"mimi.qkv", 512, 1536, 512},
                           {"mimi.out", 512, 512, 512},    {"mimi.ff1", 512, 2048, 512},
                           {"mimi.ff2", 512, 512, 2048},   {"conv0 (im2col)", 512, 512, 3584},
                           {"convtr2 (1 phase)", 3072, 128, 512}, {"res3a (im2col)", 61440, 32, 192},
                           {"prefill.qkv", 1536, 3072, 1024}, {"prefill.out", 1536, 1024, 1024},
                           {"prefill.ff1", 1536, 4096, 1024}, {"prefill.ff2", 1536, 1024, 4096},
                           {"big 4096^3", 4096, 4096, 4096}};
  float *X, *W, *Y;
  (void)hipMalloc(&X, sizeof(float) * 64 << 20);
  (void)hipMalloc(&W, sizeof(float) * 64 << 20);
  (void)hipMalloc(&Y, sizeof(float) * 64 << 20);
  (void)hipMemset(X, 0, sizeof(float) * 64 << 20);
  (void)hipMemset(W, 0, sizeof(float) * 64 << 20);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const float one = 1.f, zero = 0.f;
  for (auto& s : shapes) {
    // row-major Y[M][N] = X[M][K] * W[N][K]^T  <=>  column-major Y^T[N][M] = W^T... : C(NxM) = op(W)(NxK) * X^T(KxM)
    auto run = [&]() {
      rocblas_sgemm(h, rocblas_operation_transpose, rocblas_operation_none, s.N, s.M, s.K, &one, W, s.K, X, s.K,
                    &zero, Y, s.N);
    };
    for (int i = 0; i < 5; ++i) run();
    const int reps = 50;
    (void)hipEventRecord(e0, st);
    for (int i = 0; i < reps; ++i) run();
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = 1000.0 * ms / reps;
    printf("%-20s M%6d N%6d K%5d : %8.2f us  %6.1f TF/s\n", s.name, s.M, s.N, s.K, us,
           2.0 * s.M * s.N * s.K / us / 1e6);
  }
  return 0;
}
