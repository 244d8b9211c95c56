// GEMM-core microbenchmark (round 3): the engine's LDS-DMA tile variants against rocBLAS fp32 on
// the hot-path shapes (text-prefill passes at M = 32 x 48 rows, the Mimi decoder GEMMs at M = 512,
// the SEANet implicit-GEMM convs at B = 32). Each variant is checked against a naive fp64-accumulated
// kernel, then timed with HIP events (20 warm launches, 100 timed, median of 5 blocks of 20), on
// uniform random operands. rocBLAS is the calibration only (tools, never the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPTTS_PROBES -Iinclude -Ipocket-tts_amd/csrc tools/mm_bench.hip \
//        -lrocblas -o tools/bin/mm_bench
// Usage: mm_bench [case-substring] [layout] [S]   (S < 0: split tail of -S slices, ILV layouts)
#include "../pocket-tts_amd/csrc/kernels.hip"

#include <rocblas/rocblas.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace ptts;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d: %s\n", #x, __LINE__, hipGetErrorString(e));  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ float a_elem(const GemmArgs& a, int m, int k) {
  if (a.mode == 0) return a.X[(long)m * a.ldx + k];
  const int b = m / a.Tq, q = m % a.Tq, j = k / a.cin, ci = k % a.cin;
  const int t = q * a.stride_in + j - a.P;
  float v = t >= 0 ? a.X[((long)b * a.T_in + t) * a.ldx + ci] : a.H[((long)b * a.P + a.P + t) * a.cin + ci];
  return a.elu_in ? elu1(v) : v;
}
__global__ void k_ref(GemmArgs a, float* out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)a.M * a.N) return;
  const int m = idx / a.N, n = idx % a.N;
  const float* w = a.W + (long)n * a.K;
  double acc = 0;
  for (int k = 0; k < a.K; ++k) acc += (double)a_elem(a, m, k) * w[k];
  out[idx] = (float)acc;
}
__global__ void k_sum(const float* P, int S, long n, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s = 0;
  for (int z = 0; z < S; ++z) s += P[z * n + i];
  out[i] = s;
}

static float* drand(size_t n, unsigned seed, float scale) {
  std::vector<float> h(n);
  srand(seed);
  for (auto& v : h) v = scale * ((float)rand() / RAND_MAX * 2.f - 1.f);
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

struct Case {
  std::string name;
  GemmArgs a;
  std::vector<std::pair<int, int>> variants;  // (layout, S); layout -1 = rocBLAS (dense only)
};

int main(int argc, char** argv) {
  const char* only_case = argc > 1 ? argv[1] : nullptr;
  const int only_layout = argc > 2 ? atoi(argv[2]) : -100;
  const int only_s = argc > 3 ? atoi(argv[3]) : -1;
  setvbuf(stdout, nullptr, _IOLBF, 0);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  rocblas_handle bh;
  rocblas_create_handle(&bh);
  rocblas_set_stream(bh, st);
  const int B = 32;
  float *P, *Y, *ref, *got, *slab;
  int* tickets;
  CK(hipMalloc(&slab, sizeof(float) * (32 << 20)));
  CK(hipMalloc(&tickets, sizeof(int) * 4096));
  CK(hipMemset(tickets, 0, sizeof(int) * 4096));
  CK(hipMalloc(&P, sizeof(float) * (96 << 20)));
  CK(hipMalloc(&Y, sizeof(float) * (64 << 20)));
  CK(hipMalloc(&ref, sizeof(float) * (64 << 20)));
  CK(hipMalloc(&got, sizeof(float) * (64 << 20)));
  std::vector<Case> cases;
  auto dense = [&](const char* nm, int M, int N, int K, std::vector<std::pair<int, int>> v) {
    GemmArgs a{};
    a.mode = 0;
    a.M = M; a.N = N; a.K = K; a.Nw = (N + 31) / 32 * 32;
    a.X = drand((size_t)M * K, 1, 1.f);
    a.ldx = K;
    a.W = drand((size_t)a.Nw * K, 2, 0.05f);
    a.Y = Y;
    a.ldy = N;
    cases.push_back({nm, a, v});
  };
  // single-phase streaming conv (stride 1) over B utterances of T_in rows: taps k, history P
  auto conv = [&](const char* nm, int T_in, int cin, int P_, int k, int N, std::vector<std::pair<int, int>> v) {
    GemmArgs a{};
    a.mode = 1;
    a.Tq = T_in; a.M = B * T_in; a.N = N; a.K = k * cin; a.Nw = (N + 31) / 32 * 32;
    a.X = drand((size_t)B * T_in * cin, 3, 1.f);
    a.ldx = cin;
    a.H = drand((size_t)B * (P_ ? P_ : 1) * cin, 4, 1.f);
    a.P = P_; a.T_in = T_in; a.stride_in = 1; a.cin = cin; a.elu_in = 0;
    a.W = drand((size_t)a.Nw * a.K, 5, 0.05f);
    a.w_phase_stride = (long)N * a.K;
    a.S = 1;
    a.Y = Y;
    a.ldy = N;
    a.T_out = T_in; a.out_tstride = 1;
    cases.push_back({nm, a, v});
  };
  const std::vector<std::pair<int, int>> big = {{-1, 1}, {30, 1}, {31, 1}, {34, 1}, {35, 1}, {36, 1}, {39, 1},
                                                {30, -2}, {30, -4}, {30, -8}, {31, -2}, {31, -4}, {31, -8},
                                                {34, -2}, {34, -4}, {34, -8}, {36, -2}, {36, -4}, {36, -8},
                                                {32, -2}, {32, -4}, {35, -2}, {35, -4}, {39, -2}, {39, -4}};
  const std::vector<std::pair<int, int>> mid = {{-1, 1}, {6, 1}, {12, 1}, {15, 1}, {32, 1}, {33, 1}, {37, 1},
                                                {34, 1}, {35, 1}, {36, 1}, {39, 1}, {21, 1}, {30, 1}, {31, 1},
                                                {6, 2}, {32, 2}, {33, 2}, {34, 2}, {35, 2}, {30, 2}, {31, 2},
                                                {6, 4}, {32, 4}, {33, 4}, {30, 4}, {31, 4}, {34, 4}, {35, 4}};
  dense("prefill.qkv M1536 N3072 K1024", 1536, 3072, 1024, big);
  dense("prefill.out M1536 N1024 K1024", 1536, 1024, 1024, big);
  dense("prefill.ff1 M1536 N4096 K1024", 1536, 4096, 1024, big);
  dense("prefill.ff2 M1536 N1024 K4096", 1536, 1024, 4096, big);
  dense("mimi.qkv M512 N1536 K512", 16 * B, 1536, 512, mid);
  dense("mimi.out M512 N512 K512", 16 * B, 512, 512, mid);
  dense("mimi.ff1 M512 N2048 K512", 16 * B, 2048, 512, mid);
  dense("mimi.ff2 M512 N512 K2048", 16 * B, 512, 2048, mid);
  conv("conv0 T16 c512 k7 N512", 16, 512, 6, 7, 512, mid);
  conv("convtr0m T16 c512 k2 N1536", 16, 512, 1, 2, 1536, mid);
  conv("convtr1m T96 c256 k2 N640", 96, 256, 1, 2, 640, mid);
  conv("convtr2m T480 c128 k2 N256", 480, 128, 1, 2, 256, mid);
  conv("res3.s0 T96 c256 k3 N128", 96, 256, 2, 3, 128, mid);
  conv("res3.s1 T480 c128 k3 N64", 480, 128, 2, 3, 64, mid);
  conv("res1.s0 T96 c128 k1 N256", 96, 128, 0, 1, 256, mid);
  dense("big M4096 N4096 K4096", 4096, 4096, 4096, {{-1, 1}, {21, 1}, {30, 1}, {31, 1}, {38, 1}});

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& c : cases) {
    if (only_case && c.name.find(only_case) == std::string::npos) continue;
    GemmArgs a = c.a;
    const long out_n = (long)a.M * a.N;
    hipLaunchKernelGGL(k_ref, dim3((out_n + 255) / 256), dim3(256), 0, st, a, ref);
    std::vector<float> href(out_n);
    CK(hipMemcpyAsync(href.data(), ref, out_n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const double flops = 2.0 * a.M * a.N * a.K;
    printf("== %s  (%.1f MFLOP)\n", c.name.c_str(), flops / 1e6);
    for (auto [layout, S] : c.variants) {
      if (only_layout > -100 && (layout != only_layout || (only_s >= 0 && S != only_s))) continue;
      GemmArgs v = a;
      v.layout = layout;
      if (layout == -1 && a.mode != 0) continue;
      const int bk = (layout == 8 || layout == 15 || layout == 16) ? 64 : 32;
      if (layout >= 0 && (a.K % bk != 0 || (a.mode == 1 && a.cin % bk != 0))) continue;
      if (S < 0) {
        if (layout < 30 || a.mode != 0) continue;
        v.S = 1;
        v.partial = nullptr;
        v.tail_S = -S;
        v.tail_slab = slab;
        v.tail_cap = 32l << 20;
        v.tickets = tickets;
        v.tickets_cap = 4096;
      } else if (S > 1) {
        if (a.K / bk < S) continue;
        v.S = S;
        v.partial = P;
      } else {
        v.S = 1;
        v.partial = nullptr;
      }
      const float one = 1.f, zero = 0.f;
      auto run = [&]() {
        if (layout == -1) {
          rocblas_sgemm(bh, rocblas_operation_transpose, rocblas_operation_none, a.N, a.M, a.K, &one, a.W, a.K, a.X,
                        (rocblas_int)a.ldx, &zero, Y, a.N);
        } else {
          gemm(v, S > 0 ? S : 1, st);
        }
      };
      try {
        run();
      } catch (const std::exception& e) {
        printf("   L%d S %d : %s\n", layout, S, e.what());
        continue;
      }
      CK(hipGetLastError());
      if (S > 1) hipLaunchKernelGGL(k_sum, dim3((out_n + 255) / 256), dim3(256), 0, st, P, S, out_n, got);
      else CK(hipMemcpyAsync(got, Y, out_n * 4, hipMemcpyDeviceToDevice, st));
      std::vector<float> hgot(out_n);
      CK(hipMemcpyAsync(hgot.data(), got, out_n * 4, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      double err = 0, mx = 0;
      for (long i = 0; i < out_n; ++i) {
        err = std::max(err, (double)fabsf(hgot[i] - href[i]));
        mx = std::max(mx, (double)fabsf(href[i]));
      }
      for (int i = 0; i < 20; ++i) run();
      std::vector<float> blk;
      for (int b = 0; b < 5; ++b) {
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 20; ++i) run();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        blk.push_back(1000.f * ms / 20);
      }
      std::sort(blk.begin(), blk.end());
      const double us = blk[2];
      const double rel = err / (mx + 1e-30);
      printf("   %-7s S %2d : %8.2f us  %6.1f TF/s  relerr %.1e %s\n",
             layout == -1 ? "rocBLAS" : ("L" + std::to_string(layout)).c_str(), S, us, flops / us / 1e6, rel,
             rel < 1e-5 ? "" : "BAD");
    }
  }
  return 0;
}
