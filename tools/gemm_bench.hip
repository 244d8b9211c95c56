// Microbenchmark of the engine's GEMM / implicit-GEMM conv kernel layouts on the hot-path
// shapes (batch 32). Each variant is checked against a naive fp32 kernel, then timed with
// HIP events. Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include tools/gemm_bench.hip
#include "../pocket-tts_amd/csrc/kernels.hip"

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
__global__ void k_ref(GemmArgs a, int phase, float* out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)a.M * a.N) return;
  const int m = idx / a.N, n = idx % a.N;
  const float* w = a.W + (long)phase * a.w_phase_stride + (long)n * a.K;
  double acc = 0;
  for (int k = 0; k < a.K; ++k) acc += (double)a_elem(a, m, k) * w[k];
  out[(long)phase * a.M * a.N + idx] = (float)acc;
}
// sum of S partial slabs, or gather of the epilogue-free output, into [phases][M][N]
__global__ void k_collect(GemmArgs a, int phases, const float* src, float* out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)phases * a.M * a.N) return;
  const int ph = idx / ((long)a.M * a.N);
  const long mn = idx % ((long)a.M * a.N);
  const int m = mn / a.N, n = mn % a.N;
  if (a.partial) {
    float s = 0;
    for (int z = 0; z < a.S; ++z) s += src[((long)z * a.M + m) * a.N + n];
    out[idx] = s;
  } else {
    long yrow = m;
    if (a.mode == 1) yrow = (long)(m / a.Tq) * a.T_out + (long)(m % a.Tq) * a.out_tstride + ph;
    out[idx] = src[yrow * a.ldy + n];
  }
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
  int phases;
  std::vector<std::pair<int, int>> variants;  // (layout, S)
};

int main(int argc, char** argv) {
  // optional filter: gemm_bench <case substring> <layout> [S]  (PMC runs)
  const char* only_case = argc > 1 ? argv[1] : nullptr;
  const int only_layout = argc > 2 ? atoi(argv[2]) : -1;
  const int only_s = argc > 3 ? atoi(argv[3]) : -1;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int B = 32;
  float* P;
  CK(hipMalloc(&P, sizeof(float) * (64 << 20)));
  float* Y;
  CK(hipMalloc(&Y, sizeof(float) * (64 << 20)));
  float* ref;
  CK(hipMalloc(&ref, sizeof(float) * (64 << 20)));
  float* got;
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
    cases.push_back({nm, a, 1, v});
  };
  auto conv = [&](const char* nm, int T_in, int cin, int P_, int k, int N, int phases, int tstride,
                  std::vector<std::pair<int, int>> v) {
    GemmArgs a{};
    a.mode = 1;
    a.Tq = T_in; a.M = B * T_in; a.N = N; a.K = k * cin; a.Nw = (N + 31) / 32 * 32;
    a.X = drand((size_t)B * T_in * cin, 3, 1.f);
    a.ldx = cin;
    a.H = drand((size_t)B * (P_ ? P_ : 1) * cin, 4, 1.f);
    a.P = P_; a.T_in = T_in; a.stride_in = 1; a.cin = cin; a.elu_in = getenv("NOELU") ? 0 : 1;
    a.W = drand((size_t)phases * a.Nw * a.K, 5, 0.05f);
    a.w_phase_stride = (long)N * a.K;
    a.S = 1;
    a.Y = Y;
    a.ldy = N;
    a.T_out = T_in * tstride; a.out_tstride = tstride;
    cases.push_back({nm, a, phases, v});
  };
  std::vector<std::pair<int, int>> skinny = {{0, 8}, {0, 16}, {7, 8}, {7, 16}, {13, 8}, {13, 16}, {9, 8}, {9, 16},
                                             {10, 8}, {10, 16}, {17, 8}, {17, 16}, {0, 4}, {9, 4}};
  std::vector<std::pair<int, int>> fat = {{0, 1}, {18, 1}, {19, 1}, {20, 1}, {20, 2}, {6, 1}, {12, 1}, {12, 2},
                                          {13, 1}, {14, 1}};
  dense("flow.qkv M32 N3072 K1024", B, 3072, 1024, skinny);
  dense("flow.out M32 N1024 K1024", B, 1024, 1024, skinny);
  dense("flow.ff1 M32 N4096 K1024", B, 4096, 1024, skinny);
  dense("flow.ff2 M32 N1024 K4096", B, 1024, 4096, skinny);
  dense("head.ada M32 N10240 K512", B, 10240, 512, skinny);
  dense("head.mlp M32 N512 K512", B, 512, 512, skinny);
  dense("mimi.qkv M512 N1536 K512", 16 * B, 1536, 512, fat);
  dense("mimi.out M512 N512 K512", 16 * B, 512, 512, fat);
  dense("mimi.ff1 M512 N2048 K512", 16 * B, 2048, 512, fat);
  dense("mimi.ff2 M512 N512 K2048", 16 * B, 512, 2048, fat);
  conv("sea.conv0 T16 c512 k7 N512", 16, 512, 6, 7, 512, 1, 1, fat);
  conv("sea.convtr1 T16 c512 N256 x6", 16, 512, 1, 2, 256, 6, 6, fat);
  conv("sea.res1a T96 c256 k3 N128", 96, 256, 2, 3, 128, 1, 1, fat);
  conv("sea.convtr2 T96 c256 N128 x5", 96, 256, 1, 2, 128, 5, 5, fat);
  conv("sea.res2a T480 c128 k3 N64", 480, 128, 2, 3, 64, 1, 1, fat);
  conv("sea.convtr3 T480 c128 N64 x4", 480, 128, 1, 2, 64, 4, 4, fat);
  conv("sea.res3a T1920 c64 k3 N32", 1920, 64, 2, 3, 32, 1, 1, fat);
  conv("sea.res3b T1920 c32 k1 N64", 1920, 32, 0, 1, 64, 1, 1, fat);
  // register-blocked LDS-DMA tiles; transposed convs with the r phases merged into N (one
  // 2-tap conv whose output row q holds the r output rows q*r .. q*r+r-1)
  std::vector<std::pair<int, int>> rb = {{6, 1}, {12, 1}, {20, 1}, {21, 1}, {22, 1}, {23, 1}, {24, 1},
                                         {25, 1}, {26, 1}, {27, 1}};
  std::vector<std::pair<int, int>> rbk = {{0, 1}, {21, 1}, {21, 2}, {21, 4}, {22, 1}, {22, 2}, {22, 4},
                                          {23, 2}, {23, 4}, {25, 2}, {25, 4}, {27, 2}, {27, 4}};
  conv("rb.conv0 T16 c512 k7 N512", 16, 512, 6, 7, 512, 1, 1, rbk);
  conv("rb.convtr1m T16 c512 N1536", 16, 512, 1, 2, 1536, 1, 1, rb);
  conv("rb.res1a T96 c256 k3 N128", 96, 256, 2, 3, 128, 1, 1, rbk);
  conv("rb.res1b T96 c128 k1 N256", 96, 128, 0, 1, 256, 1, 1, rb);
  conv("rb.convtr2m T96 c256 N640", 96, 256, 1, 2, 640, 1, 1, rb);
  conv("rb.res2a T480 c128 k3 N64", 480, 128, 2, 3, 64, 1, 1, rb);
  conv("rb.res2b T480 c64 k1 N128", 480, 64, 0, 1, 128, 1, 1, rb);
  conv("rb.convtr3m T480 c128 N256", 480, 128, 1, 2, 256, 1, 1, rb);
  conv("rb.res3a T1920 c64 k3 N32", 1920, 64, 2, 3, 32, 1, 1, rb);
  conv("rb.res3b T1920 c32 k1 N64", 1920, 32, 0, 1, 64, 1, 1, rb);
  // shape study: the convtr3m GEMM as a dense GEMM, and the same flops at long K
  dense("study.dense M15360 N256 K256", 15360, 256, 256, rb);
  dense("study.dense M3840 N256 K1024", 3840, 256, 1024, rb);
  dense("study.dense M1920 N256 K2048", 1920, 256, 2048, rb);
  dense("study.dense M30720 N256 K128", 30720, 256, 128, rb);
  std::vector<std::pair<int, int>> kv = {{0, 1}, {9, 1}, {10, 1}, {17, 1}, {18, 1}, {6, 2}, {6, 4}, {6, 8},
                                         {12, 4}, {22, 4}, {22, 8}, {23, 8}, {25, 8}, {27, 8}};
  conv("c0.conv0 T16 c512 k7 N512", 16, 512, 6, 7, 512, 1, 1, kv);
  std::vector<std::pair<int, int>> kv2 = {{6, 1}, {6, 2}, {6, 4}, {20, 1}, {22, 1}, {22, 2}, {22, 4}, {12, 2},
                                          {27, 2}, {25, 2}, {23, 2}};
  conv("c1.convtr1m T16 c512 N1536", 16, 512, 1, 2, 1536, 1, 1, kv2);
  std::vector<std::pair<int, int>> kv3 = {{6, 1}, {14, 1}, {3, 1}, {0, 1}, {24, 1}, {25, 1}, {12, 1}, {11, 1}};
  conv("c1.res3a T1920 c64 k3 N32", 1920, 64, 2, 3, 32, 1, 1, kv3);
  conv("c1.res3b T1920 c32 k1 N64", 1920, 32, 0, 1, 64, 1, 1, kv3);
  conv("c1.res2a T480 c128 k3 N64", 480, 128, 2, 3, 64, 1, 1, kv3);
  std::vector<std::pair<int, int>> kv4 = {{6, 1}, {6, 2}, {22, 1}, {22, 2}, {12, 1}, {12, 2}, {11, 1}, {27, 1},
                                          {13, 1}, {16, 1}, {15, 1}};
  conv("c2.convtr2m T96 c256 N640", 96, 256, 1, 2, 640, 1, 1, kv4);
  conv("c2.convtr3m T480 c128 N256", 480, 128, 1, 2, 256, 1, 1, kv4);
  conv("c2.res1a T96 c256 k3 N128", 96, 256, 2, 3, 128, 1, 1, kv4);
  conv("c2.res1b T96 c128 k1 N256", 96, 128, 0, 1, 256, 1, 1, kv4);
  dense("c2.mimi.qkv M512 N1536 K512", 16 * B, 1536, 512, kv4);
  dense("c2.mimi.ff1 M512 N2048 K512", 16 * B, 2048, 512, kv4);
  conv("c0.res1a T96 c256 k3 N128", 96, 256, 2, 3, 128, 1, 1, kv);
  dense("c0.mimi.ff2 M512 N512 K2048", 16 * B, 512, 2048, kv);
  std::vector<std::pair<int, int>> lk = {{6, 1}, {21, 1}, {22, 1}};
  dense("kstudy M3840 N256 K32", 3840, 256, 32, lk);
  dense("kstudy M3840 N256 K64", 3840, 256, 64, lk);
  dense("kstudy M3840 N256 K128", 3840, 256, 128, lk);
  dense("kstudy M3840 N256 K256", 3840, 256, 256, lk);
  dense("kstudy M3840 N256 K512", 3840, 256, 512, lk);
  dense("kstudy M256 N256 K32", 256, 256, 32, lk);
  dense("kstudy M256 N256 K1024", 256, 256, 1024, lk);
  dense("rb.mimi.qkv M512 N1536 K512", 16 * B, 1536, 512, rbk);
  dense("rb.mimi.ff1 M512 N2048 K512", 16 * B, 2048, 512, rbk);
  dense("rb.mimi.ff2 M512 N512 K2048", 16 * B, 512, 2048, rbk);
  dense("rb.mimi.out M512 N512 K512", 16 * B, 512, 512, rbk);

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& c : cases) {
    if (only_case && c.name.find(only_case) == std::string::npos) continue;
    GemmArgs a = c.a;
    const long out_n = (long)c.phases * a.M * a.N;
    for (int ph = 0; ph < c.phases; ++ph)
      hipLaunchKernelGGL(k_ref, dim3((a.M * a.N + 255) / 256), dim3(256), 0, st, a, ph, ref);
    std::vector<float> href(out_n);
    CK(hipMemcpyAsync(href.data(), ref, out_n * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const double flops = 2.0 * a.M * a.N * a.K * c.phases;
    const double wbytes = 4.0 * c.phases * a.N * a.K;
    printf("== %s  (%.1f MFLOP, W %.2f MB)\n", c.name.c_str(), flops / 1e6, wbytes / 1e6);
    for (auto [layout, S] : c.variants) {
      if (only_layout >= 0 && (layout != only_layout || (only_s >= 0 && S != only_s))) continue;
      GemmArgs v = a;
      v.layout = layout;
      const int bk = (layout == 8 || layout == 15 || layout == 16) ? 64 : 32;
      if (layout >= 6 && (a.K % bk != 0 || (a.mode == 1 && a.cin % bk != 0))) continue;
      int gz = c.phases;
      if (S > 1 && a.mode == 1 && (c.phases > 1 || layout < 6 || (layout >= 9 && layout <= 10) ||
                                   (layout >= 17 && layout <= 20))) continue;
      if (S > 1) {  // dense split-K, or K-sliced single-phase conv (register-blocked LDS-DMA)
        if (a.K / bk < S) continue;
        v.S = S;
        v.partial = P;
        gz = S;
      } else {
        v.S = 1;
        v.partial = nullptr;
      }
      gemm(v, gz, st);
      CK(hipGetLastError());
      hipLaunchKernelGGL(k_collect, dim3((out_n + 255) / 256), dim3(256), 0, st, v, c.phases, v.partial ? P : Y, got);
      std::vector<float> hgot(out_n);
      CK(hipMemcpyAsync(hgot.data(), got, out_n * 4, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      double err = 0, mx = 0;
      for (long i = 0; i < out_n; ++i) {
        err = std::max(err, (double)fabsf(hgot[i] - href[i]));
        mx = std::max(mx, (double)fabsf(href[i]));
      }
      for (int i = 0; i < 3; ++i) gemm(v, gz, st);
      const int reps = 50;
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) gemm(v, gz, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1000.0 * ms / reps;
      printf("   layout %d S %2d : %8.2f us  %7.1f TF/s  W %6.0f GB/s  relerr %.1e %s\n", layout, S, us,
             flops / us / 1e6, wbytes / us / 1e3, err / (mx + 1e-30), err / (mx + 1e-30) < 1e-5 ? "" : "BAD");
    }
  }
  return 0;
}
