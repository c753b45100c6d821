// Standalone check + A/B of the one-wave-per-SIMD GEMM (csrc/kernels/gemm4.hip) against the
// 8-wave gemm_tile.hip kernel on the Llama-3-70B decode shapes (M = 512), random operands,
// weights rotated past the Infinity Cache, interleaved rounds in one process.
//
// Both kernels run the same MFMA instruction with the same operand order over the same k order,
// so the bf16 store and the fp32 split-K partials must be BIT-identical; the fused SwiGLU output
// is checked against silu(gate) * up recomputed on the host from the plain product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_llm_inference/csrc/kernels \
//         scripts/experiments/gemm4_bench.hip -o tools_bin/gemm4_bench
//   tools_bin/gemm4_bench [rounds] [gate|up grid override]
#define GEMM_STAMPS 1
#define DLI_GEMM4_ALL_VARIANTS 1
#include "../../distributed_llm_inference/csrc/kernels/gemm_tile.hip"
#include "../../distributed_llm_inference/csrc/kernels/gemm4.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void fill_rand(__bf16* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (__bf16)(((float)(x & 0xffffff) / 16777216.f * 2.f - 1.f) * scale);
  }
}

__global__ void fill_fp8(unsigned char* p, size_t n, unsigned seed) {   // finite e4m3, |x| < 256
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (unsigned char)(x & 0xF7u);   // exponent field <= 14
  }
}

static float bf2f(__bf16 v) { return (float)v; }
static bool g_fp8 = false;   // argv[3] == "fp8": time the fp8 e4m3 paths (checks: tests/test_gemm_gpu.py)

struct Shape { const char* name; int M, N, K, splits, epi; };

static int g_grid = 0;
static int g_var = 0;   // gemm4 schedule variant under check
constexpr int kVars = 10;

static int check(const Shape& c) {
  int bad = 0;
  for (int M : {c.M, 300, 40}) {
    const int N = c.N, K = c.K;
    __bf16 *A, *B, *C0, *C1;
    float *W0 = nullptr, *W1 = nullptr;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C0, (size_t)M * N * 2));
    CK(hipMalloc(&C1, (size_t)M * N * 2));
    fill_rand<<<1024, 256>>>(A, (size_t)M * K, 3, 1.f);
    fill_rand<<<4096, 256>>>(B, (size_t)N * K, 11, 0.05f);
    const bool sk = c.splits > 1;
    if (sk) {
      CK(hipMalloc(&W0, (size_t)c.splits * M * N * 4));
      CK(hipMalloc(&W1, (size_t)c.splits * M * N * 4));
    }
    int r0 = dli::launch_gemm_tile(C0, A, B, nullptr, nullptr, W0, M, N, K, c.splits, sk ? 1 : 0,
                                   0, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
    int r1 = dli::launch_gemm4(sk ? (void*)W1 : (void*)C1, A, B, M, N, K, c.splits, sk ? 1 : 0,
                               0, 0, g_var);
    CK(hipDeviceSynchronize());
    if (r0 || r1) { printf("launch rc %d %d\n", r0, r1); return 1; }
    size_t nbytes = sk ? (size_t)c.splits * M * N * 4 : (size_t)M * N * 2;
    std::vector<char> h0(nbytes), h1(nbytes);
    CK(hipMemcpy(h0.data(), sk ? (void*)W0 : (void*)C0, nbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), sk ? (void*)W1 : (void*)C1, nbytes, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < nbytes; ++i) diff += h0[i] != h1[i];
    printf("check v%d %-16s M=%d %s: %zu differing bytes of %zu\n", g_var, c.name, M,
           sk ? "fp32 partials" : "bf16 store", diff, nbytes);
    bad += diff != 0;
    if (sk) {   // bf16 partials: the same sums rounded
      __bf16* P1;
      CK(hipMalloc(&P1, (size_t)c.splits * M * N * 2));
      int r2 = dli::launch_gemm4(P1, A, B, M, N, K, c.splits, 4, 0, 0, g_var);
      CK(hipDeviceSynchronize());
      if (r2) { printf("bf16 parts rc %d\n", r2); return 1; }
      std::vector<__bf16> hp((size_t)c.splits * M * N);
      CK(hipMemcpy(hp.data(), P1, hp.size() * 2, hipMemcpyDeviceToHost));
      const float* f = reinterpret_cast<const float*>(h0.data());
      size_t nd = 0;
      for (size_t i = 0; i < hp.size(); ++i) nd += bf2f(hp[i]) != bf2f((__bf16)f[i]);
      printf("check %-16s M=%d bf16 partials: %zu differing of %zu\n", c.name, M, nd, hp.size());
      bad += nd != 0;
      CK(hipFree(P1));
    }
    if (!sk && c.epi == 2) {
      __bf16* S;
      CK(hipMalloc(&S, (size_t)M * N));
      int r2 = dli::launch_gemm4(S, A, B, M, N, K, 1, 2, 0, 0, g_var);
      CK(hipDeviceSynchronize());
      if (r2) { printf("swiglu rc %d\n", r2); return 1; }
      std::vector<__bf16> hs((size_t)M * N / 2), hp((size_t)M * N);
      CK(hipMemcpy(hs.data(), S, hs.size() * 2, hipMemcpyDeviceToHost));
      memcpy(hp.data(), h1.data(), hp.size() * 2);
      double maxerr = 0;
      size_t nbad = 0;
      for (int m = 0; m < M; ++m)
        for (int c2 = 0; c2 < N; ++c2) {
          if ((c2 / 16) & 1) continue;   // gate columns: 16-blocks 2p; up = +16
          const int out = (c2 / 32) * 16 + c2 % 16;
          const float g = bf2f(hp[(size_t)m * N + c2]), u = bf2f(hp[(size_t)m * N + c2 + 16]);
          const float ref = g / (1.f + expf(-g)) * u;
          const float got = bf2f(hs[(size_t)m * (N / 2) + out]);
          const double err = fabs(got - ref) / (fabs(ref) + 1e-2);
          maxerr = std::max(maxerr, err);
          nbad += err > 2e-2;
        }
      printf("check %-16s M=%d swiglu: max rel err %.3g, %zu elements over 2e-2\n", c.name, M,
             maxerr, nbad);
      bad += nbad != 0;
      CK(hipFree(S));
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C0)); CK(hipFree(C1));
    if (W0) { CK(hipFree(W0)); CK(hipFree(W1)); }
  }
  return bad;
}

int main(int argc, char** argv) {
  std::vector<Shape> shapes = {
      {"gate_up_swiglu", 512, 57344, 8192, 1, 2},
      {"down_s4", 512, 8192, 28672, 4, 1},
      {"qkv_s3", 512, 10240, 8192, 3, 1},
      {"o_s4", 512, 8192, 8192, 4, 1},
      {"sq8192", 8192, 8192, 8192, 1, 0},
  };
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  if (argc > 2) g_grid = atoi(argv[2]);
  g_fp8 = argc > 3 && strcmp(argv[3], "fp8") == 0;
  // every launch of this build writes per-workgroup stamps: point them at a buffer first
  unsigned long long* sb;
  CK(hipMalloc(&sb, (size_t)8192 * 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(dli::g_stamp_blk), &sb, sizeof(sb)));
  int bad = 0;
  for (g_var = 0; g_var < kVars && !g_fp8; ++g_var)
    for (auto& c : shapes)
      if (c.M <= 512) bad += check(c);
  if (bad) { printf("CHECK FAILED\n"); return 2; }
  for (auto& c : shapes) {
    const int esz = g_fp8 ? 1 : 2;
    const size_t wbytes = (size_t)c.N * c.K * esz;
    const int sets = (int)std::max<size_t>(2, std::min<size_t>(6, 1200000000ull / wbytes + 1));
    __bf16 *A, *C;
    std::vector<__bf16*> B(sets);
    float* ws = nullptr;
    float *sa, *sb8;
    CK(hipMalloc(&sa, (size_t)c.M * 4));
    CK(hipMalloc(&sb8, (size_t)c.N * 4));
    {
      std::vector<float> ones((size_t)std::max(c.M, c.N), 1.f / 64);
      CK(hipMemcpy(sa, ones.data(), (size_t)c.M * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(sb8, ones.data(), (size_t)c.N * 4, hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&A, (size_t)c.M * c.K * esz));
    for (auto& b : B) CK(hipMalloc(&b, wbytes));
    CK(hipMalloc(&C, (size_t)c.M * c.N * 2));
    if (c.splits > 1) CK(hipMalloc(&ws, (size_t)c.splits * c.M * c.N * 4));
    // the production gate|up launch of the 8-wave kernel: whole tiles + stream-K tail
    const bool tile_sk = !g_fp8 && c.epi == 2 && dli::gemm_tile_sk_workspace_floats() > 0;
    float* sk_ws = nullptr;
    if (tile_sk) CK(hipMalloc(&sk_ws, (size_t)dli::gemm_tile_sk_workspace_floats() * 4));
    if (g_fp8) {
      fill_fp8<<<1024, 256>>>((unsigned char*)A, (size_t)c.M * c.K, 1);
      for (int i = 0; i < sets; ++i) fill_fp8<<<4096, 256>>>((unsigned char*)B[i], (size_t)c.N * c.K, 7 + i);
    } else {
      fill_rand<<<1024, 256>>>(A, (size_t)c.M * c.K, 1, 1.f);
      for (int i = 0; i < sets; ++i) fill_rand<<<4096, 256>>>(B[i], (size_t)c.N * c.K, 7 + i, 0.02f);
    }
    const int epi = c.splits > 1 ? 1 : c.epi;
    const int grid = (c.epi == 2 && g_grid > 0) ? g_grid : 0;
    auto run = [&](int v, int i) {
      int rc = v == 0 ? dli::launch_gemm_tile(C, A, B[i % sets], g_fp8 ? sa : nullptr,
                                              g_fp8 ? sb8 : nullptr, tile_sk ? sk_ws : ws, c.M,
                                              c.N, c.K, tile_sk ? 0 : c.splits, epi,
                                              g_fp8 ? dli::kFp8 : 0, 0, nullptr, nullptr, 0,
                                              nullptr, nullptr, nullptr)
                      : dli::launch_gemm4(c.splits > 1 ? (void*)ws : (void*)C, A, B[i % sets],
                                          c.M, c.N, c.K, c.splits, epi, grid, 0, v - 1,
                                          g_fp8 ? 1 : 0, g_fp8 ? sa : nullptr,
                                          g_fp8 ? sb8 : nullptr);
      if (rc) { fprintf(stderr, "rc %d\n", rc); exit(1); }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> t[1 + kVars];
    const int iters = c.M > 512 ? 5 : 20;
    for (int v = 0; v <= kVars; ++v) for (int i = 0; i < 5; ++i) run(v, i);
    for (int r = 0; r < rounds; ++r)
      for (int vv = 0; vv <= kVars; ++vv) {
        const int v = (r & 1) ? kVars - vv : vv;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) run(v, i);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1e3 / iters);
      }
    for (auto& x : t) std::sort(x.begin(), x.end());
    // one stamped launch of each: per-workgroup cycles of the k-loops and the clock
    for (int v = 0; v <= kVars; ++v) {
      const int tiles = ((c.M + 255) / 256) * (c.N / 256);
      const int items = tiles * c.splits;
      const bool sk0 = v == 0 && tile_sk;
      int wgs = v == 0 ? (sk0 ? tiles / 256 * 256 + 256 : items)
                       : (grid > 0 ? grid : dli::gemm4_grid(items, 256));
      CK(hipMemset(sb, 0, (size_t)8192 * 64));
      run(v, 0);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> h((size_t)wgs * 8);
      CK(hipMemcpy(h.data(), sb, h.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> cyc, clk, life;
      unsigned long long t0 = ~0ull, s1 = 0, e1 = 0;
      for (int b = 0; b < wgs; ++b) {
        const unsigned long long* q = &h[(size_t)b * 8];
        if (q[3] <= q[1]) continue;
        t0 = std::min(t0, q[0]);
        s1 = std::max(s1, q[0]);
        e1 = std::max(e1, q[2]);
        life.push_back((q[2] - q[0]) / 100.0);
        cyc.push_back((double)(q[3] - q[1]));
        const double us = (q[2] - q[0]) / 100.0;
        if (us > 0) clk.push_back((q[3] - q[1]) / us / 1e3);
      }
      std::sort(cyc.begin(), cyc.end());
      std::sort(clk.begin(), clk.end());
      std::sort(life.begin(), life.end());
      if (!life.empty())   // dispatch skew and the slowest workgroup, wall-clock (100 MHz ticks)
        printf("%-16s %s%d wall: start skew %.1f us, WG life med %.1f / max %.1f us, span %.1f us\n",
               c.name, v == 0 ? "gemm_tile" : "gemm4 v", v - 1, (s1 - t0) / 100.0,
               life[life.size() / 2], life.back(), (e1 - t0) / 100.0);
      // k-tiles per workgroup: gemm_tile = one item each (stream-K: ~ the same), gemm4 = items / grid
      const double kt_item = (double)c.K * esz / 128 / c.splits;
      const double per_wg = v == 0 ? kt_item * (double)items / wgs : kt_item * ((double)items / wgs);
      if (!cyc.empty())
        printf("%-16s %s%d stamps: %d wgs, med %.0f cyc/wg = %.0f per k-tile, clock %.2f GHz\n",
               c.name, v == 0 ? "gemm_tile" : "gemm4 v", v - 1, wgs, cyc[cyc.size() / 2],
               cyc[cyc.size() / 2] / per_wg, clk.empty() ? 0.0 : clk[clk.size() / 2]);
    }
    const double fl = 2.0 * c.M * c.N * c.K;
    printf("%s%-16s M=%d N=%d K=%d s=%d | gemm_tile %.1f us (min %.1f, %.0f TF)", g_fp8 ? "fp8 " : "", c.name, c.M, c.N,
           c.K, c.splits, t[0][t[0].size() / 2], t[0][0], fl / t[0][t[0].size() / 2] / 1e6);
    for (int v = 1; v <= kVars; ++v)
      printf(" | v%d %.1f us (%.0f TF, %.3f)", v - 1, t[v][t[v].size() / 2],
             fl / t[v][t[v].size() / 2] / 1e6, t[v][t[v].size() / 2] / t[0][t[0].size() / 2]);
    printf("\n");
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(sa)); CK(hipFree(sb8));
    for (auto& b : B) CK(hipFree(b));
    CK(hipFree(C));
    if (ws) CK(hipFree(ws));
    if (sk_ws) CK(hipFree(sk_ws));
  }
  return 0;
}
