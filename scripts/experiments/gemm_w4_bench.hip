// Standalone check + A/B of the 4-wave tile GEMM (gemm_w4.hip) against the 8-wave gemm_tile.hip
// kernel on the Llama-3-70B decode shapes (M = 512), random operands, weights rotated past the
// Infinity Cache, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
//
// Correctness: the two kernels run the same MFMA instruction over the same k order, so the bf16
// store and the fp32 split-K partials must be BIT-identical; the fused SwiGLU output is checked
// against silu(gate) * up recomputed on the host from the plain product (its own interleave).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_llm_inference/csrc/kernels \
//         -I scripts/experiments scripts/experiments/gemm_w4_bench.hip -o tools_bin/gemm_w4_bench
#define GEMM_STAMPS 1
#include "gemm_tile.hip"
#include "gemm_w4.hip"

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

static float bf2f(__bf16 v) { return (float)v; }

static int g_pipe = 2;

struct Shape { const char* name; int M, N, K, splits, epi; };

static int check(const Shape& c) {
  // small-M variants of the shape (partial M tile) and the full one
  int bad = 0;
  for (int M : {c.M, 300}) {
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
    int r0 = dli::launch_gemm_tile(C0, A, B, nullptr, nullptr, W0, M, N, K, c.splits, sk ? 1 : 0, 0, 0);
    int r1 = dli::launch_gemm_w4(C1, A, B, W1, M, N, K, c.splits, sk ? 1 : 0, 0, g_pipe);
    CK(hipDeviceSynchronize());
    if (r0 || r1) { printf("launch rc %d %d\n", r0, r1); return 1; }
    size_t nbytes = sk ? (size_t)c.splits * M * N * 4 : (size_t)M * N * 2;
    std::vector<char> h0(nbytes), h1(nbytes);
    CK(hipMemcpy(h0.data(), sk ? (void*)W0 : (void*)C0, nbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), sk ? (void*)W1 : (void*)C1, nbytes, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < nbytes; ++i) diff += h0[i] != h1[i];
    printf("check %-16s M=%d %s: %zu differing bytes of %zu\n", c.name, M,
           sk ? "fp32 partials" : "bf16 store", diff, nbytes);
    bad += diff != 0;
    if (!sk && c.epi == 2) {
      // fused SwiGLU (w4 interleave: tile-local row c -> wave column c/128, fragment (c%128)/16)
      __bf16* S;
      CK(hipMalloc(&S, (size_t)M * N));
      int r2 = dli::launch_gemm_w4(S, A, B, nullptr, M, N, K, 1, 2, 0, g_pipe);
      CK(hipDeviceSynchronize());
      if (r2) { printf("swiglu rc %d\n", r2); return 1; }
      std::vector<__bf16> hs((size_t)M * N / 2), hp((size_t)M * N);
      CK(hipMemcpy(hs.data(), S, hs.size() * 2, hipMemcpyDeviceToHost));
      memcpy(hp.data(), h1.data(), hp.size() * 2);
      double maxerr = 0;
      size_t nbad = 0;
      for (int m = 0; m < M; ++m)
        for (int c2 = 0; c2 < N; ++c2) {
          const int tile = c2 / 256, cl = c2 % 256, wave = cl / 128, f = (cl % 128) / 16, lc = cl % 16;
          if (f & 1) continue;
          const int out = tile * 128 + wave * 64 + (f / 2) * 16 + lc;
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
  };
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  if (argc > 2) g_pipe = atoi(argv[2]);
  printf("gemm_w4 pipeline variant %d\n", g_pipe);
  // every launch of this build writes per-workgroup stamps: point them at a buffer first
  unsigned long long* sb;
  CK(hipMalloc(&sb, (size_t)8192 * 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(dli::g_stamp_blk), &sb, sizeof(sb)));
  int bad = 0;
  for (auto& c : shapes) bad += check(c);
  if (bad) { printf("CHECK FAILED\n"); return 2; }
  for (auto& c : shapes) {
    const size_t wbytes = (size_t)c.N * c.K * 2;
    const int sets = (int)std::max<size_t>(2, std::min<size_t>(6, 1200000000ull / wbytes + 1));
    __bf16 *A, *C;
    std::vector<__bf16*> B(sets);
    float* ws = nullptr;
    CK(hipMalloc(&A, (size_t)c.M * c.K * 2));
    for (auto& b : B) CK(hipMalloc(&b, wbytes));
    CK(hipMalloc(&C, (size_t)c.M * c.N * 2));
    if (c.splits > 1) CK(hipMalloc(&ws, (size_t)c.splits * c.M * c.N * 4));
    fill_rand<<<1024, 256>>>(A, (size_t)c.M * c.K, 1, 1.f);
    for (int i = 0; i < sets; ++i) fill_rand<<<4096, 256>>>(B[i], (size_t)c.N * c.K, 7 + i, 0.02f);
    const int epi = c.splits > 1 ? 1 : c.epi;
    auto run = [&](int v, int i) {
      int rc = v == 0 ? dli::launch_gemm_tile(C, A, B[i % sets], nullptr, nullptr, ws, c.M, c.N, c.K,
                                              c.splits, epi, 0, 0)
                      : dli::launch_gemm_w4(C, A, B[i % sets], ws, c.M, c.N, c.K, c.splits, epi, 0, g_pipe);
      if (rc) { fprintf(stderr, "rc %d\n", rc); exit(1); }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> t[2];
    const int iters = 20;
    for (int v = 0; v < 2; ++v) for (int i = 0; i < 5; ++i) run(v, i);
    for (int r = 0; r < rounds; ++r)
      for (int vv = 0; vv < 2; ++vv) {
        const int v = (r & 1) ? 1 - vv : vv;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) run(v, i);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1e3 / iters);
      }
    for (auto& x : t) std::sort(x.begin(), x.end());
    // one stamped launch of each: per-workgroup cycles (whole, main loop), clock
    const int wgs = ((c.M + 255) / 256) * (c.N / 256) * c.splits;
    if (wgs > 8192) { fprintf(stderr, "too many workgroups for the stamp buffer\n"); return 1; }
    double st_cyc[2], st_loop[2], st_clk[2];
    for (int v = 0; v < 2; ++v) {
      CK(hipMemset(sb, 0, (size_t)wgs * 64));
      for (int i = 0; i < 10; ++i) run(v, i);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> h((size_t)wgs * 8);
      CK(hipMemcpy(h.data(), sb, h.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> cyc, loop, clk;
      for (int b = 0; b < wgs; ++b) {
        const unsigned long long* q = &h[(size_t)b * 8];
        cyc.push_back((double)(q[3] - q[1]));
        loop.push_back((double)(q[7] - q[1]));
        const double us = (q[2] - q[0]) / 100.0;
        if (us > 0) clk.push_back((q[3] - q[1]) / us / 1e3);
      }
      std::sort(cyc.begin(), cyc.end());
      std::sort(loop.begin(), loop.end());
      std::sort(clk.begin(), clk.end());
      st_cyc[v] = cyc[cyc.size() / 2];
      st_loop[v] = loop[loop.size() / 2];
      st_clk[v] = clk[clk.size() / 2];
    }
    const int kt = c.K * 2 / 128 / c.splits;
    printf("%-16s stamps: gemm_tile %.0f cyc/wg (loop %.0f = %.0f per k-tile), %.2f GHz | gemm_w4 "
           "%.0f cyc/wg (loop %.0f = %.0f per k-tile), %.2f GHz\n",
           c.name, st_cyc[0], st_loop[0], st_loop[0] / kt, st_clk[0], st_cyc[1], st_loop[1],
           st_loop[1] / kt, st_clk[1]);
    const double fl = 2.0 * c.M * c.N * c.K;
    printf("%-16s M=%d N=%d K=%d s=%d | gemm_tile %.1f us (min %.1f, %.0f TF) | gemm_w4 %.1f us "
           "(min %.1f, %.0f TF) | w4/tile %.3f\n",
           c.name, c.M, c.N, c.K, c.splits, t[0][t[0].size() / 2], t[0][0],
           fl / t[0][t[0].size() / 2] / 1e6, t[1][t[1].size() / 2], t[1][0],
           fl / t[1][t[1].size() / 2] / 1e6, t[1][t[1].size() / 2] / t[0][t[0].size() / 2]);
    fflush(stdout);
    CK(hipFree(A));
    for (auto& b : B) CK(hipFree(b));
    CK(hipFree(C));
    if (ws) CK(hipFree(ws));
  }
  return 0;
}
