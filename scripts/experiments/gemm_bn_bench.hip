// Tile-width A/B of the tile GEMM (gemm_tile.hip, tile 256 x bn) on the Llama-3-70B decode shapes
// at M = 512: correctness (every bn produces the BIT-identical bf16 product: same MFMA, same k
// order; fused SwiGLU vs silu(gate) * up recomputed on the host) and time per (bn, splits)
// candidate, interleaved rounds in one process, random operands, weights rotated past the
// Infinity Cache; per-workgroup clock stamps give cycles per k-tile and the clock.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_llm_inference/csrc/kernels \
//         -I scripts/experiments scripts/experiments/gemm_bn_bench.hip -o tools_bin/gemm_bn_bench
#define GEMM_STAMPS 1
#include "gemm_tile_bn.hip"   // scripts/experiments: the generalized (rejected) kernel

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

struct Cand { int bn, splits; };
struct Shape { const char* name; int M, N, K; bool swiglu; std::vector<Cand> cands; };

static int check(int M, int N, int K) {
  __bf16 *A, *B, *C0, *C1, *S;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C0, (size_t)M * N * 2));
  CK(hipMalloc(&C1, (size_t)M * N * 2));
  CK(hipMalloc(&S, (size_t)M * N));
  fill_rand<<<1024, 256>>>(A, (size_t)M * K, 3, 1.f);
  fill_rand<<<4096, 256>>>(B, (size_t)N * K, 11, 0.05f);
  int bad = 0;
  std::vector<__bf16> h0((size_t)M * N), h1((size_t)M * N), hs((size_t)M * N / 2);
  if (dli::launch_gemm_tile(C0, A, B, nullptr, nullptr, nullptr, M, N, K, 1, 0, 0, 0, 256)) return 1;
  CK(hipMemcpy(h0.data(), C0, h0.size() * 2, hipMemcpyDeviceToHost));
  for (int bn : {128, 160, 192, 224, 256}) {
    if (N % bn) continue;
    CK(hipMemset(C1, 0xff, (size_t)M * N * 2));
    if (dli::launch_gemm_tile(C1, A, B, nullptr, nullptr, nullptr, M, N, K, 1, 0, 0, 0, bn)) return 1;
    if (dli::launch_gemm_tile(S, A, B, nullptr, nullptr, nullptr, M, N, K, 1, 2, 0, 0, bn)) return 1;
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h1.data(), C1, h1.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), S, hs.size() * 2, hipMemcpyDeviceToHost));
    const size_t diff = memcmp(h0.data(), h1.data(), h0.size() * 2) ? 1 : 0;
    double maxerr = 0;
    size_t nbad = 0;
    for (int m = 0; m < M; ++m)
      for (int c = 0; c < N / 2; ++c) {
        const float g = (float)h1[(size_t)m * N + 2 * c], u = (float)h1[(size_t)m * N + 2 * c + 1];
        const float ref = g / (1.f + expf(-g)) * u, got = (float)hs[(size_t)m * (N / 2) + c];
        const double err = fabs(got - ref) / (fabs(ref) + 1e-2);
        maxerr = std::max(maxerr, err);
        nbad += err > 2e-2;
      }
    printf("check M=%d N=%d K=%d bn=%d: store %s, swiglu max rel err %.3g (%zu over 2e-2)\n", M, N,
           K, bn, diff ? "DIFFERS" : "bit-identical", maxerr, nbad);
    bad += diff != 0 || nbad != 0;
  }
  CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C0)); CK(hipFree(C1)); CK(hipFree(S));
  return bad;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  unsigned long long* sb;
  CK(hipMalloc(&sb, (size_t)16384 * 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(dli::g_stamp_blk), &sb, sizeof(sb)));
  int bad = check(512, 57344 / 4, 8192) + check(300, 8960, 4096) + check(512, 10240, 1024);
  if (bad) { printf("CHECK FAILED\n"); return 2; }
  std::vector<Shape> shapes = {
      {"gate_up_swiglu", 512, 57344, 8192, true, {{256, 1}, {224, 1}}},
      {"qkv", 512, 10240, 8192, false, {{256, 3}, {160, 2}, {256, 2}, {128, 2}}},
      {"o", 512, 8192, 8192, false, {{256, 4}, {128, 2}, {256, 2}, {128, 4}}},
      {"down", 512, 8192, 28672, false, {{256, 4}, {128, 2}, {128, 4}}},
      {"gate_up_swiglu_M256", 256, 57344, 8192, true, {{256, 1}, {224, 1}}},
  };
  for (auto& c : shapes) {
    const size_t wbytes = (size_t)c.N * c.K * 2;
    const int sets = (int)std::max<size_t>(2, std::min<size_t>(6, 1200000000ull / wbytes + 1));
    __bf16 *A, *C;
    std::vector<__bf16*> B(sets);
    float* ws = nullptr;
    CK(hipMalloc(&A, (size_t)c.M * c.K * 2));
    for (auto& b : B) CK(hipMalloc(&b, wbytes));
    CK(hipMalloc(&C, (size_t)c.M * c.N * 2));
    CK(hipMalloc(&ws, (size_t)8 * c.M * c.N * 4));
    fill_rand<<<1024, 256>>>(A, (size_t)c.M * c.K, 1, 1.f);
    for (int i = 0; i < sets; ++i) fill_rand<<<4096, 256>>>(B[i], (size_t)c.N * c.K, 7 + i, 0.02f);
    const int nv = (int)c.cands.size();
    auto run = [&](int v, int i) {
      const Cand& d = c.cands[v];
      const int epi = d.splits > 1 ? 1 : (c.swiglu ? 2 : 0);
      int rc = dli::launch_gemm_tile(C, A, B[i % sets], nullptr, nullptr, ws, c.M, c.N, c.K,
                                     d.splits, epi, 0, 0, d.bn);
      if (rc) { fprintf(stderr, "rc %d\n", rc); exit(1); }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> t(nv);
    const int iters = 20;
    for (int v = 0; v < nv; ++v) for (int i = 0; i < 5; ++i) run(v, i);
    for (int r = 0; r < rounds; ++r)
      for (int vv = 0; vv < nv; ++vv) {
        const int v = (r & 1) ? nv - 1 - vv : vv;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) run(v, i);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1e3 / iters);
      }
    const double fl = 2.0 * c.M * c.N * c.K;
    for (int v = 0; v < nv; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const Cand& d = c.cands[v];
      const int wgs = ((c.M + 255) / 256) * (c.N / d.bn) * d.splits;
      CK(hipMemset(sb, 0, (size_t)wgs * 64));
      for (int i = 0; i < 10; ++i) run(v, i);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> h((size_t)wgs * 8);
      CK(hipMemcpy(h.data(), sb, h.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> loop, clk;
      for (int b = 0; b < wgs; ++b) {
        const unsigned long long* q = &h[(size_t)b * 8];
        loop.push_back((double)(q[7] - q[1]));
        const double us = (q[2] - q[0]) / 100.0;
        if (us > 0) clk.push_back((q[3] - q[1]) / us / 1e3);
      }
      std::sort(loop.begin(), loop.end());
      std::sort(clk.begin(), clk.end());
      const int kt = (c.K * 2 / 128 + d.splits - 1) / d.splits;
      printf("%-20s bn=%3d splits=%d wgs=%4d | %7.1f us (min %7.1f) %5.0f TF | loop %6.0f cyc/k-tile "
             "(%5.0f per 256-wide) | %.2f GHz\n",
             c.name, d.bn, d.splits, wgs, t[v][t[v].size() / 2], t[v][0], fl / t[v][t[v].size() / 2] / 1e6,
             loop[loop.size() / 2] / kt, loop[loop.size() / 2] / kt * 256.0 / d.bn,
             clk[clk.size() / 2]);
    }
    fflush(stdout);
    CK(hipFree(A));
    for (auto& b : B) CK(hipFree(b));
    CK(hipFree(C));
    CK(hipFree(ws));
  }
  return 0;
}
