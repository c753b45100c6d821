// Clock-stamp diagnostic of the tile GEMM (standalone, no torch): where does a decode-shape
// GEMM spend its time?  Builds gemm_tile.hip with GEMM_STAMPS (per-workgroup begin/end
// shader-cycle + wall stamps, HW ids) and optionally GEMM_STAMPS_KT_REMOVED (per-k-tile stamps of
// wave 0), runs the 70B decode shapes at M = 512 on random operands with the weights rotated past
// the Infinity Cache, and prints per case: wall us (events), per-workgroup duration (us, cycles),
// clock, round structure (workgroups starting in the first vs later rounds and their durations),
// and the steady-state cycles per k-tile.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_llm_inference/csrc/kernels \
//         scripts/experiments/gemm_stamps.hip -o tools_bin/gemm_stamps && tools_bin/gemm_stamps
// (the per-k-tile stamps of the profiles/gemm_clock_stamps.txt second half came from a wave-0
// stamp at the top of every k-tile, since removed from the kernel: it perturbed the loop)
#define GEMM_STAMPS 1
#include "gemm_tile.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void fill_fp8(unsigned char* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (unsigned char)((x & 0xb7) | 0x30);   // |v| in [2^-2, 2^1): never NaN / inf
  }
}

__global__ void fill_ones(float* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 1.f;
}

__global__ void fill_rand(__bf16* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (__bf16)(((float)(x & 0xffffff) / 16777216.f * 2.f - 1.f) * scale);
  }
}

struct Case { const char* name; int M, N, K, splits, epi, prec = 0; };

static double med(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  std::vector<Case> cases = {
      {"gate_up_swiglu", 512, 57344, 8192, 1, 2},
      {"gate_up_256tiles", 512, 32768, 8192, 1, 2},
      {"gate_up_M256", 256, 57344, 8192, 1, 2},
      {"down_s4", 512, 8192, 28672, 4, 1},
      {"qkv_s3", 512, 10240, 8192, 3, 1},
      {"o_s4", 512, 8192, 8192, 4, 1},
      {"fp8_gate_up_swiglu", 512, 57344, 8192, 1, 2, 1},
      {"fp8_o_s4", 512, 8192, 8192, 4, 1, 1},
  };
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  for (const Case& c : cases) {
    const int esz = c.prec ? 1 : 2;
    const size_t wbytes = (size_t)c.N * c.K * esz;
    const int sets = (int)std::max<size_t>(1, std::min<size_t>(6, 1200000000ull / wbytes + 1));
    __bf16 *A, *C;
    std::vector<__bf16*> B(sets);
    float* ws = nullptr;
    CK(hipMalloc(&A, (size_t)c.M * c.K * esz));
    for (auto& b : B) CK(hipMalloc(&b, wbytes));
    CK(hipMalloc(&C, (size_t)c.M * c.N * 2));
    if (c.splits > 1) CK(hipMalloc(&ws, (size_t)c.splits * c.M * c.N * 4));
    float *sa = nullptr, *sbs = nullptr;
    CK(hipMalloc(&sa, (size_t)c.M * 4));
    CK(hipMalloc(&sbs, (size_t)c.N * 4));
    fill_ones<<<64, 256>>>(sa, c.M);
    fill_ones<<<256, 256>>>(sbs, c.N);
    if (c.prec) {
      fill_fp8<<<1024, 256>>>((unsigned char*)A, (size_t)c.M * c.K, 1);
      for (int i = 0; i < sets; ++i) fill_fp8<<<4096, 256>>>((unsigned char*)B[i], (size_t)c.N * c.K, 7 + i);
    } else {
      fill_rand<<<1024, 256>>>(A, (size_t)c.M * c.K, 1, 1.f);
      for (int i = 0; i < sets; ++i) fill_rand<<<4096, 256>>>(B[i], (size_t)c.N * c.K, 7 + i, 0.02f);
    }
    const int tiles = ((c.M + 255) / 256) * (c.N / 256) * c.splits;
    unsigned long long *sb, *sk;
    CK(hipMalloc(&sb, (size_t)tiles * 8 * 8));
    CK(hipMalloc(&sk, (size_t)tiles * 256 * 8));
    CK(hipMemset(sk, 0, (size_t)tiles * 256 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(dli::g_stamp_blk), &sb, sizeof(sb)));
    auto run = [&](int i) {
      int rc = dli::launch_gemm_tile(C, A, B[i % sets], sa, sbs, ws, c.M, c.N, c.K,
                                     c.splits, c.epi, c.prec, 0);
      if (rc) { fprintf(stderr, "launch rc %d\n", rc); exit(1); }
    };
    for (int i = 0; i < 10; ++i) run(i);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) run(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double wall_us = ms * 1e3 / iters;
    // one more (stamped) launch, alone
    run(iters);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> hb((size_t)tiles * 8), hk((size_t)tiles * 256);
    CK(hipMemcpy(hb.data(), sb, hb.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hk.data(), sk, hk.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int b = 0; b < tiles; ++b) {
      t0 = std::min(t0, hb[b * 8 + 0]);
      t1 = std::max(t1, hb[b * 8 + 2]);
    }
    std::vector<double> dur_us, dur_cyc, clk, r1, r2, kt, loopc;
    double start_late = 0;
    for (int b = 0; b < tiles; ++b) {
      const double us = (hb[b * 8 + 2] - hb[b * 8 + 0]) / 100.0;
      const double cyc = (double)(hb[b * 8 + 3] - hb[b * 8 + 1]);
      dur_us.push_back(us);
      dur_cyc.push_back(cyc);
      loopc.push_back((double)(hb[b * 8 + 7] - hb[b * 8 + 1]));
      if (us > 1) clk.push_back(cyc / us / 1e3);
    }
    const double md = med(dur_us);
    for (int b = 0; b < tiles; ++b) {
      const double st = (hb[b * 8 + 0] - t0) / 100.0;
      (st > 0.5 * md ? r2 : r1).push_back(dur_us[b]);
      start_late = std::max(start_late, st);
      const int T = std::min(255, (c.K * esz / 128) / c.splits);
      for (int t = T / 4; t + 1 < T * 3 / 4; ++t)
        if (hk[(size_t)b * 256 + t] && hk[(size_t)b * 256 + t + 1] > hk[(size_t)b * 256 + t])
          kt.push_back((double)(hk[(size_t)b * 256 + t + 1] - hk[(size_t)b * 256 + t]));
    }
    const double flop = 2.0 * c.M * c.N * c.K;
    printf("%-18s M=%d N=%d K=%d s=%d wgs=%d | wall %.1f us (%.0f TF) | stamped span %.1f us | "
           "wg dur med %.1f min %.1f max %.1f us, med %.0f cyc, clock %.2f GHz | round1 %zu wgs "
           "med %.1f us, later %zu wgs med %.1f us, last start %.1f us | k-tile med %.0f cyc "
           "(min %.0f) | main loop %.0f cyc = %.0f per k-tile\n",
           c.name, c.M, c.N, c.K, c.splits, tiles, wall_us, flop / wall_us / 1e6, (t1 - t0) / 100.0,
           md, *std::min_element(dur_us.begin(), dur_us.end()),
           *std::max_element(dur_us.begin(), dur_us.end()), med(dur_cyc), med(clk), r1.size(),
           med(r1), r2.size(), med(r2), start_late, med(kt),
           kt.empty() ? 0.0 : *std::min_element(kt.begin(), kt.end()), med(loopc),
           med(loopc) / ((c.K * esz / 128 + c.splits - 1) / c.splits));
    fflush(stdout);
    CK(hipFree(A));
    for (auto& b : B) CK(hipFree(b));
    CK(hipFree(C));
    if (ws) CK(hipFree(ws));
    CK(hipFree(sb));
    CK(hipFree(sk));
    CK(hipFree(sa));
    CK(hipFree(sbs));
  }
  return 0;
}
