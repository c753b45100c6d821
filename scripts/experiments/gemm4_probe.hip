// Where gemm4's k-loop cycles go: a GEMM_PROBE build of csrc/kernels/gemm4.hip records, per
// wave, the shader cycles stalled at each wait of the k-loop (B1 = lgkmcnt(0) + barrier, B2 =
// vmcnt + barrier, the end-of-tile LDS wait) and the whole k-loop, for the Llama-3-70B decode
// projections at M = 512 in bf16 and fp8 (production epilogues).  Per k-tile medians over waves;
// "rest" = loop - waits = MFMA issue plus everything not waiting.  The ideal k-tile is 2048
// cycles (128 bf16 16x16x32 or 64 fp8 16x16x128 MFMAs at 16 / 32 cycles).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_llm_inference/csrc/kernels \
//         scripts/experiments/gemm4_probe.hip -o tools_bin/gemm4_probe
//   tools_bin/gemm4_probe
#define GEMM_PROBE 1
#define GEMM4_FP8_VARIANTS 1
#include "../../distributed_llm_inference/csrc/kernels/gemm_tile.hip"
#include "../../distributed_llm_inference/csrc/kernels/gemm4.hip"

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

__global__ void fill_bytes(unsigned char* p, size_t n, unsigned seed, unsigned mask) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (unsigned char)(x & mask);   // bf16 pairs / e4m3 bytes with bounded exponents
  }
}

struct Case { const char* name; int M, N, K, splits, epi, prec, var; };

int main() {
  std::vector<Case> cases;
  for (int v : {6, 4, 9, 8}) {   // bf16 decode schedules (8 / 9: 4 / 6 with NT weights)
    cases.push_back({"bf16 gate_up swiglu", 512, 57344, 8192, 1, 2, 0, v});
    cases.push_back({"bf16 down s4 bf16p", 512, 8192, 28672, 4, 4, 0, v});
    cases.push_back({"bf16 qkv s3 bf16p", 512, 10240, 8192, 3, 4, 0, v});
    cases.push_back({"bf16 o s4 bf16p", 512, 8192, 8192, 4, 4, 0, v});
  }
  if (getenv("PROBE_BF16_ONLY") == nullptr) for (Case c : std::vector<Case>{
      {"fp8 gate_up swiglu-mx", 512, 57344, 8192, 1, 3, 1, 0},
      {"fp8 gate_up swiglu-mx", 512, 57344, 8192, 1, 3, 1, 1},
      {"fp8 gate_up swiglu-mx", 512, 57344, 8192, 1, 3, 1, 2},
      {"fp8 down mx s4 bf16p", 512, 8192, 28672, 4, 4, 2, 0},
      {"fp8 down mx s4 bf16p", 512, 8192, 28672, 4, 4, 2, 2},
      {"fp8 qkv s3 bf16p", 512, 10240, 8192, 3, 4, 1, 0},
  }) cases.push_back(c);
  unsigned long long* probe;
  const size_t pslots = (size_t)4096 * 4 * 8;
  CK(hipMalloc(&probe, pslots * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(dli::g_probe), &probe, sizeof(probe)));
  for (const Case& c : cases) {
    const int esz = c.prec ? 1 : 2;
    const size_t wbytes = (size_t)c.N * c.K * esz;
    const int sets = (int)std::max<size_t>(2, std::min<size_t>(6, 1200000000ull / wbytes + 1));
    std::vector<unsigned char*> B(sets);
    for (auto& b : B) {
      CK(hipMalloc(&b, wbytes));
      fill_bytes<<<4096, 256>>>(b, wbytes, 7, c.prec ? 0xF7u : 0xBDu);
    }
    unsigned char *A, *amx, *omx;
    float *sa, *sb;
    void* C;
    const int nb = (c.M + 63) / 64;
    CK(hipMalloc(&A, (size_t)c.M * c.K * esz));
    fill_bytes<<<1024, 256>>>(A, (size_t)c.M * c.K * esz, 3, c.prec ? 0xF7u : 0xBFu);
    CK(hipMalloc(&amx, (size_t)(c.K / 128) * nb * 64));
    CK(hipMemset(amx, 127, (size_t)(c.K / 128) * nb * 64));
    CK(hipMalloc(&omx, (size_t)(c.N / 256) * nb * 64 + 64));
    CK(hipMalloc(&sa, (size_t)c.M * 4));
    CK(hipMalloc(&sb, (size_t)c.N * 4));
    {
      std::vector<float> one((size_t)std::max(c.M, c.N), 1.f / 1024);
      CK(hipMemcpy(sa, one.data(), (size_t)c.M * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(sb, one.data(), (size_t)c.N * 4, hipMemcpyHostToDevice));
    }
    const size_t cbytes = (size_t)c.splits * c.M * c.N * 4;
    CK(hipMalloc(&C, cbytes));
    const bool mx = c.prec == 2;
    auto run = [&](int i) {
      int rc = dli::launch_gemm4(C, A, B[i % sets], c.M, c.N, c.K, c.splits, c.epi, 0, 0, c.var,
                                 c.prec, c.prec == 1 ? sa : nullptr, c.prec ? sb : nullptr,
                                 mx ? amx : nullptr, c.epi == 3 ? omx : nullptr);
      if (rc) { fprintf(stderr, "%s v%d: rc %d\n", c.name, c.var, rc); exit(1); }
    };
    for (int i = 0; i < 8; ++i) run(i);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> us;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) run(i);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      us.push_back(ms * 100.0);
    }
    std::sort(us.begin(), us.end());
    CK(hipMemset(probe, 0, pslots * 8));
    run(1);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(pslots);
    CK(hipMemcpy(h.data(), probe, pslots * 8, hipMemcpyDeviceToHost));
    std::vector<double> b1, b2, ew, loop, rest;
    for (size_t wv = 0; wv < pslots / 8; ++wv) {
      const unsigned long long* q = &h[wv * 8];
      if (q[4] == 0) continue;
      const double kt = (double)q[4];
      b1.push_back(q[0] / kt);
      b2.push_back(q[1] / kt);
      ew.push_back(q[2] / kt);
      loop.push_back(q[3] / kt);
      rest.push_back((q[3] - q[0] - q[1] - q[2]) / kt);
    }
    auto med = [](std::vector<double>& v) {
      std::sort(v.begin(), v.end());
      return v.empty() ? 0.0 : v[v.size() / 2];
    };
    auto p90 = [](std::vector<double>& v) { return v.empty() ? 0.0 : v[v.size() * 9 / 10]; };
    const double fl = 2.0 * c.M * c.N * c.K;
    const double t = us[us.size() / 2];
    printf("%-22s v%d  %7.1f us %5.0f TF | cycles per k-tile (median / p90 over %zu waves): "
           "loop %5.0f / %5.0f  B1 %4.0f / %4.0f  B2 %4.0f / %4.0f  end %4.0f / %4.0f  rest %5.0f\n",
           c.name, c.var, t, fl / t / 1e6, loop.size(), med(loop), p90(loop), med(b1), p90(b1),
           med(b2), p90(b2), med(ew), p90(ew), med(rest));
    fflush(stdout);
    for (auto b : B) CK(hipFree(b));
    CK(hipFree(A)); CK(hipFree(amx)); CK(hipFree(omx)); CK(hipFree(sa)); CK(hipFree(sb));
    CK(hipFree(C));
  }
  return 0;
}
