// fp8 gemm4 (csrc/kernels/gemm4.hip, 16x16x128 block-scaled MFMA, G4S8 schedules) against
// gemm_tile.hip's fp8 path on the Llama-3-70B decode projections at M = 512, with the epilogues
// the model runs: gate|up + SwiGLU quantised to MX (epilogue 3), down / O on MX activations and
// QKV on per-row scaled activations, both into bf16 split-K partials (epilogue 4).
//
// check: every G4S8 variant must give gemm_tile's bytes (outputs and MX scales) for M = 512, 300,
// 40.  timing: interleaved rounds, weights rotated past the Infinity Cache, median per launch.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_llm_inference/csrc/kernels \
//         scripts/experiments/gemm4_fp8_bench.hip -o tools_bin/gemm4_fp8_bench
//   tools_bin/gemm4_fp8_bench [rounds]
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

__global__ void fill_fp8(unsigned char* p, size_t n, unsigned seed) {   // finite e4m3, |x| < 256
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (unsigned char)(x & 0xF7u);   // exponent field <= 14
  }
}

__global__ void fill_e8m0(unsigned char* p, size_t n, unsigned seed) {   // 2^-6 .. 2^6
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 0x2c1b3c6du; x ^= x >> 12;
    p[i] = (unsigned char)(121 + x % 13);
  }
}

__global__ void fill_scale(float* p, int n, unsigned seed) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (1.f + (x & 1023) / 1024.f) / 4096.f;
  }
}

struct Shape { const char* name; int M, N, K, splits, epi, prec; };   // prec 1: row scales, 2: MX

constexpr int kVars = 3;

struct Bufs {
  unsigned char *A, *amx, *omx;
  float *sa, *sb;
  void* C;
  size_t cbytes, omx_bytes;
};

static Bufs alloc(const Shape& c, int M) {
  Bufs b{};
  const int nb = (M + 63) / 64, kt = c.K / 128;
  CK(hipMalloc(&b.A, (size_t)M * c.K));
  CK(hipMalloc(&b.amx, (size_t)kt * nb * 64));
  CK(hipMalloc(&b.sa, (size_t)M * 4));
  CK(hipMalloc(&b.sb, (size_t)c.N * 4));
  b.cbytes = c.epi == 3 ? (size_t)M * c.N / 2 : (size_t)c.splits * M * c.N * 2;
  b.omx_bytes = c.epi == 3 ? (size_t)(c.N / 2 / 128) * nb * 64 : 1;
  CK(hipMalloc(&b.C, b.cbytes));
  CK(hipMalloc(&b.omx, b.omx_bytes));
  fill_fp8<<<1024, 256>>>(b.A, (size_t)M * c.K, 1 + M);
  fill_e8m0<<<64, 256>>>(b.amx, (size_t)kt * nb * 64, 5 + M);
  fill_scale<<<64, 256>>>(b.sa, M, 9);
  fill_scale<<<64, 256>>>(b.sb, c.N, 13);
  return b;
}

static void release(Bufs& b) {
  CK(hipFree(b.A)); CK(hipFree(b.amx)); CK(hipFree(b.omx));
  CK(hipFree(b.sa)); CK(hipFree(b.sb)); CK(hipFree(b.C));
}

// v < 0: gemm_tile; else gemm4 G4S8<v>
static int run(const Shape& c, int M, Bufs& b, const unsigned char* B, int v) {
  const bool mx = c.prec == 2;
  if (v < 0)
    return dli::launch_gemm_tile(b.C, b.A, B, mx ? nullptr : b.sa, b.sb, nullptr, M, c.N, c.K,
                                 c.splits, c.epi, mx ? dli::kFp8Mx : dli::kFp8, 0, nullptr,
                                 nullptr, 0, mx ? b.amx : nullptr, c.epi == 3 ? b.omx : nullptr);
  return dli::launch_gemm4(b.C, b.A, B, M, c.N, c.K, c.splits, c.epi, 0, 0, v, mx ? 2 : 1,
                           mx ? nullptr : b.sa, b.sb, mx ? b.amx : nullptr,
                           c.epi == 3 ? b.omx : nullptr);
}

static int check(const Shape& c, unsigned char* B) {
  int bad = 0;
  for (int M : {c.M, 300, 40}) {
    Bufs b = alloc(c, M);
    std::vector<unsigned char> r0(b.cbytes), r1(b.cbytes), m0(b.omx_bytes), m1(b.omx_bytes);
    CK(hipMemset(b.C, 0x55, b.cbytes));
    CK(hipMemset(b.omx, 0x55, b.omx_bytes));
    if (int rc = run(c, M, b, B, -1)) { printf("gemm_tile rc %d\n", rc); return 1; }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r0.data(), b.C, b.cbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m0.data(), b.omx, b.omx_bytes, hipMemcpyDeviceToHost));
    for (int v = 0; v < kVars; ++v) {
      CK(hipMemset(b.C, 0x33, b.cbytes));
      CK(hipMemset(b.omx, 0x55, b.omx_bytes));
      if (int rc = run(c, M, b, B, v)) { printf("gemm4 v%d rc %d\n", v, rc); return 1; }
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(r1.data(), b.C, b.cbytes, hipMemcpyDeviceToHost));
      CK(hipMemcpy(m1.data(), b.omx, b.omx_bytes, hipMemcpyDeviceToHost));
      size_t d = 0, dm = 0;
      for (size_t i = 0; i < r0.size(); ++i) d += r0[i] != r1[i];
      for (size_t i = 0; i < m0.size(); ++i) dm += m0[i] != m1[i];
      printf("check v%d %-12s M=%d: %zu / %zu bytes differ, mx scales %zu / %zu\n", v, c.name, M,
             d, r0.size(), dm, m0.size());
      bad += d != 0 || dm != 0;
    }
    release(b);
  }
  return bad;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  std::vector<Shape> shapes = {
      {"gate_up_mx", 512, 57344, 8192, 1, 3, 1},
      {"down_mx_s4", 512, 8192, 28672, 4, 4, 2},
      {"qkv_s3", 512, 10240, 8192, 3, 4, 1},
      {"o_mx_s4", 512, 8192, 8192, 4, 4, 2},
  };
  int bad = 0;
  for (auto& c : shapes) {
    unsigned char* B;
    CK(hipMalloc(&B, (size_t)c.N * c.K));
    fill_fp8<<<4096, 256>>>(B, (size_t)c.N * c.K, 77);
    bad += check(c, B);
    CK(hipFree(B));
  }
  if (bad) { printf("CHECK FAILED\n"); return 2; }
  for (auto& c : shapes) {
    const size_t wbytes = (size_t)c.N * c.K;
    const int sets = (int)std::max<size_t>(2, std::min<size_t>(6, 1200000000ull / wbytes + 1));
    std::vector<unsigned char*> B(sets);
    for (int i = 0; i < sets; ++i) {
      CK(hipMalloc(&B[i], wbytes));
      fill_fp8<<<4096, 256>>>(B[i], wbytes, 7 + i);
    }
    Bufs b = alloc(c, c.M);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> t[1 + kVars];
    const int iters = 20;
    for (int v = -1; v < kVars; ++v)
      for (int i = 0; i < 5; ++i) run(c, c.M, b, B[i % sets], v);
    for (int r = 0; r < rounds; ++r)
      for (int vv = 0; vv <= kVars; ++vv) {
        const int v = ((r & 1) ? kVars - vv : vv) - 1;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) run(c, c.M, b, B[i % sets], v);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v + 1].push_back(ms * 1e3 / iters);
      }
    for (auto& x : t) std::sort(x.begin(), x.end());
    const double fl = 2.0 * c.M * c.N * c.K;
    const double t0 = t[0][t[0].size() / 2];
    printf("fp8 %-12s M=%d N=%d K=%d s=%d epi=%d | gemm_tile %.1f us (%.0f TF)", c.name, c.M, c.N,
           c.K, c.splits, c.epi, t0, fl / t0 / 1e6);
    for (int v = 0; v < kVars; ++v) {
      const double tv = t[v + 1][t[v + 1].size() / 2];
      printf(" | v%d %.1f us (%.0f TF, %.3f)", v, tv, fl / tv / 1e6, tv / t0);
    }
    printf("\n");
    fflush(stdout);
    release(b);
    for (auto p : B) CK(hipFree(p));
  }
  return 0;
}
