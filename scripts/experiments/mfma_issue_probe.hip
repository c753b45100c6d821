// Does an MFMA leave issue slots for the other instructions of its SIMD?  One wave per SIMD (4 per
// workgroup, 256 workgroups), each wave loops over 8 independent MFMAs per iteration, with and
// without one ds_read_b128 placed after every MFMA (sched_barrier-pinned order); shader-cycle
// stamps around the loop give cycles per MFMA.  Compared: v_mfma_f32_16x16x32_bf16 (16 cycles),
// the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (fp8, 2x the bf16 FLOPs per cycle) and
// v_mfma_f32_32x32x16_bf16 (32 cycles).  If an MFMA blocks vector issue for its whole duration,
// the ds_reads add their own issue time per MFMA instead of hiding in its shadow.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/experiments/mfma_issue_probe.hip \
//         -o tools_bin/mfma_issue_probe && tools_bin/mfma_issue_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 2000;

template <int KIND, bool READS>
__global__ void __launch_bounds__(256) probe(float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<float*>(lds)[i] = 1e-3f * (i & 7);
  __syncthreads();
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * (lane + j)); b[j] = (__bf16)(0.02f * (j - lane)); }
  i32x8 fa = {}, fb = {};
  for (int j = 0; j < 8; ++j) { fa[j] = 0x38383838 + lane; fb[j] = 0x30303030 + j; }
  f32x4 acc[8];
  f32x16 acc32[8];
  for (int i = 0; i < 8; ++i) { acc[i] = f32x4{0, 0, 0, 0}; acc32[i] = f32x16{}; }
  bf16x8 r[8];
  const int base = (threadIdx.x * 16) & 65535;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
      if (KIND == 1)
        acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa, fb, acc[i], 0, 0, 0, 127, 0, 127);
      if (KIND == 2) acc32[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc32[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (READS) {
        r[i] = *reinterpret_cast<const bf16x8*>(lds + ((base + i * 1024 + it * 16) & 65535));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (READS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" :: "v"(r[i]));   // keep all 16 B of each read live
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc32[i][0] + (float)a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND, bool READS>
static double run(float* out, unsigned long long* cyc) {
  probe<KIND, READS><<<256, 256>>>(out, cyc);
  probe<KIND, READS><<<256, 256>>>(out, cyc);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(1024);
  hipMemcpy(h.data(), cyc, 8 * 1024, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  return (double)h[512] / (kIters * 8);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 8 * 1024);
  const char* names[3] = {"16x16x32 bf16", "16x16x128 f8 scaled", "32x32x16 bf16"};
  double c[3][2];
  c[0][0] = run<0, false>(out, cyc); c[0][1] = run<0, true>(out, cyc);
  c[1][0] = run<1, false>(out, cyc); c[1][1] = run<1, true>(out, cyc);
  c[2][0] = run<2, false>(out, cyc); c[2][1] = run<2, true>(out, cyc);
  for (int k = 0; k < 3; ++k)
    printf("%-22s cycles/MFMA alone %.1f, with one ds_read_b128 after each %.1f (+%.1f)\n", names[k],
           c[k][0], c[k][1], c[k][1] - c[k][0]);
  return 0;
}
