// Skinny GEMM for small decode batches:  y[M, N] = x[M, K] . W[N, K]^T (+ bias),  M <= 4.
//
// At M <= 4 a projection is a pure weight stream (70B bf16: 140 GB per decode step), and the
// tuned hipBLASLt solutions reach only ~4.7 TB/s of it (measured: Llama-3-70B batch 1 decode
// 29.8 ms/token against a 17.6 ms HBM floor).  cdna_hip_programming.md's rule for "GEMV / M <= 16
// decode weights: operand streamed once per block and not shared across waves": no LDS, load
// straight to VGPRs, deep unroll, late vmcnt.  So:
//   * one wave per ROWS = 2 consecutive weight rows; lanes stride K by 8 elements (16-B loads), a
//     wave instruction covers 1 KiB of a row;
//   * UNROLL = 4 k-steps of loads are issued before any FMA (8 x 16 B of weights in flight per
//     lane, ~16 waves per CU -> ~128 KiB per CU in flight, enough to cover HBM latency);
//   * weight loads are non-temporal (streamed exactly once: keep them out of the way of x, which
//     every wave re-reads and stays L1/L2-resident);
//   * v_dot2c_f32_bf16 (two bf16 products into an fp32 accumulator per instruction, no bf16->f32
//     conversions): plain conversions + FMAs made M = 4 VALU-bound; one wave reduction per
//     (m, row) at the end, lane 0 stores.
#include "kernels.h"

namespace dli {

namespace {

constexpr int kRows = 2;
constexpr int kUnroll = 4;

template <int M>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(const bf16* __restrict__ x,
                                                          const bf16* __restrict__ W,
                                                          const bf16* __restrict__ bias,
                                                          bf16* __restrict__ y, int N, int K) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int n0 = wave * kRows;
  if (n0 >= N) return;
  float acc[M][kRows];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kRows; ++r) acc[m][r] = 0.f;

  const bf16* wrow[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) wrow[r] = W + (size_t)min(n0 + r, N - 1) * K;

  constexpr int kStep = 64 * 8;  // elements per wave instruction
  for (int k0 = lane * 8; k0 < K; k0 += kStep * kUnroll) {
    bf16x8 wv[kUnroll][kRows];
    bf16x8 xv[kUnroll][M];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = k0 + u * kStep;
      if (k < K) {
#pragma unroll
        for (int r = 0; r < kRows; ++r)
          wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wrow[r] + k));
#pragma unroll
        for (int m = 0; m < M; ++m)
          xv[u][m] = *reinterpret_cast<const bf16x8*>(x + (size_t)m * K + k);
      } else {
#pragma unroll
        for (int r = 0; r < kRows; ++r) wv[u][r] = bf16x8{};
#pragma unroll
        for (int m = 0; m < M; ++m) xv[u][m] = bf16x8{};
      }
    }
    // v_dot2c_f32_bf16: two bf16 products accumulated in fp32 per instruction, no conversions
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const bf16x2 xp = {xv[u][m][2 * j], xv[u][m][2 * j + 1]};
#pragma unroll
          for (int r = 0; r < kRows; ++r) {
            const bf16x2 wp = {wv[u][r][2 * j], wv[u][r][2 * j + 1]};
            acc[m][r] = __builtin_amdgcn_fdot2_f32_bf16(xp, wp, acc[m][r], false);
          }
        }
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const float v = wave_reduce_sum(acc[m][r]);
      const int n = n0 + r;
      if (lane == 0 && n < N) y[(size_t)m * N + n] = (bf16)(v + (bias ? (float)bias[n] : 0.f));
    }
}

}  // namespace

int launch_skinny_gemm(bf16* y, const bf16* x, const bf16* W, const bf16* bias, int M, int N,
                       int K, hipStream_t stream) {
  if (M < 1 || M > 4 || K % 8 != 0 || N < 1) return -1;
  const int waves = (N + kRows - 1) / kRows;
  const int grid = (waves + 3) / 4;
  switch (M) {
    case 1: skinny_gemm_kernel<1><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K); break;
    case 2: skinny_gemm_kernel<2><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K); break;
    case 3: skinny_gemm_kernel<3><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K); break;
    case 4: skinny_gemm_kernel<4><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K); break;
  }
  return 0;
}

}  // namespace dli
