// fp8 (OCP e4m3fn — gfx950's native format, NOT MI300's fnuz) row-wise quantisation.
//
// The reference quantises with bitsandbytes LLM.int8 (utils/model.py:93-123).  On
// CDNA4 the natural 8-bit format is fp8 e4m3 with per-output-channel weight scales (done once at
// load time) and per-token dynamic activation scales (this kernel, every GEMM input), feeding the
// fp8 MFMA GEMM (hipBLASLt row-wise scaled GEMM).  Optionally fused with RMSNorm so the normalised
// activation is produced directly in fp8 — one HBM pass instead of three.
#include "kernels.h"

namespace dli {

constexpr float kFp8Max = 448.f;

__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  int r = 0;
  r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, r, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (unsigned)r;
}

// x [rows, K] bf16 -> q [rows, K] fp8, scale [rows] f32 (x ~= q * scale).
// If `norm_w` is given the row is first RMS-normalised (with optional residual add, like
// rms_norm_kernel) and `norm_out` (optional) receives the bf16 normalised row.
template <int VPT>
__global__ void __launch_bounds__(256) quant_rowwise_kernel(
    uint8_t* __restrict__ q, float* __restrict__ scale, const bf16* __restrict__ x,
    bf16* __restrict__ residual, const bf16* __restrict__ norm_w, float eps, int K,
    int add_residual) {
  __shared__ float scratch[8];
  const int row = blockIdx.x;
  const int nvec = K >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * K);
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + (size_t)row * K);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      bf16x8 a = xr[idx];
      if (add_residual) {
        bf16x8 r = rr[idx];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (bf16)((float)a[j] + (float)r[j]);
        rr[idx] = a;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = (float)a[j];
        ss += v[i][j] * v[i][j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  if (norm_w) {
    ss = block_reduce_sum(ss, scratch);
    const float rstd = rsqrtf(ss / (float)K + eps);
    const bf16x8* wr = reinterpret_cast<const bf16x8*>(norm_w);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int idx = threadIdx.x + i * blockDim.x;
      if (idx < nvec) {
        bf16x8 ww = wr[idx];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (float)(bf16)(v[i][j] * rstd * (float)ww[j]);
      }
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
  amax = block_reduce_max(amax, scratch);
  const float s = amax > 0.f ? amax / kFp8Max : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[row] = s;
  uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * K);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = fminf(fmaxf(v[i][j] * inv, -kFp8Max), kFp8Max);
      uint2 o;
      o.x = pack4_fp8(t[0], t[1], t[2], t[3]);
      o.y = pack4_fp8(t[4], t[5], t[6], t[7]);
      qr[idx] = o;
    }
  }
}

int launch_quant_rowwise(uint8_t* q, float* scale, const bf16* x, bf16* residual,
                         const bf16* norm_w, float eps, int rows, int K, bool add_residual,
                         hipStream_t stream) {
  if (K % 8 != 0) return -1;
  if (rows == 0) return 0;
  const int nvec = K / 8;
  int threads = ((nvec + 63) / 64) * 64;
  if (threads > 256) threads = 256;
  const int vpt = (nvec + threads - 1) / threads;
  const int ar = add_residual ? 1 : 0;
  if (vpt <= 1) quant_rowwise_kernel<1><<<rows, threads, 0, stream>>>(q, scale, x, residual, norm_w, eps, K, ar);
  else if (vpt <= 2) quant_rowwise_kernel<2><<<rows, threads, 0, stream>>>(q, scale, x, residual, norm_w, eps, K, ar);
  else if (vpt <= 4) quant_rowwise_kernel<4><<<rows, threads, 0, stream>>>(q, scale, x, residual, norm_w, eps, K, ar);
  else if (vpt <= 8) quant_rowwise_kernel<8><<<rows, threads, 0, stream>>>(q, scale, x, residual, norm_w, eps, K, ar);
  else if (vpt <= 16) quant_rowwise_kernel<16><<<rows, threads, 0, stream>>>(q, scale, x, residual, norm_w, eps, K, ar);
  else return -1;
  return 0;
}

}  // namespace dli
