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

// One workgroup per row; threads chosen so each holds <= 4 bf16x8 vectors (<= 1024 threads): a
// 28672-wide row (70B down-projection input) gets 896 threads x 4 vectors instead of 256 x 14,
// ~4x the loads in flight per CU at a quarter of the registers.  Rows up to 8192 wide keep 256
// threads (the same block shape, so the same reduction order, as before).
static inline int row_threads(int nvec) {
  int t = (nvec + 3) / 4;
  t = (t + 63) / 64 * 64;
  if (t < 256) t = ((nvec + 63) / 64) * 64 < 256 ? ((nvec + 63) / 64) * 64 : 256;
  return t > 1024 ? 1024 : t;
}

// Row amax -> scale, then quantise the VPT x 8 register-resident values of each thread (vector
// index threadIdx.x + i * blockDim.x) and store them as 8-byte fp8 groups.
template <int VPT>
__device__ __forceinline__ void store_fp8_row(float (&v)[VPT][8], uint8_t* __restrict__ qrow,
                                              float* __restrict__ srow, int nvec, float* scratch) {
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
  amax = block_reduce_max(amax, scratch);
  const float s = amax > 0.f ? amax / kFp8Max : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) *srow = s;
  uint2* qr = reinterpret_cast<uint2*>(qrow);
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

// x [rows, K] bf16 -> q [rows, K] fp8, scale [rows] f32 (x ~= q * scale).
// If `residual_in` is given, x + residual_in is quantised and also written to `residual_out`
// (which may alias residual_in; like rms_norm_kernel).  If `norm_w` is given the row is
// RMS-normalised first, so "add residual -> RMSNorm -> fp8" is one HBM pass.
// x_parts (optional): x given as split-K partials [splits, rows, K] of the tile GEMM that
// produced it, summed and rounded to bf16 on load: fp32 (bit-identical to the reduce pass) or,
// with parts_bf16, bf16 partials (fp8 path)
template <int VPT, int NS, bool PB>
__global__ void __launch_bounds__(1024) quant_rowwise_kernel(
    uint8_t* __restrict__ q, float* __restrict__ scale, const bf16* __restrict__ x,
    const bf16* residual_in, bf16* residual_out, const bf16* __restrict__ norm_w, float eps,
    int K, const void* __restrict__ x_parts, size_t split_stride) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = K >> 3;
  const bool add_residual = residual_in != nullptr;
  const size_t row_off = (size_t)row * K;
  const bf16x8* ri = reinterpret_cast<const bf16x8*>(residual_in + row_off);
  bf16x8* ro = reinterpret_cast<bf16x8*>(residual_out + row_off);
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(norm_w);
  // the row's loads first (common.h load_row_vecs): norm weights, residual, x / partials
  bf16x8 wv[VPT], rv[VPT], a[VPT];
  if (norm_w) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) wv[i] = wr[row_vec_idx(i, nvec)];
  }
  if (add_residual) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) rv[i] = ri[row_vec_idx(i, nvec)];
  }
  load_row_vecs<VPT, NS, PB>(a, x, x_parts, row_off, split_stride, nvec);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const bool ok = row_valid(i, nvec);
    if (add_residual) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[i][j] = (bf16)((float)a[i][j] + (float)rv[i][j]);
      if (ok) ro[threadIdx.x + i * blockDim.x] = a[i];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[i][j] = ok ? (float)a[i][j] : 0.f;
      ss = __builtin_fmaf(v[i][j], v[i][j], ss);   // explicit: same rounding in every instantiation
    }
  }
  if (norm_w) {
    ss = block_reduce_sum(ss, scratch);
    const float rstd = rsqrtf(ss / (float)K + eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      if (row_valid(i, nvec)) {
        const bf16x8 ww = wv[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (float)(bf16)(v[i][j] * rstd * (float)ww[j]);
      }
    }
  }
  store_fp8_row<VPT>(v, q + (size_t)row * K, scale + row, nvec, scratch);
}

// out = silu(x[:, :I]) * x[:, I:] quantised per row: [rows, 2I] bf16 -> [rows, I] fp8 + scale.
// The activation is rounded to bf16 before quantisation, exactly as silu_mul_kernel would store
// it, so the fp8 path differs from the bf16 path only by the quantisation step.
template <int VPT>
__global__ void __launch_bounds__(1024) silu_mul_quant_kernel(uint8_t* __restrict__ q,
                                                             float* __restrict__ scale,
                                                             const bf16* __restrict__ x, int I) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = I >> 3;
  const bf16x8* g = reinterpret_cast<const bf16x8*>(x + (size_t)row * 2 * I);
  const bf16x8* u = reinterpret_cast<const bf16x8*>(x + (size_t)row * 2 * I + I);
  float v[VPT][8];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      const bf16x8 a = g[idx], b = u[idx];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = (float)(bf16)(silu((float)a[j]) * (float)b[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  store_fp8_row<VPT>(v, q + (size_t)row * I, scale + row, nvec, scratch);
}

// LLM.int8 activation quantisation (reference utils/model.py:93-113 -> bitsandbytes Linear8bitLt):
// x [rows, K] bf16 -> q [rows, K] int8, scale [rows] f32 with x ~= q * scale on the regular
// columns.  Columns flagged in `outlier` (nullable) are zeroed here: they are multiplied in bf16
// by the caller (the mixed-precision decomposition of LLM.int8).
template <int VPT>
__global__ void __launch_bounds__(1024) quant_rowwise_int8_kernel(
    int8_t* __restrict__ q, float* __restrict__ scale, const bf16* __restrict__ x,
    const uint8_t* __restrict__ outlier, int K) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = K >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * K);
  const uint2* fr = reinterpret_cast<const uint2*>(outlier);
  float v[VPT][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      const bf16x8 a = xr[idx];
      uint2 f = {0u, 0u};
      if (outlier) f = fr[idx];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned byte = ((j < 4 ? f.x : f.y) >> (8 * (j & 3))) & 0xffu;
        v[i][j] = byte ? 0.f : (float)a[j];
        amax = fmaxf(amax, fabsf(v[i][j]));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  amax = block_reduce_max(amax, scratch);
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[row] = s;
  uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * K);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      unsigned w[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qi = (int)rintf(fminf(fmaxf(v[i][j] * inv, -127.f), 127.f));
        w[j >> 2] |= ((unsigned)qi & 0xffu) << (8 * (j & 3));
      }
      qr[idx] = uint2{w[0], w[1]};
    }
  }
}

int launch_quant_rowwise_int8(int8_t* q, float* scale, const bf16* x, const uint8_t* outlier,
                              int rows, int K, hipStream_t stream) {
  if (K % 8 != 0) return -1;
  if (rows == 0) return 0;
  const int nvec = K / 8;
  const int threads = row_threads(nvec);
  const int vpt = (nvec + threads - 1) / threads;
#define QI8_LAUNCH(V) \
  quant_rowwise_int8_kernel<V><<<rows, threads, 0, stream>>>(q, scale, x, outlier, K)
  if (vpt <= 1) QI8_LAUNCH(1);
  else if (vpt <= 2) QI8_LAUNCH(2);
  else if (vpt <= 4) QI8_LAUNCH(4);
  else if (vpt <= 8) QI8_LAUNCH(8);
  else if (vpt <= 16) QI8_LAUNCH(16);
  else return -1;
#undef QI8_LAUNCH
  return 0;
}

int launch_quant_rowwise(uint8_t* q, float* scale, const bf16* x, const bf16* residual_in,
                         bf16* residual_out, const bf16* norm_w, float eps, int rows, int K,
                         hipStream_t stream, const void* x_parts, int splits, bool parts_bf16) {
  if (K % 8 != 0) return -1;
  if (x_parts != nullptr && splits < 1) return -3;
  const size_t split_stride = (size_t)rows * K;
  if (residual_in != nullptr && residual_out == nullptr) return -2;
  if (rows == 0) return 0;
  const int nvec = K / 8;
  const int threads = row_threads(nvec);
  const int vpt = (nvec + threads - 1) / threads;
#ifdef PROBE_NS1   // diagnostic (scripts/split_k_upper_bound.sh): read split 0 only
  const int ns = x_parts != nullptr ? 1 : 0;
#else
  const int ns = x_parts != nullptr ? splits : 0;
#endif
#define QUANT_LAUNCH(V, NS)                                                                     \
  do {                                                                                       \
    if (NS > 0 && parts_bf16)                                                                \
      quant_rowwise_kernel<V, NS, true><<<rows, threads, 0, stream>>>(                       \
          q, scale, x, residual_in, residual_out, norm_w, eps, K, x_parts, split_stride);    \
    else                                                                                     \
      quant_rowwise_kernel<V, NS, false><<<rows, threads, 0, stream>>>(                      \
          q, scale, x, residual_in, residual_out, norm_w, eps, K, x_parts, split_stride);    \
  } while (0)
#define QUANT_LAUNCH_NS(NS)                       \
  do {                                         \
    if (vpt <= 1) QUANT_LAUNCH(1, NS);            \
    else if (vpt <= 2) QUANT_LAUNCH(2, NS);       \
    else if (vpt <= 4) QUANT_LAUNCH(4, NS);       \
    else if (vpt <= 8) QUANT_LAUNCH(8, NS);       \
    else if (vpt <= 16) QUANT_LAUNCH(16, NS);     \
    else return -1;                            \
  } while (0)
  SPLITS_SWITCH(ns, QUANT_LAUNCH_NS)
#undef QUANT_LAUNCH_NS
#undef QUANT_LAUNCH
  return 0;
}

int launch_silu_mul_quant(uint8_t* q, float* scale, const bf16* x, int rows, int inter,
                          hipStream_t stream) {
  if (inter % 8 != 0) return -1;
  if (rows == 0) return 0;
  const int nvec = inter / 8;
  const int threads = row_threads(nvec);
  const int vpt = (nvec + threads - 1) / threads;
#define SMQ_LAUNCH(V) silu_mul_quant_kernel<V><<<rows, threads, 0, stream>>>(q, scale, x, inter)
  if (vpt <= 1) SMQ_LAUNCH(1);
  else if (vpt <= 2) SMQ_LAUNCH(2);
  else if (vpt <= 4) SMQ_LAUNCH(4);
  else if (vpt <= 8) SMQ_LAUNCH(8);
  else if (vpt <= 16) SMQ_LAUNCH(16);
  else return -1;
#undef SMQ_LAUNCH
  return 0;
}

}  // namespace dli
