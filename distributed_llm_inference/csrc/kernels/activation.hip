// Element-wise activation kernels.
//
//  * silu_mul: SwiGLU gate of LlamaMLP (reference modules.py:123, 181 -> HF LlamaMLP
//    `down(silu(gate(x)) * up(x))`).  The gate and up projections are one fused GEMM whose output
//    row is [gate(I) | up(I)]; this kernel reads both halves once and writes silu(g)*u.
//  * gelu_tanh (+bias): GPT-2 MLP activation ("gelu_new").
//  * add: residual merge at a pipeline-stage boundary.
// All memory-bound: bf16x8 (16-byte) accesses, grid-stride loops capped at 8 WG/CU.
#include "kernels.h"

namespace dli {

// INTERLEAVED: the row is in the tile-GEMM SwiGLU order (ops.swiglu_interleave): output column o
// = 128 t + 32 w + 16 p + l has its gate at 256 t + 64 w + 32 p + l and its up 16 columns later.
template <bool INTERLEAVED>
__global__ void __launch_bounds__(256) silu_mul_kernel(bf16* __restrict__ out,
                                                       const bf16* __restrict__ x, int rows,
                                                       int inter) {
  const int nvec = inter >> 3;
  const size_t total = (size_t)rows * nvec;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / nvec, c = i % nvec;
    const bf16* row = x + r * 2 * inter;
    bf16x8 g, u;
    if (INTERLEAVED) {
      const int o = (int)c * 8;
      const int gc = (o >> 7) * 256 + ((o & 127) >> 5) * 64 + ((o & 31) >> 4) * 32 + (o & 15);
      g = *reinterpret_cast<const bf16x8*>(row + gc);
      u = *reinterpret_cast<const bf16x8*>(row + gc + 16);
    } else {
      g = reinterpret_cast<const bf16x8*>(row)[c];
      u = reinterpret_cast<const bf16x8*>(row + inter)[c];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)(silu((float)g[j]) * (float)u[j]);
    reinterpret_cast<bf16x8*>(out + r * inter)[c] = o;
  }
}

__global__ void __launch_bounds__(256) gelu_bias_kernel(bf16* __restrict__ out,
                                                        const bf16* __restrict__ x,
                                                        const bf16* __restrict__ bias, int rows,
                                                        int cols) {
  const int nvec = cols >> 3;
  const size_t total = (size_t)rows * nvec;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t c = i % nvec;
    const bf16x8 a = reinterpret_cast<const bf16x8*>(x)[i];
    bf16x8 o;
    if (bias) {
      const bf16x8 b = reinterpret_cast<const bf16x8*>(bias)[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_tanh((float)a[j] + (float)b[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_tanh((float)a[j]);
    }
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

__global__ void __launch_bounds__(256) add_kernel(bf16* __restrict__ out, const bf16* __restrict__ a,
                                                  const bf16* __restrict__ b, size_t nvec) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec;
       i += (size_t)gridDim.x * blockDim.x) {
    const bf16x8 x = reinterpret_cast<const bf16x8*>(a)[i];
    const bf16x8 y = reinterpret_cast<const bf16x8*>(b)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)x[j] + (float)y[j]);
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

static inline int ew_grid(size_t work) {
  size_t g = (work + 255) / 256;
  if (g > 2048) g = 2048;  // 8 WG per CU, grid-stride the rest
  if (g < 1) g = 1;
  return (int)g;
}

int launch_silu_mul(bf16* out, const bf16* x, int rows, int inter, bool interleaved,
                    hipStream_t stream) {
  if (inter % 8 != 0 || (interleaved && inter % 128 != 0)) return -1;
  if (rows == 0) return 0;
  if (interleaved)
    silu_mul_kernel<true><<<ew_grid((size_t)rows * inter / 8), 256, 0, stream>>>(out, x, rows, inter);
  else
    silu_mul_kernel<false><<<ew_grid((size_t)rows * inter / 8), 256, 0, stream>>>(out, x, rows, inter);
  return 0;
}

int launch_gelu_bias(bf16* out, const bf16* x, const bf16* bias, int rows, int cols,
                     hipStream_t stream) {
  if (cols % 8 != 0) return -1;
  if (rows == 0) return 0;
  gelu_bias_kernel<<<ew_grid((size_t)rows * cols / 8), 256, 0, stream>>>(out, x, bias, rows, cols);
  return 0;
}

int launch_add(bf16* out, const bf16* a, const bf16* b, size_t n, hipStream_t stream) {
  if (n % 8 != 0) return -1;
  if (n == 0) return 0;
  add_kernel<<<ew_grid(n / 8), 256, 0, stream>>>(out, a, b, n / 8);
  return 0;
}

}  // namespace dli
