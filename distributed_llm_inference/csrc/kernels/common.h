// Shared helpers for the CDNA4 (gfx950 / MI355X) kernels of distributed_llm_inference.
//
// Conventions used by every kernel in this directory:
//   * wave64: lane = threadIdx.x & 63, wave = threadIdx.x >> 6.  Never 32-wide idioms.
//   * bf16 is the clang __bf16 type; (float)<->(__bf16) casts lower to v_cvt_pk_bf16_f32 on gfx950
//     (round-to-nearest-even, NaN preserving).
//   * every memory-bound kernel moves 16 bytes per lane per access (bf16x8), see
//     /opt/skills/guides/cdna_hip_programming.md Guideline 13.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dli {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

template <typename T>
__device__ __forceinline__ T wave_reduce_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum of one float per thread.  `scratch` must hold >= blockDim.x/64 floats.
__device__ __forceinline__ float block_reduce_sum(float v, float* scratch) {
  v = wave_reduce_sum(v);
  const int nw = blockDim.x >> 6;
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_reduce_max(float v, float* scratch) {
  v = wave_reduce_max(v);
  const int nw = blockDim.x >> 6;
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

}  // namespace dli

#define DLI_HIP_CHECK(expr)                                                         \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, \
              __LINE__);                                                            \
      abort();                                                                      \
    }                                                                               \
  } while (0)
