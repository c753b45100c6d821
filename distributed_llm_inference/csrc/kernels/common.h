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

// store; WT: device-scope write-through (sc1), so the value is visible to every XCD once the
// store completes (no L2 write-back before a grid barrier / arrival counter)
template <bool WT, typename T>
__device__ __forceinline__ void gst(T* p, T v) {
  if constexpr (!WT) {
    *p = v;
  } else if constexpr (sizeof(T) == 1) {
    asm volatile("global_store_byte %0, %1, off sc1" :: "v"(p), "v"((unsigned)__builtin_bit_cast(unsigned char, v)) : "memory");
  } else if constexpr (sizeof(T) == 2) {
    asm volatile("global_store_short %0, %1, off sc1" :: "v"(p), "v"((unsigned)__builtin_bit_cast(unsigned short, v)) : "memory");
  } else if constexpr (sizeof(T) == 4) {
    asm volatile("global_store_dword %0, %1, off sc1" :: "v"(p), "v"(__builtin_bit_cast(unsigned, v)) : "memory");
  } else if constexpr (sizeof(T) == 8) {
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    asm volatile("global_store_dwordx2 %0, %1, off sc1" :: "v"(p), "v"(__builtin_bit_cast(u32x2_t, v)) : "memory");
  } else {
    static_assert(sizeof(T) == 16, "gst: 1, 2, 4, 8 or 16 bytes");
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(__builtin_bit_cast(u32x4_t, v)) : "memory");
  }
}

// Block-wide sum of one float per thread.  `scratch` must hold >= blockDim.x/64 floats.
// Split-K partials consumed in place of a reduce pass (gemm_tile.hip kStoreF32 slabs).  NS
// partials of N consecutive fp32 elements, all loads issued before the adds (NS is a compile-time
// count so they are independent and in flight together), summed in split order 0..NS-1 and
// rounded to bf16 once: bit-identical to tile_splitk_reduce_kernel.
template <int NS>
__device__ __forceinline__ void sum_parts8(const float* p, size_t stride, bf16x8& out) {
  f32x4 a[NS], b[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    a[k] = *reinterpret_cast<const f32x4*>(p + k * stride);
    b[k] = *reinterpret_cast<const f32x4*>(p + k * stride + 4);
  }
  f32x4 s0 = a[0], s1 = b[0];
#pragma unroll
  for (int k = 1; k < NS; ++k) {
    s0 += a[k];
    s1 += b[k];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[j] = (bf16)s0[j];
    out[j + 4] = (bf16)s1[j];
  }
}

template <int NS>
__device__ __forceinline__ void sum_parts4(const float* p, size_t stride, bf16x4& out) {
  f32x4 a[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) a[k] = *reinterpret_cast<const f32x4*>(p + k * stride);
  f32x4 s = a[0];
#pragma unroll
  for (int k = 1; k < NS; ++k) s += a[k];
#pragma unroll
  for (int j = 0; j < 4; ++j) out[j] = (bf16)s[j];
}

template <int NS>
__device__ __forceinline__ bf16 sum_parts1(const float* p, size_t stride) {
  float a[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) a[k] = p[k * stride];
  float s = a[0];
#pragma unroll
  for (int k = 1; k < NS; ++k) s += a[k];
  return (bf16)s;
}

// bf16 partials (the fp8 path's gemm_tile epilogue 4: half the partial bytes; the fp8 activations
// already carry far more error than rounding each partial to bf16 adds): summed in fp32
template <int NS>
__device__ __forceinline__ void sum_parts8(const bf16* p, size_t stride, bf16x8& out) {
  bf16x8 a[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) a[k] = *reinterpret_cast<const bf16x8*>(p + k * stride);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = (float)a[0][j];
#pragma unroll
    for (int k = 1; k < NS; ++k) s += (float)a[k][j];
    out[j] = (bf16)s;
  }
}

template <int NS>
__device__ __forceinline__ void sum_parts4(const bf16* p, size_t stride, bf16x4& out) {
  bf16x4 a[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) a[k] = *reinterpret_cast<const bf16x4*>(p + k * stride);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float s = (float)a[0][j];
#pragma unroll
    for (int k = 1; k < NS; ++k) s += (float)a[k][j];
    out[j] = (bf16)s;
  }
}

template <int NS>
__device__ __forceinline__ bf16 sum_parts1(const bf16* p, size_t stride) {
  float s = (float)p[0];
#pragma unroll
  for (int k = 1; k < NS; ++k) s += (float)p[k * stride];
  return (bf16)s;
}

// One row of a row-per-workgroup kernel (RMSNorm, the fp8 row quantiser): VPT 16-byte vectors per
// lane at vector index lane + i * blockDim.x, the row's global loads issued before any is used -
// one memory round trip per row (per ~64 VGPRs of split-K partials).  (Loads guarded per vector by `idx < nvec` made hipcc wait
// for each vector's loads before issuing the next vector's: VPT serial round trips per row, plus
// one more for the residual.)  Lanes past the row's end load its last vector and must discard
// what they get (`row_valid`).  NS > 0: the vector is the sum of NS split-K partials (PB: bf16
// partials), summed in split order and rounded once, exactly as sum_parts8.
__device__ __forceinline__ int row_vec_idx(int i, int nvec) {
  const int idx = (int)threadIdx.x + i * (int)blockDim.x;
  return idx < nvec ? idx : nvec - 1;
}
__device__ __forceinline__ bool row_valid(int i, int nvec) {
  return (int)threadIdx.x + i * (int)blockDim.x < nvec;
}

template <int VPT, int NS, bool PB>
__device__ __forceinline__ void load_row_vecs(bf16x8 (&a)[VPT], const bf16* x, const void* parts,
                                              size_t row_off, size_t stride, int nvec) {
  if constexpr (NS == 0) {
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row_off);
#pragma unroll
    for (int i = 0; i < VPT; ++i) a[i] = xr[row_vec_idx(i, nvec)];
  } else {
    // partial vectors in flight per lane: ~64 VGPRs of them (a bf16 vector is 4, an fp32 one 8),
    // so at most CH vectors' partials per round trip
    constexpr int CH0 = PB ? 16 / NS : 8 / NS;
    constexpr int CH = CH0 < 1 ? 1 : (CH0 > VPT ? VPT : CH0);
#pragma unroll
    for (int c = 0; c < VPT; c += CH) {
      if constexpr (PB) {
        const bf16* pp = static_cast<const bf16*>(parts) + row_off;
        bf16x8 r[CH][NS];
#pragma unroll
        for (int i = 0; i < CH; ++i)
#pragma unroll
          for (int k = 0; k < NS; ++k)
            if (c + i < VPT)
              r[i][k] = *reinterpret_cast<const bf16x8*>(
                  pp + k * stride + (size_t)row_vec_idx(c + i, nvec) * 8);
#pragma unroll
        for (int i = 0; i < CH; ++i)
          if (c + i < VPT)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float sm = (float)r[i][0][j];
#pragma unroll
              for (int k = 1; k < NS; ++k) sm += (float)r[i][k][j];
              a[c + i][j] = (bf16)sm;
            }
      } else {
        const float* pp = static_cast<const float*>(parts) + row_off;
        f32x4 r0[CH][NS], r1[CH][NS];
#pragma unroll
        for (int i = 0; i < CH; ++i)
#pragma unroll
          for (int k = 0; k < NS; ++k)
            if (c + i < VPT) {
              const float* q = pp + k * stride + (size_t)row_vec_idx(c + i, nvec) * 8;
              r0[i][k] = *reinterpret_cast<const f32x4*>(q);
              r1[i][k] = *reinterpret_cast<const f32x4*>(q + 4);
            }
#pragma unroll
        for (int i = 0; i < CH; ++i)
          if (c + i < VPT) {
            f32x4 s0 = r0[i][0], s1 = r1[i][0];
#pragma unroll
            for (int k = 1; k < NS; ++k) {
              s0 += r0[i][k];
              s1 += r1[i][k];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              a[c + i][j] = (bf16)s0[j];
              a[c + i][j + 4] = (bf16)s1[j];
            }
          }
      }
    }
  }
}

// dispatch a runtime split count 1..8 to a compile-time NS (0 = no partials)
#define SPLITS_SWITCH(splits, MACRO) \
  switch (splits) {                      \
    case 0: MACRO(0); break;             \
    case 1: MACRO(1); break;             \
    case 2: MACRO(2); break;             \
    case 3: MACRO(3); break;             \
    case 4: MACRO(4); break;             \
    case 5: MACRO(5); break;             \
    case 6: MACRO(6); break;             \
    case 7: MACRO(7); break;             \
    case 8: MACRO(8); break;             \
    default: return -2;                  \
  }

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

// ---- fp8 e4m3 (OCP "fn" encoding: gfx950's native fp8, identical to torch.float8_e4m3fn) ------
// 4 floats -> 4 packed fp8 bytes (saturating conversion in hardware).
__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  int r = 0;
  r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, r, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (unsigned)r;
}

// ---- MX (e8m0 block-scaled) fp8 activations: one power-of-two scale per (row, 128 columns) -----
// Byte of (row r, 128-column block kt) at ((kt * nb + r / 64) * 64 + (r % 16) * 4 + (r % 64) / 16),
// nb = ceil(M / 64): the 4 rows r0 + 16 i (i = 0..3) of one 64-row block that an MFMA lane
// scales are one dword (gemm_tile.hip kFp8Mx reads them that way).  Rows in [M, 64 nb) hold 127.
__device__ __forceinline__ size_t mx_off(int kt, int r, int nb) {
  return ((size_t)kt * nb + (r >> 6)) * 64 + (r & 15) * 4 + ((r & 63) >> 4);
}

// the smallest k with amax / 2^k <= 448 (e4m3's largest finite value), clamped to e8m0's range;
// the stored byte is k + 127 and the quantised value e4m3(x * 2^-k)  (ops.mx_quantize's rule)
__device__ __forceinline__ int mx_exponent(float amax) {
  int k = 0;
  if (amax > 0.f) {
    const unsigned bits = __float_as_uint(amax / 448.f);
    k = (int)((bits >> 23) & 0xff) - 127 + ((bits & 0x7fffff) ? 1 : 0);
    k = min(max(k, -126), 126);
  }
  return k;
}
__device__ __forceinline__ float mx_inv_scale(int k) {   // 2^-k, exact
  return __uint_as_float((unsigned)(127 - k) << 23);
}

// 8 packed fp8 bytes -> 8 bf16 (exact: every e4m3 value is representable in bf16).  gfx950's
// v_cvt_scalef32_pk_bf16_fp8 widens two bytes straight to packed bf16 (scale 1.0): 4 VALU ops per
// 8 bytes instead of 4 fp8->f32 pairs + 4 f32->bf16 packs.
__device__ __forceinline__ bf16x8 fp8x8_to_bf16x8(uint2 v) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, 1.0f, false);
  const bf16x2_t b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, 1.0f, true);
  const bf16x2_t c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, 1.0f, false);
  const bf16x2_t d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, 1.0f, true);
  bf16x8 o;
  o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1];
  o[4] = c[0]; o[5] = c[1]; o[6] = d[0]; o[7] = d[1];
  return o;
}

__device__ __forceinline__ uint8_t f32_to_fp8(float x) {
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(x, 0.f, 0, false) & 0xff);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

}  // namespace dli

#define CHECK_HIP(expr)                                                         \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, \
              __LINE__);                                                            \
      abort();                                                                      \
    }                                                                               \
  } while (0)
