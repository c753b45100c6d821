// Weight-streaming GEMV building blocks shared by gemv.hip and the batch-1 decode-layer kernel
// (decode_layer.hip): row assignment and epilogues (plain / SwiGLU / RoPE + paged KV write).
#pragma once
#include "kernels.h"

namespace dli {
namespace {

constexpr int kRows = 2;
typedef unsigned u32x4n __attribute__((ext_vector_type(4)));   // nontemporal-loadable 16 B

// Epilogues.  kEpPlain: y[m, n] for rows n = 2w, 2w+1.  kEpSwiGLU (over a swiglu_interleave'd
// gate|up weight, N = 2I rows): the wave takes output column o = w, its gate row 32 (o / 16) +
// o % 16 and the up row 16 further, and stores silu(gate) * up.  kEpRope (the fused QKV weight
// [(nh + 2 nkv) D, K]): a wave of the q / k part takes rows (h D + d, h D + d + D/2) -- both
// rotation partners -- applies RoPE at the row's position and stores q packed [M, nh, D] or k
// into the paged K cache; a wave of the v part takes two consecutive rows and scatters them into
// the paged V^T cache: rope_cache.hip's arithmetic, element for element, minus its launch.
enum GemvEp { kEpPlain = 0, kEpSwiGLU = 1, kEpRope = 2 };

template <int EP>
__device__ __forceinline__ int gemv_row(int wave, int r, const GemvRope& rp) {
  if constexpr (EP == kEpSwiGLU) return 32 * (wave >> 4) + (wave & 15) + 16 * r;
  if constexpr (EP == kEpRope) {
    const int half = rp.D >> 1, nqk = rp.nh + rp.nkv;
    if (wave < nqk * half) {
      const int h = wave / half;
      return h * rp.D + (wave - h * half) + r * half;
    }
    return nqk * rp.D + 2 * (wave - nqk * half) + r;
  }
  return wave * kRows + r;
}

// outputs of a wave: kRows values per row m (final fp32, every lane holds them), lane 0 stores
template <int EP, int M, bool WT = false>
__device__ __forceinline__ void gemv_store(const float (&v)[M][kRows], int wave, int lane, int N,
                                           bf16* __restrict__ y, const GemvRope& rp) {
  if (lane != 0) return;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if constexpr (EP == kEpPlain) {
#pragma unroll
      for (int r = 0; r < kRows; ++r)
        if (wave * kRows + r < N) gst<WT>(y + (size_t)m * N + wave * kRows + r, (bf16)v[m][r]);
    } else if constexpr (EP == kEpSwiGLU) {   // gate and up rounded to bf16 first (unfused path)
      const float g = (float)(bf16)v[m][0], u = (float)(bf16)v[m][1];
      gst<WT>(y + (size_t)m * (N >> 1) + wave, (bf16)(g / (1.f + __expf(-g)) * u));
    } else {
      const int D = rp.D, half = D >> 1, nqk = rp.nh + rp.nkv;
      const bf16 b0 = (bf16)v[m][0], b1 = (bf16)v[m][1];   // the GEMM output, rounded
      const long slot = rp.slot_mapping ? rp.slot_mapping[m] : -1;
      const long blk = slot >= 0 ? slot / rp.bs : 0;
      const int off = slot >= 0 ? (int)(slot % rp.bs) : 0;
      if (wave < nqk * half) {
        const int h = wave / half, d = wave - h * half;
        bf16 o0 = b0, o1 = b1;
        if (rp.cos_sin) {
          int pc = rp.positions ? rp.positions[m] : 0;
          pc = pc < 0 ? 0 : (pc >= rp.max_pos ? rp.max_pos - 1 : pc);
          const float c = rp.cos_sin[(size_t)pc * D + d], sn = rp.cos_sin[(size_t)pc * D + half + d];
          const float x0 = (float)b0, x1 = (float)b1;
          o0 = (bf16)__builtin_fmaf(x0, c, -(x1 * sn));
          o1 = (bf16)__builtin_fmaf(x1, c, x0 * sn);
        }
        if (h < rp.nh) {
          bf16* q = rp.q_out + ((size_t)m * rp.nh + h) * D;
          gst<WT>(q + d, o0);
          gst<WT>(q + d + half, o1);
        } else if (slot >= 0) {
          const size_t base = (((size_t)blk * rp.nkv + (h - rp.nh)) * rp.bs + off) * D;
          if (rp.kv_fp8) {
            uint8_t* kc = static_cast<uint8_t*>(rp.k_cache) + base;
            gst<WT>(kc + d, (uint8_t)f32_to_fp8((float)o0 * rp.k_inv_scale));
            gst<WT>(kc + d + half, (uint8_t)f32_to_fp8((float)o1 * rp.k_inv_scale));
          } else {
            bf16* kc = static_cast<bf16*>(rp.k_cache) + base;
            gst<WT>(kc + d, o0);
            gst<WT>(kc + d + half, o1);
          }
        }
      } else if (slot >= 0) {
        const int e = 2 * (wave - nqk * half), kh = e / D, dd = e - kh * D;
        const size_t grp = ((size_t)blk * rp.nkv + kh) * (rp.bs >> 3) + (off >> 3);
        const size_t i0 = (grp * D + dd) * 8 + (off & 7);
        if (rp.kv_fp8) {
          uint8_t* vc = static_cast<uint8_t*>(rp.v_cache);
          gst<WT>(vc + i0, (uint8_t)f32_to_fp8((float)b0 * rp.v_inv_scale));
          gst<WT>(vc + i0 + 8, (uint8_t)f32_to_fp8((float)b1 * rp.v_inv_scale));
        } else {
          bf16* vc = static_cast<bf16*>(rp.v_cache);
          gst<WT>(vc + i0, b0);
          gst<WT>(vc + i0 + 8, b1);
        }
      }
    }
  }
}

__device__ __forceinline__ bf16x2 u8pair_to_bf16x2(unsigned u, int j) {
  const float lo = (float)((u >> (16 * j)) & 0xFFu);
  const float hi = (float)((u >> (16 * j + 8)) & 0xFFu);
  const unsigned p = __builtin_amdgcn_perm(__builtin_bit_cast(unsigned, hi),
                                           __builtin_bit_cast(unsigned, lo), 0x07060302u);
  return __builtin_bit_cast(bf16x2, p);
}


}  // namespace
}  // namespace dli
