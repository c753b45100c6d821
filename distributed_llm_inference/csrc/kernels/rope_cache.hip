// Fused RoPE + paged-KV-cache write.
//
// Replaces, per layer, the reference's rotary application (modules.py:17-20, 71-76; cos/sin from
// model.py:55 — computed there in int64) and the per-token `torch.cat` KV append
// (cache.py:103-109, an O(S) copy per token per layer).  Here one pass over the fused QKV GEMM
// output:
//   * rotates q (rotate-half convention, fp32 math, cos/sin from a host-built fp32 table that
//     already contains llama3 rope scaling) and writes it packed [T, nh, D];
//   * in attention-sink (StreamingLLM) mode also writes q rotated at the *in-window* position
//     min(pos, W-1) — the attention kernel scores sink keys with it, which is exactly the
//     reference's key re-rotation (cache.py:21-48, 111-124) expressed on the query side, so no
//     cached key is ever re-rotated;
//   * rotates k and scatters it into the paged K cache [blocks, nkv, bs, D];
//   * with an fp8 KV cache, k and v are stored as e4m3 (x * inv_scale), converted in registers;
//   * scatters v into the paged V^T cache [blocks, nkv, bs/8, D, 8] (8-key groups) — the MFMA
//     P·V product reads 8 consecutive keys of one d as a 16-byte-per-lane operand (attention.hip),
//     and one token's write stays inside 16 cache lines per head instead of D (one per d row).
// slot_mapping[t] = physical slot (block*bs + offset) or -1 to skip the cache write.
#include "kernels.h"

namespace dli {


__device__ __forceinline__ void rotate4(const bf16x4& a, const bf16x4& b, const float* cs,
                                        int i, int half, bf16x4& oa, bf16x4& ob) {
  // out[i] = a*cos - b*sin ; out[i+half] = b*cos + a*sin   (i .. i+3)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float c = cs[i + j], s = cs[half + i + j];
    const float x = (float)a[j], y = (float)b[j];
    // explicit fma: every instantiation (bf16 input, split-K partials) rounds identically,
    // whatever contraction -ffp-contract=fast would pick per instantiation
    oa[j] = (bf16)__builtin_fmaf(x, c, -(y * s));
    ob[j] = (bf16)__builtin_fmaf(y, c, x * s);
  }
}

// 4 consecutive qkv elements of token row t starting at column c: from the bf16 GEMM output, or
// (NS > 0) summed over the NS fp32 split-K partials and rounded once (bit-identical to the
// reduce pass)
template <int NS>
__device__ __forceinline__ bf16x4 load_qkv4(const RopeCacheParams& p, const bf16* row, int t,
                                            int c) {
  if constexpr (NS == 0) {
    return *reinterpret_cast<const bf16x4*>(row + c);
  } else {
    bf16x4 o;
    const size_t off = (size_t)t * p.qkv_stride + c;
    if (p.parts_bf16)
      sum_parts4<NS>(static_cast<const bf16*>(p.qkv_parts) + off, p.split_stride, o);
    else
      sum_parts4<NS>(static_cast<const float*>(p.qkv_parts) + off, p.split_stride, o);
    return o;
  }
}

template <int NS>
__device__ __forceinline__ bf16 load_qkv1(const RopeCacheParams& p, const bf16* row, int t,
                                          int c) {
  if constexpr (NS == 0)
    return row[c];
  else
    return p.parts_bf16
               ? sum_parts1<NS>(static_cast<const bf16*>(p.qkv_parts) + (size_t)t * p.qkv_stride + c,
                                p.split_stride)
               : sum_parts1<NS>(static_cast<const float*>(p.qkv_parts) + (size_t)t * p.qkv_stride + c,
                                p.split_stride);
}

// grid (T, ceil(total_heads / kHeadsPerWG)): one workgroup per (token, group of 8 heads) so a
// decode step of B tokens launches B * 10 workgroups (70B) instead of B — the kernel is
// latency-bound, not bandwidth-bound, at one workgroup per token.
#ifndef ROPE_HPW
#define ROPE_HPW 8
#endif
constexpr int kHeadsPerWG = ROPE_HPW;

template <bool FP8, int NS>
__global__ void __launch_bounds__(128) rope_cache_kernel(RopeCacheParams p) {
  const int t = blockIdx.x;
  const int h_lo = blockIdx.y * kHeadsPerWG;
  const int D = p.D, half = D >> 1;
  const int gpr = half >> 2;  // 4-element groups per rotation half
  const bf16* row = p.qkv + (size_t)t * p.qkv_stride;
  const int pos = p.positions ? p.positions[t] : 0;
  const float* cs = nullptr;
  const float* cs_sink = nullptr;
  if (p.cos_sin) {
    int pc = pos < 0 ? 0 : (pos >= p.max_pos ? p.max_pos - 1 : pos);
    cs = p.cos_sin + (size_t)pc * D;
    if (p.q_sink_out) {
      int ps = pos < p.window - 1 ? pos : p.window - 1;
      ps = ps < 0 ? 0 : (ps >= p.max_pos ? p.max_pos - 1 : ps);
      cs_sink = p.cos_sin + (size_t)ps * D;
    }
  }
  const long slot = p.slot_mapping ? p.slot_mapping[t] : -1;
  const long blk = slot >= 0 ? slot / p.bs : 0;
  const int off = slot >= 0 ? (int)(slot % p.bs) : 0;

  // heads of this workgroup: [h_lo, h_hi) over the concatenated q | k | v head list
  const int n_qk = p.nh + p.nkv;
  const int h_hi = min(h_lo + kHeadsPerWG, n_qk + p.nkv);

  // ---- q and k heads (rotation) -------------------------------------------------------------
  const int rot_lo = h_lo * gpr, rot_hi = min(h_hi, n_qk) * gpr;
  for (int it = rot_lo + threadIdx.x; it < rot_hi; it += blockDim.x) {
    const int head = it / gpr;
    const int i = (it % gpr) * 4;
    const bf16x4 a = load_qkv4<NS>(p, row, t, head * D + i);
    const bf16x4 b = load_qkv4<NS>(p, row, t, head * D + half + i);
    bf16x4 oa = a, ob = b;
    if (cs) rotate4(a, b, cs, i, half, oa, ob);
    if (head < p.nh) {
      bf16* dst = p.q_out + ((size_t)t * p.nh + head) * D;
      *reinterpret_cast<bf16x4*>(dst + i) = oa;
      *reinterpret_cast<bf16x4*>(dst + half + i) = ob;
      if (p.q_sink_out) {
        bf16x4 sa = a, sb = b;
        if (cs_sink) rotate4(a, b, cs_sink, i, half, sa, sb);
        bf16* ds = p.q_sink_out + ((size_t)t * p.nh + head) * D;
        *reinterpret_cast<bf16x4*>(ds + i) = sa;
        *reinterpret_cast<bf16x4*>(ds + half + i) = sb;
      }
    } else if (slot >= 0) {
      const int kh = head - p.nh;
      const size_t base = (((size_t)blk * p.nkv + kh) * p.bs + off) * D;
      if (FP8) {
        uint8_t* dst = static_cast<uint8_t*>(p.k_cache) + base;
        const float s = p.k_inv_scale;
        *reinterpret_cast<unsigned*>(dst + i) =
            pack4_fp8((float)oa[0] * s, (float)oa[1] * s, (float)oa[2] * s, (float)oa[3] * s);
        *reinterpret_cast<unsigned*>(dst + half + i) =
            pack4_fp8((float)ob[0] * s, (float)ob[1] * s, (float)ob[2] * s, (float)ob[3] * s);
      } else {
        bf16* dst = static_cast<bf16*>(p.k_cache) + base;
        *reinterpret_cast<bf16x4*>(dst + i) = oa;
        *reinterpret_cast<bf16x4*>(dst + half + i) = ob;
      }
    }
  }
  // ---- v heads (V^T scatter) ----------------------------------------------------------------
  // one element per lane, consecutive lanes -> consecutive d: in the [bs/8, D, 8] layout the 8
  // lanes d0..d0+7 store into ONE 128-B line (16-B stride, same key slot), so a wave's store
  // instruction touches 8 lines instead of 64
  if (slot >= 0 && h_hi > n_qk) {
    const int v_lo = max(h_lo - n_qk, 0) * D, v_hi = (h_hi - n_qk) * D;
    const int vcol = n_qk * D;
    const size_t grp = ((size_t)blk * p.nkv) * (p.bs >> 3) + (off >> 3);
    for (int it = v_lo + threadIdx.x; it < v_hi; it += blockDim.x) {
      const int kh = it / D, d = it % D;
      const size_t e = ((grp + (size_t)kh * (p.bs >> 3)) * D + d) * 8 + (off & 7);
      const bf16 v = load_qkv1<NS>(p, row, t, vcol + it);
      if (FP8)
        static_cast<uint8_t*>(p.v_cache)[e] = f32_to_fp8((float)v * p.v_inv_scale);
      else
        static_cast<bf16*>(p.v_cache)[e] = v;
    }
  }
}

// ---- 16-byte variant (D % 16 == 0): every load is 16 bytes per partial ---------------------------
// Same arithmetic per element as rope_cache_kernel (bit-identical output), but a lane rotates 8
// consecutive elements of each half (bf16x8 / two f32x4 per partial) and the V^T scatter gives a
// lane 8 consecutive d of one head: the 4- and 2-byte loads of the kernel above, and its 8-pass
// serial loop over the v heads in one workgroup per token, were what bounded it (a decode step's
// QKV partials are 3 x 512 x 10240 values).
__device__ __forceinline__ void rotate8(const bf16x8& a, const bf16x8& b, const float* cs,
                                        int i, int half, bf16x8& oa, bf16x8& ob) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float c = cs[i + j], s = cs[half + i + j];
    const float x = (float)a[j], y = (float)b[j];
    oa[j] = (bf16)__builtin_fmaf(x, c, -(y * s));
    ob[j] = (bf16)__builtin_fmaf(y, c, x * s);
  }
}

template <int NS>
__device__ __forceinline__ bf16x8 load_qkv8(const RopeCacheParams& p, const bf16* row, int t,
                                            int c) {
  if constexpr (NS == 0) {
    return *reinterpret_cast<const bf16x8*>(row + c);
  } else {
    bf16x8 o;
    const size_t off = (size_t)t * p.qkv_stride + c;
    if (p.parts_bf16)
      sum_parts8<NS>(static_cast<const bf16*>(p.qkv_parts) + off, p.split_stride, o);
    else
      sum_parts8<NS>(static_cast<const float*>(p.qkv_parts) + off, p.split_stride, o);
    return o;
  }
}

// One wave per workgroup (ROPE_THREADS): 8 heads' rotation groups are 64 lanes' work, so a
// 128-thread workgroup left its second wave idle in 9 of every 10 workgroups.  64 threads:
// 15.1 vs 17.6 us (bf16 KV) and 13.8 vs 15.9 us (fp8 KV) at 70B x 512 rows
// (scripts/rope_bench.py, profiles/r5/rope_threads/).
#ifndef ROPE_THREADS
#define ROPE_THREADS 64
#endif
template <bool FP8, int NS>
__global__ void __launch_bounds__(ROPE_THREADS) rope_cache_kernel_v8(RopeCacheParams p) {
  const int t = blockIdx.x;
  const int h_lo = blockIdx.y * kHeadsPerWG;
  const int D = p.D, half = D >> 1;
  const int gpr = half >> 3;  // 8-element groups per rotation half
  const bf16* row = p.qkv + (size_t)t * p.qkv_stride;
  const int pos = p.positions ? p.positions[t] : 0;
  const float* cs = nullptr;
  const float* cs_sink = nullptr;
  if (p.cos_sin) {
    int pc = pos < 0 ? 0 : (pos >= p.max_pos ? p.max_pos - 1 : pos);
    cs = p.cos_sin + (size_t)pc * D;
    if (p.q_sink_out) {
      int ps = pos < p.window - 1 ? pos : p.window - 1;
      ps = ps < 0 ? 0 : (ps >= p.max_pos ? p.max_pos - 1 : ps);
      cs_sink = p.cos_sin + (size_t)ps * D;
    }
  }
  const long slot = p.slot_mapping ? p.slot_mapping[t] : -1;
  const long blk = slot >= 0 ? slot / p.bs : 0;
  const int off = slot >= 0 ? (int)(slot % p.bs) : 0;
  const int n_qk = p.nh + p.nkv;
  const int h_hi = min(h_lo + kHeadsPerWG, n_qk + p.nkv);

  const int rot_lo = h_lo * gpr, rot_hi = min(h_hi, n_qk) * gpr;
  for (int it = rot_lo + threadIdx.x; it < rot_hi; it += blockDim.x) {
    const int head = it / gpr;
    const int i = (it % gpr) * 8;
    const bf16x8 a = load_qkv8<NS>(p, row, t, head * D + i);
    const bf16x8 b = load_qkv8<NS>(p, row, t, head * D + half + i);
    bf16x8 oa = a, ob = b;
    if (cs) rotate8(a, b, cs, i, half, oa, ob);
    if (head < p.nh) {
      bf16* dst = p.q_out + ((size_t)t * p.nh + head) * D;
      *reinterpret_cast<bf16x8*>(dst + i) = oa;
      *reinterpret_cast<bf16x8*>(dst + half + i) = ob;
      if (p.q_sink_out) {
        bf16x8 sa = a, sb = b;
        if (cs_sink) rotate8(a, b, cs_sink, i, half, sa, sb);
        bf16* ds = p.q_sink_out + ((size_t)t * p.nh + head) * D;
        *reinterpret_cast<bf16x8*>(ds + i) = sa;
        *reinterpret_cast<bf16x8*>(ds + half + i) = sb;
      }
    } else if (slot >= 0) {
      const int kh = head - p.nh;
      const size_t base = (((size_t)blk * p.nkv + kh) * p.bs + off) * D;
      if (FP8) {
        uint8_t* dst = static_cast<uint8_t*>(p.k_cache) + base;
        const float s = p.k_inv_scale;
        uint2 va, vb;
        va.x = pack4_fp8((float)oa[0] * s, (float)oa[1] * s, (float)oa[2] * s, (float)oa[3] * s);
        va.y = pack4_fp8((float)oa[4] * s, (float)oa[5] * s, (float)oa[6] * s, (float)oa[7] * s);
        vb.x = pack4_fp8((float)ob[0] * s, (float)ob[1] * s, (float)ob[2] * s, (float)ob[3] * s);
        vb.y = pack4_fp8((float)ob[4] * s, (float)ob[5] * s, (float)ob[6] * s, (float)ob[7] * s);
        *reinterpret_cast<uint2*>(dst + i) = va;
        *reinterpret_cast<uint2*>(dst + half + i) = vb;
      } else {
        bf16* dst = static_cast<bf16*>(p.k_cache) + base;
        *reinterpret_cast<bf16x8*>(dst + i) = oa;
        *reinterpret_cast<bf16x8*>(dst + half + i) = ob;
      }
    }
  }
  // V^T scatter: lane = (v head, 8 consecutive d); its 8 stores land 16 B apart in one line
  if (slot >= 0 && h_hi > n_qk) {
    const int g8 = D >> 3;
    const int v_lo = max(h_lo - n_qk, 0) * g8, v_hi = (h_hi - n_qk) * g8;
    const int vcol = n_qk * D;
    const size_t grp = ((size_t)blk * p.nkv) * (p.bs >> 3) + (off >> 3);
    for (int it = v_lo + threadIdx.x; it < v_hi; it += blockDim.x) {
      const int kh = it / g8, d0 = (it % g8) * 8;
      const bf16x8 v = load_qkv8<NS>(p, row, t, vcol + kh * D + d0);
      const size_t e0 = ((grp + (size_t)kh * (p.bs >> 3)) * D + d0) * 8 + (off & 7);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (FP8)
          static_cast<uint8_t*>(p.v_cache)[e0 + 8 * j] = f32_to_fp8((float)v[j] * p.v_inv_scale);
        else
          static_cast<bf16*>(p.v_cache)[e0 + 8 * j] = v[j];
      }
    }
  }
}

int launch_rope_cache(const RopeCacheParams& p, int num_tokens, hipStream_t stream) {
  if (num_tokens == 0) return 0;
  if (p.D % 8 != 0 || p.qkv_stride % 4 != 0) return -1;
  if (p.qkv_parts != nullptr && (p.splits < 1 || p.split_stride % 4 != 0)) return -2;
  const int heads = p.nh + 2 * p.nkv;
  dim3 grid(num_tokens, (heads + kHeadsPerWG - 1) / kHeadsPerWG);
#ifdef PROBE_NS1   // diagnostic (scripts/split_k_upper_bound.sh): read split 0 only
  const int ns = p.qkv_parts != nullptr ? 1 : 0;
#else
  const int ns = p.qkv_parts != nullptr ? p.splits : 0;
#endif
  // 16-byte path: both rotation halves and every head start on 16-byte boundaries of every
  // partial (otherwise the 4-element kernel)
  const bool v8 = p.D % 16 == 0 && p.qkv_stride % 8 == 0 &&
                  (p.qkv_parts == nullptr || p.split_stride % 8 == 0);
#define ROPE_LAUNCH(NS)                                                   \
  do {                                                                 \
    if (v8) {                                                          \
      if (p.kv_fp8)                                                    \
        rope_cache_kernel_v8<true, NS><<<grid, ROPE_THREADS, 0, stream>>>(p);   \
      else                                                             \
        rope_cache_kernel_v8<false, NS><<<grid, ROPE_THREADS, 0, stream>>>(p);  \
    } else if (p.kv_fp8)                                               \
      rope_cache_kernel<true, NS><<<grid, 128, 0, stream>>>(p);        \
    else                                                               \
      rope_cache_kernel<false, NS><<<grid, 128, 0, stream>>>(p);       \
  } while (0)
  SPLITS_SWITCH(ns, ROPE_LAUNCH)
#undef ROPE_LAUNCH
  return 0;
}

}  // namespace dli
