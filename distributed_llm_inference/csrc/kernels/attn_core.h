// Decode / prefill attention building blocks shared by attention.hip and the batch-1 decode-layer
// kernel (decode_layer.hip): MFMA fragments, online softmax, K / V^T cache loads, slot masks.
// Layouts and the swapped-operand orientation are described at the top of attention.hip.
#pragma once
#include "kernels.h"

namespace dli {

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Block-table entry of a wave-uniform index, by a scalar load waited on in place.  A plain
// bt[i] inside the decode loop compiles to a VECTOR load (the loop's sched_barrier is a memory
// side effect to the clobber analysis, so the load is not proven read-only-so-far), and its
// vmcnt(0) wait drained the prefetched K/V of the next step every step.  The scalar load joins
// only the lgkm queue: the K/V loads in flight stay in flight.
__device__ __forceinline__ int bt_entry(const int* bt, int i) {
  const int* a = bt + __builtin_amdgcn_readfirstlane(i);
  int v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a));
  return v;
}

__device__ __forceinline__ bf16x8 zero8() {
  i32x4 z = {0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, z);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Absolute token index of ring slot `u` (window mode) given the sequence length L.
__device__ __forceinline__ int ring_abs(int u, int L, const AttnParams& p) {
  const int o = u - p.sink_pad;
  const int newest = (L - 1 - p.n_sink) % p.ring;
  int back = newest - o;
  if (back < 0) back += p.ring;
  return (L - 1) - back;
}

// Online-softmax state of one wave: O^T accumulators, running max (log2 domain) and row sum.
template <int D>
struct WaveState {
  f32x4 o[D / 16];
  float m, l;
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int e = 0; e < D / 16; ++e) o[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    m = -1e30f;
    l = 0.f;
  }
};

// K/V fragments of one 32-key step (registers): K rows permuted (see header), V^T rows.
template <int D>
struct KVFrag {
  bf16x8 k[2][D / 32];
  bf16x8 v[D / 16];
};

// fp8 decode with D % 64 == 0 reads K and V^T with 16-byte loads (like bf16) by permuting the
// head dimension d, which both products are free to do as long as every operand agrees:
//   * S^T = K . Q^T sums over d: lane (col, h4) takes d = 64c' + 16h4 + [0, 16) of a chunk pair
//     (2c', 2c'+1) — one 16-byte K load — and Q is loaded with the same map (q_dofs);
//   * O^T rows are d: row i of V^T blocks (2e', 2e'+1) is d = 32e' + 2i + {0, 1}, one 16-byte
//     load of two adjacent d's 8 keys each, so a lane's accumulators hold d = 32e' + 8h4 + [0, 8)
//     (o_dofs) and the output is written with that map.
template <int D, bool FP8>
struct DPerm {
  static constexpr bool on = FP8 && D % 64 == 0;
};

// element offset of the 8 q values of chunk c held by lane group h4
template <int D, bool FP8>
__device__ __forceinline__ int q_dofs(int c, int h4) {
  return DPerm<D, FP8>::on ? 64 * (c >> 1) + 16 * h4 + 8 * (c & 1) : 32 * c + 8 * h4;
}

//   kc/vc: the K / V^T caches, hb: element offset of this kv head's page, offk: slot offset of the
//   step inside the page.  fp8 caches widen to bf16 in registers (exact), so both MFMA products
//   stay bf16 x bf16.
// 16-B K/V load; NT = non-temporal (the cache is streamed once per step: no reuse to keep)
template <bool NT>
__device__ __forceinline__ bf16x8 kv_ld16(const bf16* p) {
  if constexpr (NT) {
    typedef int i32x4_t __attribute__((ext_vector_type(4)));
    return __builtin_bit_cast(bf16x8, __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(p)));
  } else {
    return *reinterpret_cast<const bf16x8*>(p);
  }
}

// nvalid (< 32: the sequence's last step): key rows / 8-key V^T groups at or past it are not
// fetched (zeros; their scores are masked anyway) - on average half a step per sequence and kv
// head, ~2.5 % of the KV bytes at 600-token contexts.
template <int D, bool FP8, bool NT = false>
__device__ __forceinline__ void attn_load(KVFrag<D>& f, const void* __restrict__ kc,
                                          const void* __restrict__ vc, size_t hb, int offk,
                                          int nvalid = 32) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, h4 = lane >> 4;
  const int krow0 = offk + 8 * (col >> 2) + (col & 3);
  if constexpr (DPerm<D, FP8>::on) {
    const uint8_t* k8 = static_cast<const uint8_t*>(kc);
    const uint8_t* v8 = static_cast<const uint8_t*>(vc);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c2 = 0; c2 < D / 64; ++c2) {
        const uint4 r = *reinterpret_cast<const uint4*>(k8 + hb + (size_t)(krow0 + 4 * t) * D + 64 * c2 + 16 * h4);
        f.k[t][2 * c2] = fp8x8_to_bf16x8(make_uint2(r.x, r.y));
        f.k[t][2 * c2 + 1] = fp8x8_to_bf16x8(make_uint2(r.z, r.w));
      }
#pragma unroll
    for (int e2 = 0; e2 < D / 32; ++e2) {
      const uint4 r = *reinterpret_cast<const uint4*>(
          v8 + hb + ((size_t)((offk >> 3) + h4) * D + 32 * e2 + 2 * col) * 8);
      f.v[2 * e2] = fp8x8_to_bf16x8(make_uint2(r.x, r.y));
      f.v[2 * e2 + 1] = fp8x8_to_bf16x8(make_uint2(r.z, r.w));
    }
    return;
  }
  // Keys past the sequence end (nvalid >= 1 of this step's 32) are not fetched: their rows /
  // 8-key groups are clamped to the last valid one, a line already being read, so every load is
  // issued unconditionally (no exec-masked branches: hipcc then counts the vmcnt waits and the
  // next step's prefetch stays in flight through this step's MFMAs).  The clamped keys are
  // invisible to the softmax (p = 0 exactly) and their finite V values add exact zeros.
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kr = min(krow0 + 4 * t, offk + nvalid - 1);
#pragma unroll
    for (int c = 0; c < D / 32; ++c) {
      const size_t e = hb + (size_t)kr * D + 32 * c + 8 * h4;
      if (FP8)
        f.k[t][c] = fp8x8_to_bf16x8(*reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(kc) + e));
      else
        f.k[t][c] = kv_ld16<NT>(static_cast<const bf16*>(kc) + e);
    }
  }
  const int vg = min(h4, (nvalid - 1) >> 3);
#pragma unroll
  for (int e = 0; e < D / 16; ++e) {
    const size_t o = hb + ((size_t)((offk >> 3) + vg) * D + 16 * e + col) * 8;
    if (FP8)
      f.v[e] = fp8x8_to_bf16x8(*reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(vc) + o));
    else
      f.v[e] = kv_ld16<NT>(static_cast<const bf16*>(vc) + o);
  }
}

// fp8 decode (DPerm on): the raw bytes of one 32-key step — half the registers of the widened
// fragments, so the loop can keep three steps in flight and widen each just before its MFMAs.
template <int D>
struct KVRaw {
  uint4 k[2][D / 64];
  uint4 v[D / 32];
};

template <int D>
__device__ __forceinline__ void attn_load_raw(KVRaw<D>& r, const void* __restrict__ kc,
                                              const void* __restrict__ vc, size_t hb, int offk) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, h4 = lane >> 4;
  const int krow0 = offk + 8 * (col >> 2) + (col & 3);
  const uint8_t* k8 = static_cast<const uint8_t*>(kc);
  const uint8_t* v8 = static_cast<const uint8_t*>(vc);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c2 = 0; c2 < D / 64; ++c2)
      r.k[t][c2] = *reinterpret_cast<const uint4*>(k8 + hb + (size_t)(krow0 + 4 * t) * D + 64 * c2 + 16 * h4);
#pragma unroll
  for (int e2 = 0; e2 < D / 32; ++e2)
    r.v[e2] = *reinterpret_cast<const uint4*>(v8 + hb + ((size_t)((offk >> 3) + h4) * D + 32 * e2 + 2 * col) * 8);
}

template <int D>
__device__ __forceinline__ void attn_widen(KVFrag<D>& f, const KVRaw<D>& r) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c2 = 0; c2 < D / 64; ++c2) {
      f.k[t][2 * c2] = fp8x8_to_bf16x8(make_uint2(r.k[t][c2].x, r.k[t][c2].y));
      f.k[t][2 * c2 + 1] = fp8x8_to_bf16x8(make_uint2(r.k[t][c2].z, r.k[t][c2].w));
    }
#pragma unroll
  for (int e2 = 0; e2 < D / 32; ++e2) {
    f.v[2 * e2] = fp8x8_to_bf16x8(make_uint2(r.v[e2].x, r.v[e2].y));
    f.v[2 * e2 + 1] = fp8x8_to_bf16x8(make_uint2(r.v[e2].z, r.v[e2].w));
  }
}

// The D/16 f32x4 units of O^T a lane holds (query column col): unit u -> first d and values.
template <int D, bool FP8>
__device__ __forceinline__ void o_unit(const WaveState<D>& st, int u, int h4, int& d, f32x4& v) {
  if constexpr (DPerm<D, FP8>::on) {
    const int e2 = u >> 1, r0 = (u & 1) * 2;
    d = 32 * e2 + 8 * h4 + 4 * (u & 1);
    v = f32x4{st.o[2 * e2][r0], st.o[2 * e2 + 1][r0], st.o[2 * e2][r0 + 1], st.o[2 * e2 + 1][r0 + 1]};
  } else {
    d = 16 * u + 4 * h4;
    v = st.o[u];
  }
}

// One 32-key step of online-softmax attention for the 16 query columns held by this wave.
// visible(j) decides visibility of key 8h+j (h = lane>>4) for this lane's column.  The softmax
// scale is folded into the exponent's FMA (exp2(s * scale - m)), so a masked key costs one select
// and the scores are never scaled on their own.
// (Skipping the O rescale when no running max moved, or a mask-free copy of this step for keys
// below the diagonal, cut the prefill loop's VALU count but raised its VGPRs: fewer workgroups
// per CU, measured slower.)
struct NoBias {
  __device__ __forceinline__ float operator()(int) const { return 0.f; }
};

template <int D, typename Visible, typename Bias = NoBias>
__device__ __forceinline__ void attn_core(WaveState<D>& st, const bf16x8 (&qf)[D / 32],
                                          const KVFrag<D>& f, float scale_log2, Visible visible,
                                          Bias bias = Bias()) {
  // ---- S^T = K . Q^T ----
  f32x4 s[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < D / 32; ++c) s[t] = mfma16(f.k[t][c], qf[c], s[t]);
  }
  // ---- online softmax over the 8 keys 8h..8h+7 of this lane (log2 domain) ----
  float x[8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x[j] = visible(j) ? s[j >> 2][j & 3] + bias(j) : -INFINITY;
    mx = fmaxf(mx, x[j]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float m_new = fmaxf(st.m, mx * scale_log2);
  const float alpha = __builtin_amdgcn_exp2f(st.m - m_new);
  bf16x8 pb;
  float ps = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float pj = __builtin_amdgcn_exp2f(fmaf(x[j], scale_log2, -m_new));
    ps += pj;
    pb[j] = (bf16)pj;
  }
  st.l = st.l * alpha + ps;
  st.m = m_new;
  // ---- O^T += V^T . P^T ----
#pragma unroll
  for (int e = 0; e < D / 16; ++e) {
    st.o[e] *= alpha;
    st.o[e] = mfma16(f.v[e], pb, st.o[e]);
  }
}

// valid_mask bit j = visibility of key 8h+j
template <int D>
__device__ __forceinline__ void attn_compute(WaveState<D>& st, const bf16x8 (&qf)[D / 32],
                                             const KVFrag<D>& f, float scale_log2,
                                             unsigned valid_mask) {
  attn_core<D>(st, qf, f, scale_log2, [&](int j) { return ((valid_mask >> j) & 1u) != 0; });
}

// causal: keys 8h+j with j <= lim are visible (lim = the column's position - the lane's first key)
template <int D>
__device__ __forceinline__ void attn_compute_causal(WaveState<D>& st, const bf16x8 (&qf)[D / 32],
                                                    const KVFrag<D>& f, float scale_log2, int lim) {
  attn_core<D>(st, qf, f, scale_log2, [&](int j) { return j <= lim; });
}

template <int D, bool FP8>
__device__ __forceinline__ void attn_step(WaveState<D>& st, const bf16x8 (&qf)[D / 32],
                                          const void* kc, const void* vc, size_t hb, int offk,
                                          float scale_log2, unsigned valid_mask) {
  KVFrag<D> f;
  attn_load<D, FP8>(f, kc, vc, hb, offk);
  attn_compute<D>(st, qf, f, scale_log2, valid_mask);
}

template <int D, bool WIN>
__device__ __forceinline__ unsigned step_mask(int u0, int h4, int seg_base, int seg_len, int L,
                                              const AttnParams& p) {
  unsigned vm = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int u = u0 + 8 * h4 + j;
    bool ok = (u - seg_base) < seg_len;
    if (WIN && ok) {
      const int a = ring_abs(u, L, p);
      ok = a >= p.n_sink && (L - 1 - a) < (p.window - p.n_sink);
    }
    vm |= (ok ? 1u : 0u) << j;
  }
  return vm;
}

// One decode work item (sequence b, kv head, group of 16 q heads, split) of a wave: its online-
// softmax state over the split's keys (and the sink segment in window mode).  attn_decode_kernel
// writes / merges the result; the batch-1 decode-layer kernel writes split partials.
struct DecodeItem {
  int split, b, kvh, g0, G, hgroups;
  bool col_valid;
  float vsc;   // fp8 caches: V's scale, applied to the output
};

template <int D, bool WIN, bool FP8, bool NT, bool ONE_STEP = false>
__device__ __forceinline__ DecodeItem attn_decode_item(const AttnParams& p, int item, bool live,
                                                       WaveState<D>& st) {
  const int splits = p.num_splits;
  const int split = item % splits;
  int rest = item / splits;
  const int G = p.nh / p.nkv;
  const int hgroups = (G + 15) >> 4;
  const int g0 = (rest % hgroups) * 16;
  rest /= hgroups;
  const int kvh = rest % p.nkv;
  const int b = rest / p.nkv;
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, h4 = lane >> 4;
  const bool col_valid = (g0 + col) < G;
  const int qh = kvh * G + g0 + (col_valid ? col : 0);
  const int L = live ? p.seq_lens[b] : 0;
  const int* bt = p.block_tables + (size_t)b * p.bt_stride;
  const size_t head_stride = (size_t)p.bs * D;  // per (block, kv head)

  // fp8 caches: K's scale folds into the softmax scale, V's into the output
  const float sl2 = FP8 ? p.scale_log2 * p.k_scale : p.scale_log2;
  const float vsc = FP8 ? p.v_scale : 1.f;
  st.init();
  if (L > 0) {
    bf16x8 qf[D / 32];
    const bf16* qrow = p.q + ((size_t)b * p.nh + qh) * D;
#pragma unroll
    for (int c = 0; c < D / 32; ++c)
      qf[c] = col_valid ? *reinterpret_cast<const bf16x8*>(qrow + q_dofs<D, FP8>(c, h4)) : zero8();
    // ---- rolling / full segment ----
    int seg_base, seg_len;
    if (WIN) {
      seg_base = p.sink_pad;
      seg_len = L > p.n_sink ? min(p.ring, L - p.n_sink) : 0;
    } else {
      seg_base = 0;
      seg_len = L;
    }
    const int nsteps = (seg_len + 31) >> 5;
    const int per_split = (nsteps + splits - 1) / splits;
    const int s_lo = split * per_split;
    const int s_hi = min(nsteps, s_lo + per_split);
    if (s_lo < s_hi) {
      auto load = [&](KVFrag<D>& f, int sidx) {
        const int u0 = seg_base + sidx * 32;
        const int page = bt_entry(bt, u0 / p.bs);
        const size_t hb = ((size_t)page * p.nkv + kvh) * head_stride;
        // full-cache mode: keys past the sequence end are not fetched (ring mode: all 32, its
        // validity is positional)
        attn_load<D, FP8, NT>(f, p.k_cache, p.v_cache, hb, u0 % p.bs,
                              WIN ? 32 : seg_len - sidx * 32);
      };
      if constexpr (DPerm<D, FP8>::on) {
        // three raw steps in flight, each widened right before its MFMAs
        auto rload = [&](KVRaw<D>& r, int sidx) {
          const int u0 = seg_base + sidx * 32;
          const int page = bt_entry(bt, u0 / p.bs);
          const size_t hb = ((size_t)page * p.nkv + kvh) * head_stride;
          attn_load_raw<D>(r, p.k_cache, p.v_cache, hb, u0 % p.bs);
        };
        auto step = [&](const KVRaw<D>& r, int sidx) {
          KVFrag<D> f;
          attn_widen<D>(f, r);
          attn_compute<D>(st, qf, f, sl2,
                          step_mask<D, WIN>(seg_base + sidx * 32, h4, seg_base, seg_len, L, p));
        };
        if constexpr (ONE_STEP) {   // one raw step per wave at 4 waves per SIMD (see below)
          for (int sidx = s_lo; sidx < s_hi; ++sidx) {
            KVRaw<D> r;
            rload(r, sidx);
            step(r, sidx);
          }
        } else {
        KVRaw<D> r0, r1, r2;
        rload(r0, s_lo);
        rload(r1, min(s_lo + 1, s_hi - 1));
        for (int sidx = s_lo; sidx < s_hi; sidx += 3) {
          rload(r2, min(sidx + 2, s_hi - 1));
          __builtin_amdgcn_sched_barrier(0);
          step(r0, sidx);
          rload(r0, min(sidx + 3, s_hi - 1));
          __builtin_amdgcn_sched_barrier(0);
          if (sidx + 1 < s_hi) step(r1, sidx + 1);
          rload(r1, min(sidx + 4, s_hi - 1));
          __builtin_amdgcn_sched_barrier(0);
          if (sidx + 2 < s_hi) step(r2, sidx + 2);
        }
        }
      } else {
      if constexpr (ONE_STEP) {
        // one step per wave in flight and 4 waves per SIMD (96 VGPRs; attn_decode_kernel's
        // launch bounds) instead of two steps at 2 waves: the same bytes in flight per SIMD,
        // twice the waves to hide latency, and B = 512 x 8 kv heads = 4096 waves in ONE round
        // (profiles/r5/attn_one_step.md: 600 keys 213.6 vs 220.7 us, 1100 keys 397 vs 405)
        for (int sidx = s_lo; sidx < s_hi; ++sidx) {
          KVFrag<D> f;
          load(f, sidx);
          attn_compute<D>(st, qf, f, sl2,
                          step_mask<D, WIN>(seg_base + sidx * 32, h4, seg_base, seg_len, L, p));
        }
      } else {
      KVFrag<D> fa, fb;
      load(fa, s_lo);
      // sched_barrier(0): keep each prefetch group issued ahead of the previous step's MFMAs
      // (the machine scheduler otherwise sinks the loads next to their first use)
      for (int sidx = s_lo; sidx < s_hi; sidx += 2) {
        load(fb, min(sidx + 1, s_hi - 1));
        __builtin_amdgcn_sched_barrier(0);
        attn_compute<D>(st, qf, fa, sl2,
                        step_mask<D, WIN>(seg_base + sidx * 32, h4, seg_base, seg_len, L, p));
        load(fa, min(sidx + 2, s_hi - 1));
        __builtin_amdgcn_sched_barrier(0);
        if (sidx + 1 < s_hi)
          attn_compute<D>(st, qf, fb, sl2,
                          step_mask<D, WIN>(seg_base + (sidx + 1) * 32, h4, seg_base, seg_len, L, p));
      }
      }
      }
    }
    // ---- sink segment (window mode): scored with q_sink by the split-0 wave ----
    if (WIN && split == 0 && p.n_sink > 0) {
      bf16x8 qs[D / 32];
      const bf16* qsrow = p.q_sink + ((size_t)b * p.nh + qh) * D;
#pragma unroll
      for (int c = 0; c < D / 32; ++c)
        qs[c] = col_valid ? *reinterpret_cast<const bf16x8*>(qsrow + q_dofs<D, FP8>(c, h4)) : zero8();
      const int nS = min(p.n_sink, L);
      for (int u0 = 0; u0 < nS; u0 += 32) {
        const int page = bt_entry(bt, u0 / p.bs);
        const size_t hb = ((size_t)page * p.nkv + kvh) * head_stride;
        unsigned vm = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) vm |= ((u0 + 8 * h4 + j) < nS ? 1u : 0u) << j;
        attn_step<D, FP8>(st, qs, p.k_cache, p.v_cache, hb, u0 % p.bs, sl2, vm);
      }
    }
  }
  DecodeItem di;
  di.split = split;
  di.b = b;
  di.kvh = kvh;
  di.g0 = g0;
  di.G = G;
  di.hgroups = hgroups;
  di.col_valid = col_valid;
  di.vsc = vsc;
  return di;
}

}  // namespace dli
