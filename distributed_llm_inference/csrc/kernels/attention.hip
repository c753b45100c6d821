// Paged attention for CDNA4 (gfx950): decode (split-K flash-decoding) and prefill (causal flash).
//
// Replaces the reference's eager attention core (modules.py:87-97: repeat_kv materialisation,
// QK^T/sqrt(D) + additive mask, fp32 softmax, PV) and its mask builder (model.py:78-143).
//   * GQA is native: one workgroup serves all q heads of a kv head (decode) — K/V are read once.
//   * causality / window / padding come from seq_lens and slot arithmetic, never from a mask tensor.
//   * both products run on MFMA v_mfma_f32_16x16x32_bf16 in the "swapped" orientation
//        S^T[key, q] = K[key, d] . Q^T[d, q]        (A = K rows, B = Q^T)
//        O^T[d, q]  += V^T[d, key] . P^T[key, q]     (A = V^T rows, B = P^T)
//     With K cached as [blocks, nkv, bs, D] and V cached as V^T in 8-key groups
//     [blocks, nkv, bs/8, D, 8] (16 lanes with consecutive d read 256 contiguous bytes), every
//     MFMA A operand is one 16-byte global load per lane, and the S^T accumulator is re-used as the
//     P^T operand with no lane movement: the K rows of the two 16-key S tiles of a 32-key step are
//     permuted (row i of tile t holds key 8(i>>2) + 4t + (i&3)) so that lane (h=l>>4, col=l&15)
//     ends up holding the scores of keys 8h..8h+7 for query column col — exactly the k-slice the
//     P^T operand of the next MFMA needs (cdna_hip_programming.md §3, "accumulator as operand").
//   * softmax is online (running max per column, exp2 with log2(e) folded into the scale); the
//     row max needs two xor-shuffles (lanes 16 and 32 apart share a column); row sums are kept
//     per lane and reduced once at the end.
//   * Attention-sink (StreamingLLM) windows, the reference's PartialLlamaSinkCache semantics
//     (cache.py:64-135), are handled in slot space: sink slots [0, n_sink) are scored with
//     q_sink (q rotated at min(pos, W-1)); rolling slots live in a ring of `ring` slots starting
//     at `sink_pad`, stored rotated at their absolute positions and scored with q rotated at its
//     absolute position — relative distances are then exactly the re-rotated ones, with no
//     re-rotation pass over the cache.
#include "kernels.h"
#include "attn_core.h"

#include <type_traits>

namespace dli {

// ===========================================================================================
// Decode: one wave per work item (sequence b, kv head, group of 16 q heads, split), 4 waves per
// 256-thread workgroup.  A wave walks its split's 32-key steps with the loads of step s+1 in flight
// while step s computes (two register fragment sets; the prefetch index is clamped instead of
// branched so the loads stay straight-line and hipcc can wait with a counted vmcnt).
//   * one split (large batches): 4 independent waves, no LDS, no barrier; each writes the
//     normalised output;
//   * num_splits > 1 (small batches / long contexts: up to hundreds of splits so that even B = 1
//     puts several waves on every CU): the workgroup's waves hold `gs` (4 or 2) consecutive
//     splits of one item and merge them through LDS (online-softmax rescale, padded O^T image),
//     so only num_splits / gs partials per head go to HBM — and none when num_splits == gs;
//     attn_combine_kernel merges what is left.  (A last-arrival merge inside this kernel was
//     measured slower than the combine launch at B = 1 - 600 keys 11.3 vs 10.6 us, 8k keys
//     28.1 vs 15.0 us, one workgroup merging up to 32 partials serially - and lives in
//     scripts/experiments/.)
// ===========================================================================================
// ONE (full-cache single-split decode of a batch large enough to fill the chip, bf16 or fp8
// KV): one key step per wave in flight at 4 waves per SIMD (attn_core.h ONE_STEP, 96 / 104
// VGPRs) instead of two (fp8: three raw) steps at 2 waves -- the same bytes in flight per SIMD,
// twice the waves, and B = 512 x 8 kv heads = 4096 waves in ONE round.  With fewer waves than
// the chip holds at 4 per SIMD the deeper prefetch wins (fp8 KV at 1024 waves: 148 vs 99 us),
// so decode_grid picks ONE by the item count (profiles/r5/attn_one_step.md).
template <int D, bool WIN, bool FP8, bool GRP, bool ONE = false>
__global__ void __launch_bounds__(256, (ONE ? 4 : 1))
attn_decode_kernel(AttnParams p, int items, int gs) {
  // GRP (num_splits > 1): the `gs` consecutive splits of one work item that share this
  // workgroup are merged in LDS, so only num_splits / gs partials per head reach global memory
  // (none when gs == num_splits: the workgroup writes the normalised output itself)
  constexpr int LROW = D + 4;  // padded O^T column: conflict-free ds_write_b128
  __shared__ __attribute__((aligned(16))) float lds[GRP ? 4 * 16 * (LROW + 2) : 1];
  const int wave = threadIdx.x >> 6;
  const int item_raw = blockIdx.x * 4 + wave;
  const bool live = item_raw < items;
  if (!GRP && !live) return;  // whole wave idle (no barrier in the ungrouped kernel)
  // wave-uniform by construction; readfirstlane tells hipcc so, which turns every index derived
  // from it (seq_lens, block-table entries) into scalar loads that never join the vmcnt queue
  // of the K/V prefetch
  const int item = __builtin_amdgcn_readfirstlane(live ? item_raw : items - 1);
  WaveState<D> st;
  const DecodeItem di = attn_decode_item<D, WIN, FP8, false, ONE>(p, item, live, st);
  const int splits = p.num_splits, split = di.split, G = di.G, hgroups = di.hgroups;
  const int g0 = di.g0, kvh = di.kvh, b = di.b;
  const int lane = threadIdx.x & 63, col = lane & 15, h4 = lane >> 4;
  const bool col_valid = di.col_valid;
  const float vsc = di.vsc;
  // ---- write: lane (col, h4) holds the O^T units o_unit() of query column col ----
  float lsum = st.l;
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const size_t B = (size_t)items / ((size_t)splits * hgroups * p.nkv);
  if constexpr (!GRP) {
    if (!col_valid) return;
    const int head = kvh * G + g0 + col;
    if (splits == 1) {
      const float inv = lsum > 0.f ? vsc / lsum : 0.f;
      if constexpr (D == 128) {
        if (p.out_q != nullptr) {
          // MX fp8 hand-off to the O projection (ops.attn_decode mx_out): the values the bf16
          // store would write, one e8m0 scale per head row (= one 128-column block of O's
          // input), amax over the 4 lanes holding the row (h4 = lane >> 4)
          f32x4 vals[D / 16];
          int dd[D / 16];
          float a = 0.f;
#pragma unroll
          for (int u = 0; u < D / 16; ++u) {
            f32x4 o;
            o_unit<D, FP8>(st, u, h4, dd[u], o);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              vals[u][r] = (float)(bf16)(o[r] * inv);
              a = fmaxf(a, fabsf(vals[u][r]));
            }
          }
          a = fmaxf(a, __shfl_xor(a, 16, 64));
          a = fmaxf(a, __shfl_xor(a, 32, 64));
          const int k = mx_exponent(a);
          const float si = mx_inv_scale(k);
          uint8_t* qrow = p.out_q + ((size_t)b * p.nh + head) * D;
#pragma unroll
          for (int u = 0; u < D / 16; ++u) {
            const f32x4 v = vals[u] * si;
            *reinterpret_cast<unsigned*>(qrow + dd[u]) = pack4_fp8(v[0], v[1], v[2], v[3]);
          }
          if (h4 == 0) {
            const int nb = ((int)B + 63) / 64;
            p.out_mx[mx_off(head, b, nb)] = (uint8_t)(k + 127);
            if (b == (int)B - 1)   // padding rows of the last 64-row block: scale 2^0
              for (int r = (int)B; r < nb * 64; ++r) p.out_mx[mx_off(head, r, nb)] = 127;
          }
          return;
        }
      }
      bf16* orow = p.out + ((size_t)b * p.nh + head) * D;
#pragma unroll
      for (int u = 0; u < D / 16; ++u) {
        int d;
        f32x4 o;
        o_unit<D, FP8>(st, u, h4, d, o);
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[r] * inv);
        *reinterpret_cast<bf16x4*>(orow + d) = v;
      }
    } else {
      const size_t r0 = ((size_t)split * B + b) * p.nh + head;
      float* prow = p.part_o + r0 * D;
#pragma unroll
      for (int u = 0; u < D / 16; ++u) {
        int d;
        f32x4 o;
        o_unit<D, FP8>(st, u, h4, d, o);
        *reinterpret_cast<f32x4*>(prow + d) = o * vsc;
      }
      if (h4 == 0) {
        p.part_ml[r0 * 2] = st.m;
        p.part_ml[r0 * 2 + 1] = lsum;
      }
    }
  } else {
    // ---- merge the gs waves of each group in LDS ----
    float* lo = lds + (wave * 16 + col) * LROW;
    float* lml = lds + 4 * 16 * LROW;  // [wave][col][m, l]
#pragma unroll
    for (int u = 0; u < D / 16; ++u) {
      int d;
      f32x4 o;
      o_unit<D, FP8>(st, u, h4, d, o);
      *reinterpret_cast<f32x4*>(lo + d) = o;
    }
    if (h4 == 0) {
      lml[(wave * 16 + col) * 2] = st.m;
      lml[(wave * 16 + col) * 2 + 1] = lsum;
    }
    __syncthreads();
    const int g = wave / gs;                     // group of this wave
    const int w0 = g * gs;                       // its first wave
    const int gitem = blockIdx.x * 4 + w0;       // the group's first work item
    if (gitem >= items) return;
    const int S2 = splits / gs;                  // partials per head after the merge
    const int s2 = (gitem % splits) / gs;
    const int tg = (wave - w0) * 64 + lane;      // thread index inside the group
    constexpr int V4 = 16 * D / 4;               // f32x4 units of one group's output
    for (int u = tg; u < V4; u += gs * 64) {
      const int c = u / (D / 4), d4 = (u % (D / 4)) * 4;
      if (g0 + c >= G) continue;
      float M = -1e30f;
      for (int w = w0; w < w0 + gs; ++w) M = fmaxf(M, lml[(w * 16 + c) * 2]);
      float Lt = 0.f;
      f32x4 O = {0.f, 0.f, 0.f, 0.f};
      for (int w = w0; w < w0 + gs; ++w) {
        const float f = __builtin_amdgcn_exp2f(lml[(w * 16 + c) * 2] - M);
        Lt += f * lml[(w * 16 + c) * 2 + 1];
        O += f * *reinterpret_cast<const f32x4*>(lds + (w * 16 + c) * LROW + d4);
      }
      const int head = kvh * G + g0 + c;
      if (S2 == 1) {
        const float inv = Lt > 0.f ? vsc / Lt : 0.f;
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(O[r] * inv);
        *reinterpret_cast<bf16x4*>(p.out + ((size_t)b * p.nh + head) * D + d4) = v;
      } else {
        const size_t r0 = ((size_t)s2 * B + b) * p.nh + head;
        *reinterpret_cast<f32x4*>(p.part_o + r0 * D + d4) = O * vsc;
        if (d4 == 0) {
          p.part_ml[r0 * 2] = M;
          p.part_ml[r0 * 2 + 1] = Lt;
        }
      }
    }
  }
}

// Merge split-K partials: one 256-thread workgroup per (token, head).  D/4 lanes hold one f32x4
// of O each; the 256 / (D/4) lane groups merge every NG-th split with an online rescale (their
// loads are independent, so a group keeps several in flight instead of one dependent round trip
// per split), then the group states merge through LDS.
template <int D>
__global__ void __launch_bounds__(256) attn_combine_kernel(AttnParams p, int T) {
  constexpr int LG = D / 4, NG = 256 / LG;
  __shared__ f32x4 so[NG][LG];
  __shared__ float sml[NG][2];
  const int th = blockIdx.x;  // t * nh + head
  const int grp = threadIdx.x / LG, l = threadIdx.x % LG;
  const size_t stride = (size_t)T * p.nh;
  float m = -1e30f, s = 0.f;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int sp = grp; sp < p.num_splits; sp += NG) {
    const size_t r = (size_t)sp * stride + th;
    const float mi = p.part_ml[r * 2], li = p.part_ml[r * 2 + 1];
    const f32x4 oi = *reinterpret_cast<const f32x4*>(p.part_o + r * D + 4 * l);
    const float mn = fmaxf(m, mi);
    const float a = __builtin_amdgcn_exp2f(m - mn), b = __builtin_amdgcn_exp2f(mi - mn);
    o = o * a + oi * b;
    s = s * a + li * b;
    m = mn;
  }
  so[grp][l] = o;
  if (l == 0) {
    sml[grp][0] = m;
    sml[grp][1] = s;
  }
  __syncthreads();
  if (grp != 0) return;
  float M = -1e30f;
#pragma unroll
  for (int g = 0; g < NG; ++g) M = fmaxf(M, sml[g][0]);
  float Lt = 0.f;
  f32x4 O = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const float f = __builtin_amdgcn_exp2f(sml[g][0] - M);
    Lt += f * sml[g][1];
    O += f * so[g][l];
  }
  const float inv = Lt > 0.f ? 1.f / Lt : 0.f;
  bf16x4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = (bf16)(O[r] * inv);
  *reinterpret_cast<bf16x4*>(p.out + (size_t)th * D + 4 * l) = v;
}

// ===========================================================================================
// Prefill (varlen, chunked) with LDS-staged K/V tiles.
//
// Workgroup = 4 waves = HPW q heads (of ONE kv head) x TPW tiles of 16 query tokens, HPW*TPW = 4
// (HPW = 4 when the GQA group allows it: the 4 waves then share every K/V tile).  Grid
// (n_tiles, nkv * G / HPW) over a host-built (sequence, tile) list — so decode rows mixed into a
// prefill batch cost one tile each — or the dense (ceil(max_q / (16 TPW)), nkv * G / HPW, B).  Per 32-key step the workgroup copies the K tile
// (32 rows x D, contiguous in the page) and the V^T tile (4 groups x D x 8, contiguous) into one of
// two LDS buffers (register-staged: the global loads of step s+1 are issued before the MFMAs of
// step s and written after them; one barrier per step).  Waves read their MFMA fragments from LDS:
//   * K rows are stored with the 16-B chunk c of row r at c ^ kswz(r), kswz(r) = (r & 3) |
//     ((r >> 3) & 3) << 2 (masked to the row's chunk count): the permuted-row A-fragment reads
//     (rows 8(i>>2) + 4t + (i&3), chunk 4c + h) then hit 16 distinct 16-B bank slots in every
//     ds_read_b128 lane group (derivation in docs/kernels.md);
//   * V^T units (group h, d) are read by 16 lanes with consecutive d: conflict-free unswizzled.
// Causality / windows / sinks use the same masks as decode; waves whose tokens are past the end of
// the chunk still join every barrier and only skip their store.
// ===========================================================================================
template <int D>
__device__ __forceinline__ int kswz(int row) {
  constexpr int CH = D / 8;  // 16-B chunks per K row
  return ((row & 3) | (((row >> 3) & 3) << 2)) & (CH - 1);
}

template <int D, bool WIN, bool FP8, int QB, bool MASK = false>
__global__ void __launch_bounds__(256, (WIN && QB == 2) ? 1 : 2) attn_prefill_kernel(AttnParams p, int hpw) {
  static_assert(!MASK || (!WIN && QB == 1), "custom masks: full cache, one query block per wave");
  // QB = 16-token query blocks per wave: every K / V fragment read from LDS feeds QB blocks'
  // MFMAs.  Measured (profiles/attn_prefill_qb_ab.json): QB = 2 is +2 % on 2k-4k chunks and -25 %
  // on 16-token ones, so QB = 1 is the default; what paid was occupancy — the 2-waves-per-SIMD
  // bound lets the QB = 1 kernel settle at ~120 VGPRs (4 workgroups per CU instead of 2):
  // 508 -> 633 TFLOP/s on a 4k causal chunk
  constexpr int CH = D / 8;            // 16-B units per K row
  constexpr int UNITS = 32 * CH;       // 16-B units per K tile (= per V^T tile)
  constexpr int UPT = (UNITS + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[2][2][32 * D];  // [buf][K | V][...]

  // work item: from the compact tile list (mixed prefill/decode batches: a 1-token decode row
  // gets one tile instead of max_q / 16 empty ones) or the dense (tile, ., sequence) grid
  int b, tile, grp;
  if (p.tile_map) {
    // 1-D grid padded to a multiple of 8; workgroup L runs on XCD L % 8 (round-robin dispatch).
    // Give every XCD one contiguous run of work items w = grp * n_tiles + t, so consecutive
    // token tiles of one (sequence, kv-head group) — which read the same K/V — share an L2.
    const int total = p.n_tiles * p.nkv * ((p.nh / p.nkv) / hpw);
    const int per = (int)gridDim.x >> 3;
    const int L = (int)blockIdx.x;
    const int w = (L & 7) * per + (L >> 3);
    if (w >= total) return;  // padding (uniform per workgroup: before any barrier)
    grp = w / p.n_tiles;
    const int t = w - grp * p.n_tiles;
    b = p.tile_map[2 * t];
    tile = p.tile_map[2 * t + 1];
  } else {
    b = blockIdx.z;
    tile = blockIdx.x;
    grp = blockIdx.y;
  }
  const int G = p.nh / p.nkv;
  const int tpw = 4 / hpw;
  const int wgs_per_kv = G / hpw;
  const int kvh = grp / wgs_per_kv;
  const int h0 = kvh * G + (grp % wgs_per_kv) * hpw;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, h4 = lane >> 4;
  const int qh = h0 + (w % hpw);
  const int qs0 = p.q_start[b];
  const int qlen = p.q_start[b + 1] - qs0;
  const int wg_tok0 = tile * 16 * tpw * QB;
  if (wg_tok0 >= qlen) return;  // whole workgroup idle (uniform: before any barrier)
  const int tok0 = wg_tok0 + (w / hpw) * 16 * QB;
  const int L = p.seq_lens[b];
  int tok[QB], pq[QB];
  bool col_valid[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    tok[qb] = tok0 + 16 * qb + col;
    col_valid[qb] = tok[qb] < qlen;
    pq[qb] = L - qlen + (col_valid[qb] ? tok[qb] : qlen - 1);  // the column's absolute position
  }
  const int pq_max = L - qlen + min(qlen - 1, wg_tok0 + 16 * tpw * QB - 1);  // workgroup's last token
  const int* bt = p.block_tables + (size_t)b * p.bt_stride;
  const size_t head_stride = (size_t)p.bs * D;

  bf16x8 qf[QB][D / 32], qsf[WIN ? QB : 1][D / 32];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const size_t qoff = ((size_t)(qs0 + (col_valid[qb] ? tok[qb] : 0)) * p.nh + qh) * D;
#pragma unroll
    for (int c = 0; c < D / 32; ++c) {
      qf[qb][c] = col_valid[qb] ? *reinterpret_cast<const bf16x8*>(p.q + qoff + 32 * c + 8 * h4)
                                : zero8();
      if constexpr (WIN)
        qsf[qb][c] = (p.n_sink > 0 && col_valid[qb])
                         ? *reinterpret_cast<const bf16x8*>(p.q_sink + qoff + 32 * c + 8 * h4) : zero8();
    }
  }

  // virtual steps: [0, n_main) = full cache / ring segment, [n_main, n_main + n_sinkst) = sinks
  int seg_len, n_main, n_sinkst = 0, nS = 0;
  if (WIN) {
    seg_len = L > p.n_sink ? min(p.ring, L - p.n_sink) : 0;
    n_main = (seg_len + 31) >> 5;
    nS = min(p.n_sink, L);
    n_sinkst = (nS + 31) >> 5;
  } else {
    // causal: keys up to the workgroup's last query; a custom mask may open any key < L
    seg_len = MASK ? L : pq_max + 1;
    n_main = (seg_len + 31) >> 5;
  }
  const int nsteps = n_main + n_sinkst;
  // custom additive mask row of this lane's query, pre-divided by the softmax scale because the
  // scores are scaled inside the exponent.  Entries <= -1e4 (-inf, finfo.min, -1e9 ...) mask the
  // key outright: exp(-1e4) is 0 in fp32 next to any live score, and keeping such magnitudes out
  // of the exponent's FMA avoids its rounding residual (half an ulp of ~1e38 is ~1e31).  A row
  // with no live key outputs zeros (the reference's fp32 softmax over finfo.min would average V;
  // such rows are padding, ops/reference.py attn_custom_mask defines them the same way).
  const float* mrow = nullptr;
  float minv = 0.f;
  int mlen = 0;   // keys [0, mlen) have a mask column (bounds of the caller's tensor)
  if constexpr (MASK) {
    const int hsel = p.mask_heads == 1 ? 0 : qh;
    const int mr = p.mask_q - qlen + (col_valid[0] ? tok[0] : qlen - 1);
    mlen = mr >= 0 ? min(L, p.mask_k) : 0;   // a row outside the mask: every key masked
    mrow = p.mask + (((size_t)b * p.mask_heads + hsel) * p.mask_q + max(mr, 0)) * p.mask_k;
    minv = 1.4426950408889634f / p.scale_log2;   // 1 / scale
  }
  auto slot0 = [&](int sidx) -> int {  // first cache slot of virtual step sidx
    if (!WIN) return sidx * 32;
    return sidx < n_main ? p.sink_pad + sidx * 32 : (sidx - n_main) * 32;
  };

  typedef int i32x4v __attribute__((ext_vector_type(4)));
  // bf16 caches: K / V^T tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4: LDS slot =
  // wave base + 16 lane, so the K swizzle is applied to the per-lane GLOBAL chunk instead); no
  // staging registers or ds_writes, ~16 fewer VGPRs.  fp8 caches stage through registers: the
  // 8-byte units are widened to bf16 on the way into LDS.
  constexpr bool DMA = !FP8 && UNITS % 256 == 0;
  auto dma = [&](int sidx, int buf) {
    const int u0 = slot0(sidx);
    const int page = bt[u0 / p.bs];
    const int offk = u0 % p.bs;
    const size_t e0 = ((size_t)page * p.nkv + kvh) * head_stride + (size_t)offk * D;
    const bf16* kg = static_cast<const bf16*>(p.k_cache) + e0;
    const bf16* vg = static_cast<const bf16*>(p.v_cache) + e0;
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int u = threadIdx.x + i * 256;
      const int row = u / CH, slot = u % CH;
      // LDS unit u = (row, slot) holds global chunk slot ^ kswz(row)
      __builtin_amdgcn_global_load_lds(
          (__attribute__((address_space(1))) void*)(kg + (row * CH + (slot ^ kswz<D>(row))) * 8),
          (__attribute__((address_space(3))) void*)&smem[buf][0][(w * 64 + i * 256) * 8], 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (__attribute__((address_space(1))) void*)(vg + (size_t)u * 8),
          (__attribute__((address_space(3))) void*)&smem[buf][1][(w * 64 + i * 256) * 8], 16, 0, 0);
    }
  };
  // staging registers: one 8-element unit per tile unit (16 B bf16, or 8 B fp8 widened to bf16
  // when written to LDS, so the LDS tiles and everything after them are bf16 either way)
  typedef typename std::conditional<FP8, uint2, i32x4v>::type Unit;
  Unit rk[DMA ? 1 : UPT], rv[DMA ? 1 : UPT];
  auto gload = [&](int sidx) {
    const int u0 = slot0(sidx);
    const int page = bt[u0 / p.bs];
    const int offk = u0 % p.bs;
    // 32 K rows x D and 4 V^T groups x D x 8, both contiguous from element offset `e0`
    const size_t e0 = ((size_t)page * p.nkv + kvh) * head_stride + (size_t)offk * D;
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int u = threadIdx.x + i * 256;
      if (UNITS % 256 == 0 || u < UNITS) {
        if constexpr (FP8) {
          rk[i] = *reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(p.k_cache) + e0 + (size_t)u * 8);
          rv[i] = *reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(p.v_cache) + e0 + (size_t)u * 8);
        } else {
          rk[i] = *reinterpret_cast<const i32x4v*>(static_cast<const bf16*>(p.k_cache) + e0 + (size_t)u * 8);
          rv[i] = *reinterpret_cast<const i32x4v*>(static_cast<const bf16*>(p.v_cache) + e0 + (size_t)u * 8);
        }
      }
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int u = threadIdx.x + i * 256;
      if (UNITS % 256 == 0 || u < UNITS) {
        const int row = u / CH, ch = u % CH;
        bf16x8* kd = reinterpret_cast<bf16x8*>(&smem[buf][0][(row * CH + (ch ^ kswz<D>(row))) * 8]);
        bf16x8* vd = reinterpret_cast<bf16x8*>(&smem[buf][1][u * 8]);
        if constexpr (FP8) {
          *kd = fp8x8_to_bf16x8(rk[i]);
          *vd = fp8x8_to_bf16x8(rv[i]);
        } else {
          *kd = __builtin_bit_cast(bf16x8, rk[i]);
          *vd = __builtin_bit_cast(bf16x8, rv[i]);
        }
      }
    }
  };
  const float sl2 = FP8 ? p.scale_log2 * p.k_scale : p.scale_log2;
  const float vsc = FP8 ? p.v_scale : 1.f;

  WaveState<D> st[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) st[qb].init();
  if (nsteps > 0) {
    if constexpr (DMA) {
      dma(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      gload(0);
      swrite(0);
    }
  }
  __syncthreads();
  for (int sidx = 0; sidx < nsteps; ++sidx) {
    const int buf = sidx & 1;
    if (sidx + 1 < nsteps) {
      if constexpr (DMA) dma(sidx + 1, buf ^ 1);   // buf ^ 1 was last read before the barrier
      else gload(sidx + 1);
    }
    // ---- fragments from LDS ----
    KVFrag<D> f;
    const int krow0 = 8 * (col >> 2) + (col & 3);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = krow0 + 4 * t;
#pragma unroll
      for (int c = 0; c < D / 32; ++c)
        f.k[t][c] = *reinterpret_cast<const bf16x8*>(
            &smem[buf][0][(row * CH + ((4 * c + h4) ^ kswz<D>(row))) * 8]);
    }
#pragma unroll
    for (int e = 0; e < D / 16; ++e)
      f.v[e] = *reinterpret_cast<const bf16x8*>(&smem[buf][1][(h4 * D + 16 * e + col) * 8]);
    // ---- visibility of keys 8h4 .. 8h4+7 for this lane's query column, per query block ----
    const int u0 = slot0(sidx);
    const bool sink_step = WIN && sidx >= n_main;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      if constexpr (MASK) {
        // keys 8h4 + j < L are candidates; the mask decides (its -inf / finfo.min entries drop out)
        const int k0 = u0 + 8 * h4;
        float madd[8];
        unsigned vis = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float mv = k0 + j < mlen ? mrow[k0 + j] : -INFINITY;
          const bool ok = mv > -1e4f;
          madd[j] = ok ? mv * minv : 0.f;
          vis |= (ok ? 1u : 0u) << j;
        }
        attn_core<D>(st[qb], qf[qb], f, sl2, [&](int j) { return ((vis >> j) & 1u) != 0; },
                     [&](int j) { return madd[j]; });
        continue;
      }
      if constexpr (!WIN) {
        attn_compute_causal<D>(st[qb], qf[qb], f, sl2, pq[qb] - (u0 + 8 * h4));
        continue;
      }
      unsigned vm = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int u = u0 + 8 * h4 + j;
        bool ok;
        if (!WIN) {
          ok = u <= pq[qb];
        } else if (sink_step) {
          ok = u < nS && u <= pq[qb];
        } else {
          ok = (u - p.sink_pad) < seg_len;
          if (ok) {
            const int a = ring_abs(u, L, p);
            ok = a >= p.n_sink && a <= pq[qb] && (pq[qb] - a) < (p.window - p.n_sink);
          }
        }
        vm |= (ok ? 1u : 0u) << j;
      }
      if constexpr (WIN) {
        if (sink_step) {
          attn_compute<D>(st[qb], qsf[qb], f, sl2, vm);
          continue;
        }
      }
      attn_compute<D>(st[qb], qf[qb], f, sl2, vm);
    }
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of step s+1 landed
    } else {
      if (sidx + 1 < nsteps) swrite(buf ^ 1);
    }
    __syncthreads();
  }
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    float lsum = st[qb].l;
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    if (col_valid[qb]) {
      const float inv = lsum > 0.f ? vsc / lsum : 0.f;
      bf16* orow = p.out + ((size_t)(qs0 + tok[qb]) * p.nh + qh) * D;
#pragma unroll
      for (int e = 0; e < D / 16; ++e) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(st[qb].o[e][r] * inv);
        *reinterpret_cast<bf16x4*>(orow + 16 * e + 4 * h4) = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
static int attn_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return 256;
    return n;
  }();
  return cus;
}

template <int D, bool WIN, bool FP8>
static void decode_grid(const AttnParams& p, int items, int gs, hipStream_t stream) {
  const int grid = (items + 3) / 4;
  if (p.num_splits > 1) {
    attn_decode_kernel<D, WIN, FP8, true><<<grid, 256, 0, stream>>>(p, items, gs);
    return;
  }
  if constexpr (!WIN) {
#ifndef ATTN_DECODE_TWO_STEP   // experiment builds: the round-4 loop at every batch
    // one-step when it fills every SIMD with 4 waves and its last round is no emptier than the
    // two-step loop's (B = 768: 6144 waves are 1.5 rounds of 4096 but 3 full rounds of 2048 --
    // one-step measured 358 vs 342 us there)
    const long s1 = 16L * attn_cus(), s2 = 8L * attn_cus();
    const long r1 = (items + s1 - 1) / s1, r2 = (items + s2 - 1) / s2;
    if (items >= s1 && (double)items / (r1 * s1) >= (double)items / (r2 * s2)) {
      attn_decode_kernel<D, WIN, FP8, false, true><<<grid, 256, 0, stream>>>(p, items, 1);
      return;
    }
#endif
  }
  attn_decode_kernel<D, WIN, FP8, false><<<grid, 256, 0, stream>>>(p, items, 1);
}

template <int D>
static int launch_decode_d(const AttnParams& p, int B, hipStream_t stream) {
  const int G = p.nh / p.nkv;
  const int hgroups = (G + 15) / 16;
  const long items = (long)B * p.nkv * hgroups * p.num_splits;
  if (items > (1L << 30)) return -3;
  // splits merged inside a workgroup (its 4 waves hold consecutive splits of one item)
  const int gs = p.num_splits % 4 == 0 ? 4 : p.num_splits % 2 == 0 ? 2 : 1;
  if (p.ring > 0) {
    if (p.kv_fp8) decode_grid<D, true, true>(p, (int)items, gs, stream);
    else decode_grid<D, true, false>(p, (int)items, gs, stream);
  } else {
    if (p.kv_fp8) decode_grid<D, false, true>(p, (int)items, gs, stream);
    else decode_grid<D, false, false>(p, (int)items, gs, stream);
  }
  if (p.num_splits > gs) {
    AttnParams pc = p;
    pc.num_splits = p.num_splits / gs;
    attn_combine_kernel<D><<<B * p.nh, 256, 0, stream>>>(pc, B);
  }
  return 0;
}

int launch_attn_decode(const AttnParams& p, int B, int D, hipStream_t stream) {
  if (B == 0) return 0;
  if (p.bs % 32 != 0 || (p.ring > 0 && (p.sink_pad % 32 != 0 || p.ring % 32 != 0))) return -2;
  switch (D) {
    case 32: return launch_decode_d<32>(p, B, stream);
    case 64: return launch_decode_d<64>(p, B, stream);
    case 128: return launch_decode_d<128>(p, B, stream);
    default: return -1;
  }
}

template <int D, bool WIN, bool FP8>
static void prefill_grid(const AttnParams& p, dim3 grid, int hpw, hipStream_t stream) {
  if constexpr (!WIN) {
    if (p.mask) {   // reference 4-D additive mask (rare): one query block per wave
      attn_prefill_kernel<D, false, FP8, 1, true><<<grid, 256, 0, stream>>>(p, hpw);
      return;
    }
  }
  if (p.prefill_qb == 2)
    attn_prefill_kernel<D, WIN, FP8, 2><<<grid, 256, 0, stream>>>(p, hpw);
  else
    attn_prefill_kernel<D, WIN, FP8, 1><<<grid, 256, 0, stream>>>(p, hpw);
}

template <int D>
static int launch_prefill_d(const AttnParams& p, int B, int max_q, hipStream_t stream) {
  const int G = p.nh / p.nkv;
  const int hpw = (G % 4 == 0) ? 4 : (G % 2 == 0 ? 2 : 1);  // q heads sharing each K/V tile
  const int tpw = 4 / hpw;
  const int tt = 16 * tpw * (p.mask ? 1 : p.prefill_qb);      // query tokens per workgroup tile
  dim3 grid((max_q + tt - 1) / tt, p.nkv * (G / hpw), B);
  if (p.tile_map) {
    // XCD-aware 1-D grid over (group, tile) work items (see attn_prefill_kernel)
    const long total = (long)p.n_tiles * p.nkv * (G / hpw);
    grid = dim3((unsigned)((total + 7) / 8 * 8), 1, 1);
  }
  if (grid.x == 0) return 0;
  if (p.ring > 0) {
    if (p.kv_fp8) prefill_grid<D, true, true>(p, grid, hpw, stream);
    else prefill_grid<D, true, false>(p, grid, hpw, stream);
  } else {
    if (p.kv_fp8) prefill_grid<D, false, true>(p, grid, hpw, stream);
    else prefill_grid<D, false, false>(p, grid, hpw, stream);
  }
  return 0;
}

int launch_attn_prefill(const AttnParams& p, int B, int max_q, int D, hipStream_t stream) {
  if (B == 0 || max_q == 0) return 0;
  if (p.prefill_qb != 1 && p.prefill_qb != 2) return -3;
  if (p.bs % 32 != 0 || (p.ring > 0 && (p.sink_pad % 32 != 0 || p.ring % 32 != 0))) return -2;
  if (p.mask && (p.ring > 0 || p.tile_map || p.mask_heads < 1 || p.mask_q < 1 || p.mask_k < 1))
    return -4;   // custom masks: full cache, dense grid
  if (attn_prefill32_eligible(p, D)) return launch_attn_prefill32(p, B, max_q, stream);
  switch (D) {
    case 32: return launch_prefill_d<32>(p, B, max_q, stream);
    case 64: return launch_prefill_d<64>(p, B, max_q, stream);
    case 128: return launch_prefill_d<128>(p, B, max_q, stream);
    default: return -1;
  }
}

}  // namespace dli
