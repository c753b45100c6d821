// Causal prefill attention on the 32x32x16 bf16 MFMA: 32 query rows per wave, 64-key steps.
//
// Replaces the reference's eager prefill attention (modules.py:87-97: repeat_kv, QK^T/sqrt(D) +
// additive causal mask, fp32 softmax, PV) and its sink-cache window (cache.py) for head_dim 128:
// any GQA group incl. MHA, full caches and windowed rings (sliding windows, StreamingLLM sinks),
// bf16 or fp8 KV.  attention.hip keeps the rest (custom 4-D masks, other head sizes, short
// chunks of groups that are not a multiple of 4).
//
// Why a second kernel: attention.hip's prefill wave holds 16 query rows on the 16x16x32 MFMA, so
// every K / V^T fragment read from LDS (one ds_read_b128) feeds ONE 16-cycle MFMA: four SIMDs ask
// the LDS for 4 KB per 16 cycles = its whole 256 B/clk, and the loop sat at 0.7 PF on 4k-token
// chunks.  Here a wave holds 32 query rows on the 32x32x16 MFMA (32 cycles per fragment read):
// half the LDS bytes per FLOP, and 64-key steps halve the barriers and online-softmax rescales
// per FLOP (MI355X_MICROARCH.md "LDS"; cdna_hip_programming.md Appendix B "Fused attention
// prefill").
//
// Layout of one workgroup = GW q heads of ONE kv head (GW = 8 or 4; 2 or 1 for groups that are
// not a multiple of 4) x TQ query tokens (32, or 16 for short chunks; 64 / 32 for GW = 2, 128 / 64
// for GW = 1), NW = GW * TQ / 32 waves; row R = 32 w + c of the workgroup is token R % TQ of head
// R / TQ.  All waves share every K / V^T tile (GQA-native, no repeat_kv).
//   * S^T[key, q] = K[key, d] . Q^T[d, q] (A = K rows from LDS, B = Q^T in registers): lane
//     (c = l & 31, h = l >> 5) ends holding column c and accumulator rows (r&3) + 8(r>>2) + 4h.
//     The K tile's LDS row i holds key pi(i) = i with bits 2 and 3 swapped, so register r of lane
//     half h holds key 16(r>>3) + 8h + (r&7): registers 8s..8s+7, packed to bf16, ARE the P^T
//     operand of k-step s of the next product (keys 16s + 8h + j), with no lane movement
//     (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
//   * O^T[d, q] += V^T[d, key] . P^T[key, q]: the cache's V^T 8-key groups [g][d][8] give lane
//     (d, h) of k-step s group 2s + h as ONE 16-byte LDS read.
//   * K rows are stored with 16-byte chunk c at c ^ (row & 15): the row reads of one ds_read_b128
//     lane group (rows {0-3, 12-15, 20-27} or {4-11, 16-19, 28-31}, one chunk) then hit 16
//     distinct bank slots; the V^T reads (consecutive d) are conflict-free as stored.
//   * K / V^T tiles (2 x 16 KB of bf16 per step) go global -> LDS by LDS-DMA (fp8 caches: through
//     registers, widened to bf16 on the way) into two buffers (three for staggered workgroups):
//     the next step's fetch is issued behind this step's first MFMAs, one barrier per step.
//   * online softmax in the log2 domain with a deferred max (cdna_hip_programming.md T13): the
//     running max (and the O / l rescale) moves only when some column's max grew by more than
//     THR = 8, so P <= 2^8 (exact-scale fp32 accumulation; bf16 P keeps its relative precision).
//   * causality and windows from seq_lens / q_start / ring geometry (no mask tensor): steps run
//     from the first one holding a key inside some column's window; steps entirely inside every
//     column's window skip the mask; the half of a diagonal step past every column's position
//     skips its MFMAs.
//   * work list: the (sequence, tile) map of attention.hip walked heaviest tile first (the
//     causal tail), XCD-grouped so consecutive tiles of one kv head share an L2.  (A persistent
//     form for 4-wave workgroups, P32_PERSIST, walks several tiles with the next tile's Q and
//     first step in flight during the stores: measured, off.)
//   * counted LDS waits: K / V^T fragment reads issued ahead of their MFMAs, the DMA in its
//     buffer form (docs/kernels.md "Second pass"); output staged through LDS, stored as rows.
#include "kernels.h"
#include "attn_core.h"

#include <algorithm>
#include <type_traits>

namespace dli {

namespace {

constexpr int P32_D = 128;
constexpr float P32_THR = 8.f;   // deferred-max threshold (log2 domain)
#ifndef P32_STAGGER
#define P32_STAGGER 1   // 0: every wave runs S | softmax | PV in the same order
#endif
#ifndef P32_PERSIST
// 1: 4-wave workgroups persistent (two per CU), the next tile's Q and first K / V^T step
// fetched while this tile's output is stored.  Measured off: 512-token prompts 486 vs 496 TF,
// 4k 946 vs 984 (profiles/r6/prefill32b/r6p32j_*) - two co-resident workgroups per CU already
// overlap one tile's Q / O traffic with another's steps, and the dispatcher balances better.
#define P32_PERSIST 0
#endif
// knock-out probes (wrong results; scripts/prefill_so_ab.sh arms, docs/kernels.md)
#ifndef P32_KO_PAGES
#define P32_KO_PAGES 0   // block table read as identity
#endif
#ifndef P32_KO_Q
#define P32_KO_Q 0       // no Q load
#endif
#ifndef P32_KO_OUT
#define P32_KO_OUT 0     // no output stores
#endif
#ifndef P32_KO_LOOP
#define P32_KO_LOOP 0    // one key step per tile
#endif

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// max over lanes l and l ^ 32: v_permlane32_swap of two copies leaves each lane both halves
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return __builtin_elementwise_maximum(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ int swap23(int i) {   // pi: swap bits 2 and 3 of a 32-row index
  return (i & ~0xC) | ((i & 4) << 1) | ((i & 8) >> 1);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& s, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)s[base + j];
  return r;
}

}  // namespace

template <int TQ, int GW, bool F8, bool WIN>
__global__ void __launch_bounds__(512, 2) attn_prefill32_kernel(AttnParams p) {
  constexpr int D = P32_D;
  constexpr int CH = D / 8;                 // 16-B chunks per K row
  constexpr int NW = GW * TQ / 32;          // waves per workgroup
  // staggered waves (8-wave workgroups, one per CU) keep V(s-1) while step s+1 lands: 3 buffers
  // (not in window mode: the staggered half's S(s-1) held across the barrier next to the window
  // arithmetic would spill)
  constexpr bool STAG = P32_STAGGER && NW == 8 && !WIN;
  constexpr int NBUF = STAG ? 3 : 2;
  // persistent, with the next tile's Q / first step fetched during the stores (4-wave tiles)
  constexpr bool PF = P32_PERSIST && NW < 8;
  // [buf][K | V^T][64 keys x D]: NBUF x 2 x 16 KB
  __shared__ __attribute__((aligned(16))) bf16 smem[NBUF][2][64 * D];

  const int G = p.nh / p.nkv;
  const int wg_per_kv = G / GW;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 31, hh = lane >> 5;
  const int R = 32 * w + c;
  const size_t head_stride = (size_t)p.bs * D;
  const int bs_lg = __builtin_ctz(p.bs);
  const uint32_t page_elems = (uint32_t)p.nkv * (uint32_t)head_stride;

  // ---- work items.  With a tile map the grid is 8 x `per` workgroups, XCD-major: XCD x
  // (= blockIdx & 7) owns items [x span, (x+1) span) - one kv-head group's tiles, heaviest
  // first - and its k-th workgroup takes one of them (per = span), or, persistent, a snake walk
  // over them (below).  Without a map (dense grid) a workgroup is one (sequence, tile, group).
  struct Item {
    int b, t0, kvh, h0, qs0, qlen, L, pq_lo, pq_hi, ns, s_lo, nsteps;
    const int* bt;
  };
  // Windowed ring caches (p.ring > 0): nsk sink tokens in slots [0, nsk) (StreamingLLM; none for
  // Mistral's sliding window) and the rolling keys a >= nsk in slot sink_pad + (a - nsk) % ring
  // (ring >= window - nsk + the longest chunk - 1, so every key a chunk's queries see is still
  // there).  A rolling key is visible to the column at position q iff q - wmain < a <= q; the
  // sinks (a < min(nsk, L)) are visible to every column at or past them and score against the
  // query rotated for them (q_sink): one extra step, first.  Main steps are aligned in the
  // ring's offset a - nsk, so each 32-key half is one run of slots.  win = 0: full cache.
  // (a template flag: the window / sink arithmetic costs the full-cache kernels registers)
  const int win = WIN ? p.window : 0;
  const int nsk = WIN ? p.n_sink : 0;
  const int wmain = win - nsk;
  // Persistent walk: round n takes item n per + k on even rounds and n per + (per - 1 - k) on odd
  // ones (a snake): the map lists each sequence's tiles heaviest first, so a plain stride that
  // is a multiple of the tiles per sequence would hand one workgroup every sequence's heaviest
  // tile and another every lightest.
  int x0 = 0, k0 = 0, per = 1, span = 1, wi_end = 1, n = 0;
  if (p.tile_map) {
    const int total = p.n_tiles * p.nkv * wg_per_kv;
    per = (int)gridDim.x >> 3;
    span = (total + 7) >> 3;
    x0 = ((int)blockIdx.x & 7) * span;
    k0 = (int)blockIdx.x >> 3;
    wi_end = min(total, x0 + span);
  }
  auto item_of = [&](int n_) { return x0 + n_ * per + ((n_ & 1) ? per - 1 - k0 : k0); };
  int wi = item_of(0);
  auto decode = [&](int wi_, Item& it) {   // false: an empty tile (dense grids only)
    int b, tile, grp;
    if (p.tile_map) {
      grp = wi_ / p.n_tiles;
      const int t = p.n_tiles - 1 - (wi_ - grp * p.n_tiles);   // heaviest (last) tiles first
      b = p.tile_map[2 * t];
      tile = p.tile_map[2 * t + 1];
    } else {
      b = blockIdx.z;
      tile = gridDim.x - 1 - blockIdx.x;
      grp = blockIdx.y;
    }
    it.b = b;
    it.kvh = grp / wg_per_kv;
    it.h0 = it.kvh * G + (grp % wg_per_kv) * GW;
    it.qs0 = p.q_start[b];
    it.qlen = p.q_start[b + 1] - it.qs0;
    it.t0 = tile * TQ;
    it.L = p.seq_lens[b];
    it.pq_lo = it.L - it.qlen + it.t0;                                  // first position
    it.pq_hi = it.L - it.qlen + min(it.qlen - 1, it.t0 + TQ - 1);      // ... and last
    it.ns = nsk > 0 ? 1 : 0;                                            // the sink step
    it.s_lo = win ? max(0, it.pq_lo - wmain + 1 - nsk) >> 6 : 0;       // first main step (offset)
    const int o_hi = it.pq_hi - nsk;                                    // ... through pq_hi
#if P32_KO_LOOP
    it.nsteps = 1;
#else
    it.nsteps = it.ns + (o_hi >= 0 ? (o_hi >> 6) - it.s_lo + 1 : 0);
#endif
    it.bt = p.block_tables + (size_t)b * p.bt_stride;
    return it.t0 < it.qlen;
  };
  if (wi >= wi_end) return;                 // padding (whole workgroup, before any barrier)
  Item cur;
  if (!decode(wi, cur)) return;             // whole workgroup idle (dense grid)

  // ---- Q^T operand: lane (c, hh) holds d = 16 m + 8 hh + [0, 8) of its column, m = 0..7 ----
  // (rows past the chunk load the chunk's first token - always present - and are zeroed)
  auto load_q = [&](const Item& it, bf16x8 (&q)[D / 16], const bf16* src) {
    const int tok = it.t0 + R % TQ;
    const bool valid = tok < it.qlen;
    const bf16* qrow =
        src + ((size_t)(it.qs0 + (valid ? tok : 0)) * p.nh + it.h0 + R / TQ) * D + 8 * hh;
#pragma unroll
    for (int m = 0; m < D / 16; ++m) {
#if P32_KO_Q
      q[m] = zero8(); (void)qrow;
#else
      q[m] = *reinterpret_cast<const bf16x8*>(qrow + 16 * m);
      if (!valid) q[m] = zero8();
#endif
    }
  };

  auto bufi = [&](int g) { return NBUF == 2 ? (g & 1) : (g % 3); };
  auto kbuf = [&](int i) { return &smem[i][0][0]; };
  auto vbuf = [&](int i) { return &smem[i][1][0]; };
  // per-lane byte offsets of the LDS-DMA pieces: they depend only on the piece index
  constexpr int NPC = 16 / NW;              // pieces per image per wave and step
  int kvo[NPC], vvo[NPC];
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int u = (w + i * NW) * 64 + lane;  // 16-B unit of this lane in the 16 KB image
    const int row = u >> 4, slot = u & 15;   // K: LDS row (0..63), stored chunk
    kvo[i] = (swap23(row & 31) * D + 8 * (slot ^ (row & 15))) * 2;   // key pi(row) of its half
    vvo[i] = (u & 511) * 16;
  }
  // one 1 KB piece: the resource starts at the half's first key in the kv head's slice of the
  // page (its offset folded into the base: this compiler drops the host-side kernel stubs -
  // silently, a broken object - when the builtin's soffset is a runtime value or the resource is
  // built inline in the call)
  auto piece = [&](const void* cache, int kvh, int pg, int half_off, bf16* dst, int vo) {
    const bf16* base = static_cast<const bf16*>(cache) + (size_t)kvh * head_stride +
                       (size_t)(uint32_t)pg * page_elems + half_off;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                             vo, 0, 0, 0);
  };
  // ---- LDS-DMA of step s of tile `it` into buffer bi: K and V^T images (16 wave-instructions of
  // 1 KB each per image, NPC per wave).  Piece i of wave w is instruction j = w + i NW: K rows
  // 4j..4j+3 / V^T units 64j..64j+63, its 32-key half (j >> 3 = i NW >> 3) known at compile time.
  // A half past every column is never fetched (its block-table entry may not exist).
  // buffer_load ... lds rather than global_load_lds: the compiler's wait model treats the global
  // form as an out-of-order LDS (lgkm) access, which turns every LDS-read wait after it into
  // lgkmcnt(0).  Block size a power of two: shifts, not divisions; both halves' pages by one pair
  // of scalar loads waited once per step.
  // fp8 e4m3 caches: no LDS-DMA - each lane loads 16-byte runs of fp8 (two bf16 units' worth)
  // into registers when the DMA would be issued, and widens them into the same bf16 LDS images
  // just before the step barrier (f8_commit), so the MFMA loop is the bf16 one; K's scale folds
  // into the softmax scale, V's into the output normalisation
  constexpr int NPU = 8 / NW;               // 16-B fp8 runs per image per lane and step
  uint4 rk[F8 ? NPU : 1], rv[F8 ? NPU : 1];
  int f8_bi = 0;
  bool f8_need1 = false;
  auto f8_commit = [&]() {
    bf16* kd = kbuf(f8_bi);
    bf16* vd = vbuf(f8_bi);
#pragma unroll
    for (int i = 0; i < NPU; ++i) {
      const int pu = (i * NW + w) * 64 + lane;
      if (((i * NW + w) >> 2) && !f8_need1) continue;   // (the K and the V^T run: same half)
      const int row = pu >> 3, kk = pu & 7;
      bf16* krow = kd + row * CH * 8;
      *reinterpret_cast<bf16x8*>(krow + ((2 * kk) ^ (row & 15)) * 8) =
          fp8x8_to_bf16x8(make_uint2(rk[i].x, rk[i].y));
      *reinterpret_cast<bf16x8*>(krow + ((2 * kk + 1) ^ (row & 15)) * 8) =
          fp8x8_to_bf16x8(make_uint2(rk[i].z, rk[i].w));
      *reinterpret_cast<bf16x8*>(vd + (2 * pu) * 8) =
          fp8x8_to_bf16x8(make_uint2(rv[i].x, rv[i].y));
      *reinterpret_cast<bf16x8*>(vd + (2 * pu + 1) * 8) =
          fp8x8_to_bf16x8(make_uint2(rv[i].z, rv[i].w));
    }
  };
  auto dma_step = [&](const Item& it, int s, int bi) {
    const bool sink = s < it.ns;
    const int o0 = (it.s_lo + s - it.ns) * 64;   // main step: ring offset of its first key
    const int u0 = sink ? 0 : nsk + o0;          // absolute position of the step's first key
    const bool need1 = sink ? min(nsk, it.L) > 32 && it.pq_hi >= 32 : u0 + 32 <= it.pq_hi;
    int sl0 = u0, sl1 = u0 + 32;                 // cache slots of the two halves
    if (win && !sink) {
      sl0 = p.sink_pad + o0 % p.ring;
      sl1 = p.sink_pad + (o0 + 32) % p.ring;
    }
    const int i0 = sl0 >> bs_lg;
    const int i1 = need1 ? sl1 >> bs_lg : i0;
    const int* a0 = it.bt + __builtin_amdgcn_readfirstlane(i0);
    const int* a1 = it.bt + __builtin_amdgcn_readfirstlane(i1);
    int pg0, pg1;
#if P32_KO_PAGES
    pg0 = i0; pg1 = i1; (void)a0; (void)a1;
    if (false)
#endif
    asm volatile("s_load_dword %0, %2, 0x0\n\ts_load_dword %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(pg0), "=&s"(pg1) : "s"(a0), "s"(a1));
    const int so0 = (sl0 & (p.bs - 1)) * D;         // the halves' element offsets in their pages
    const int so1 = (sl1 & (p.bs - 1)) * D;
    if constexpr (F8) {
      f8_bi = bi;
      f8_need1 = need1;
      const size_t kvb = (size_t)it.kvh * head_stride;
      const size_t e0 = kvb + (size_t)(uint32_t)pg0 * page_elems + so0;   // bytes = elements
      const size_t e1 = kvb + (size_t)(uint32_t)pg1 * page_elems + so1;
      const uint8_t* kh0 = static_cast<const uint8_t*>(p.k_cache) + e0;
      const uint8_t* kh1 = static_cast<const uint8_t*>(p.k_cache) + e1;
      const uint8_t* vh0 = static_cast<const uint8_t*>(p.v_cache) + e0;
      const uint8_t* vh1 = static_cast<const uint8_t*>(p.v_cache) + e1;
#pragma unroll
      for (int i = 0; i < NPU; ++i) {
        const int pu = (i * NW + w) * 64 + lane;
        const int half = (i * NW + w) >> 2;           // wave-uniform
        if (half && !need1) continue;
        const int row = pu >> 3, kk = pu & 7;         // K: LDS row, 16-d run; key pi(row)
        rk[i] = *reinterpret_cast<const uint4*>((half ? kh1 : kh0) + swap23(row & 31) * D +
                                                16 * kk);
        const int u2 = (2 * pu) & 511;                // V^T: units (g, d), (g, d+1) of the half
        rv[i] = *reinterpret_cast<const uint4*>((half ? vh1 : vh0) + u2 * 8);
      }
      return;
    }
    bf16* kd = kbuf(bi);
    bf16* vd = vbuf(bi);
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      const int half = (i * NW) >> 3;
      if (half && !need1) continue;
      const int j = w + i * NW;
      const int pg = half ? pg1 : pg0;
      piece(p.k_cache, it.kvh, pg, half ? so1 : so0, kd + j * 64 * 8, kvo[i]);
      piece(p.v_cache, it.kvh, pg, half ? so1 : so0, vd + j * 64 * 8, vvo[i]);
    }
  };

  // LDS fragment offsets (elements): K row c (half 0) chunk (2m + hh) ^ (c & 15); V^T unit (g, d)
  const int koff = c * CH * 8;
  const int kx = c & 15;
  const int voff = (hh * D + c) * 8;
  const float sl2 = F8 ? p.scale_log2 * p.k_scale : p.scale_log2;

  bf16x8 qf[D / 16];
  load_q(cur, qf, cur.ns ? p.q_sink : p.q);   // (the sink step scores against q_sink)
  int g0 = 0;                               // global step count: buffer of (tile, step s) = g0 + s
  dma_step(cur, 0, bufi(0));
  if constexpr (F8) f8_commit();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (;;) {
    // ---- one tile ----
    const int nsteps = cur.nsteps;
    const int pq_lo = cur.pq_lo, pq_hi = cur.pq_hi;
    const int tok = cur.t0 + R % TQ;
    const int pq = cur.L - cur.qlen + (tok < cur.qlen ? tok : cur.qlen - 1);   // column position

    f32x16 o[D / 32];
#pragma unroll
    for (int db = 0; db < D / 32; ++db) o[db] = f32x16{};
    float l_run = 0.f;
    float m_run = -1e30f;
    const int ns = cur.ns;
    const int nS = min(nsk, cur.L);         // sink keys present
    const int kb0 = nsk + (cur.s_lo - ns) * 64;   // absolute position of step s's first key:
    auto akey = [&](int s) { return s < ns ? 0 : kb0 + s * 64; };   //  kb0 + 64 s (main steps)
    auto full2 = [&](int s) {               // the second half holds a visible key
      return s < ns ? nS > 32 && pq_hi >= 32 : akey(s) + 32 <= pq_hi;
    };
    auto diag = [&](int s) { return s < ns || akey(s) + 63 > pq_lo; };   // some key masked:
    auto low = [&](int s) {                 //  past some column, or before some column's window
      return win && akey(s) < pq_hi - wmain + 1;
    };
    // S^T(s) from K(s): the first half's 8 fragment reads all issued before the first MFMA, then
    // one second-half read per MFMA (the scheduler otherwise sinks each read to just before its
    // MFMA, and every MFMA waits out a whole LDS latency); the second half's MFMAs only where it
    // holds a visible key (a half past every column keeps whatever sb held: the causal mask
    // overwrites all of it - such a step is always a diagonal one - so no per-step zeroing)
    auto scores = [&](int s, f32x16& sa, f32x16& sb) {
      const bf16* kt = kbuf(bufi(g0 + s));
      bf16x8 ka[D / 16], kb8[D / 16];
#pragma unroll
      for (int m = 0; m < D / 16; ++m)
        ka[m] = *reinterpret_cast<const bf16x8*>(kt + koff + ((2 * m + hh) ^ kx) * 8);
      __builtin_amdgcn_sched_barrier(0);
      sa = f32x16{};
#pragma unroll
      for (int m = 0; m < D / 16; ++m) {
        kb8[m] = *reinterpret_cast<const bf16x8*>(kt + 32 * CH * 8 + koff + ((2 * m + hh) ^ kx) * 8);
        sa = mfma32(ka[m], qf[m], sa);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // then one MFMA
      }
      __builtin_amdgcn_sched_barrier(0);
      if (full2(s)) {
        sb = mfma32(kb8[0], qf[0], f32x16{});
#pragma unroll
        for (int m = 1; m < D / 16; ++m) sb = mfma32(kb8[m], qf[m], sb);
      }
    };
    // online softmax of S(s): causal mask on diagonal steps, row max (one cross-half exchange),
    // deferred max (T13: the running max moves only when some column grew by more than THR),
    // P = exp2(S sl2 - m) packed to bf16; l is rescaled here, O by the PV that consumes P
    auto softmax = [&](int s, f32x16& sa, f32x16& sb, bf16x8 (&pp)[4], float& alpha, bool& resc) {
      if (diag(s) || low(s)) {
        const int kb = akey(s);
        // keys <= lo: before this column's window; sink step: keys >= nS are not sinks
        const int lo = s < ns ? -1 : (win ? pq - wmain : -1);
        const int hi = s < ns ? min(pq, nS - 1) : pq;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb + 16 * (r >> 3) + 8 * hh + (r & 7);
          sa[r] = (key > hi || key <= lo) ? -INFINITY : sa[r];
          sb[r] = (key + 32 > hi || key + 32 <= lo) ? -INFINITY : sb[r];   // (an unread half:
        }                                                                  //  every key masked)
      }
      // IEEE maximum (NaN-propagating) lowers to v_maximum3_f32, one per two scores; fmaxf's
      // maxnum would first canonicalise every MFMA output with a v_max_f32 x, x of its own
      float mx = __builtin_elementwise_maximum(sa[0], sb[0]);
#pragma unroll
      for (int r = 1; r < 16; ++r)
        mx = __builtin_elementwise_maximum(mx, __builtin_elementwise_maximum(sa[r], sb[r]));
      mx = xhalf_max(mx);
      const float pmax = mx * sl2;
      resc = __any(pmax > m_run + P32_THR);
      const float m_new = resc ? fmaxf(m_run, pmax) : m_run;
      alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sa[r] = __builtin_amdgcn_exp2f(fmaf(sa[r], sl2, -m_new));
        sb[r] = __builtin_amdgcn_exp2f(fmaf(sb[r], sl2, -m_new));
      }
      float ps0 = sa[0], ps1 = sb[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        ps0 += sa[r];
        ps1 += sb[r];
      }
      l_run = l_run * alpha + (ps0 + ps1);
      pp[0] = pack8(sa, 0);
      pp[1] = pack8(sa, 8);
      pp[2] = pack8(sb, 0);
      pp[3] = pack8(sb, 8);
    };
    // O^T = alpha O^T + V^T(s) P^T(s), reads as in scores; the second half only where it holds a
    // visible key (a V^T image never loaded must not reach the accumulators, even times zero)
    auto pv = [&](int s, const bf16x8 (&pp)[4], float alpha, bool resc) {
      if (resc) {
#pragma unroll
        for (int db = 0; db < D / 32; ++db) o[db] *= alpha;
      }
      const bf16* vt = vbuf(bufi(g0 + s));
      bf16x8 va[D / 16], vb[D / 16];
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        va[2 * db] = *reinterpret_cast<const bf16x8*>(vt + voff + (0 * D + 32 * db) * 8);
        va[2 * db + 1] = *reinterpret_cast<const bf16x8*>(vt + voff + (2 * D + 32 * db) * 8);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        vb[2 * db] = *reinterpret_cast<const bf16x8*>(vt + voff + (4 * D + 32 * db) * 8);
        o[db] = mfma32(va[2 * db], pp[0], o[db]);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        vb[2 * db + 1] = *reinterpret_cast<const bf16x8*>(vt + voff + (6 * D + 32 * db) * 8);
        o[db] = mfma32(va[2 * db + 1], pp[1], o[db]);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (full2(s)) {
#pragma unroll
        for (int db = 0; db < D / 32; ++db) {
          o[db] = mfma32(vb[2 * db], pp[2], o[db]);
          o[db] = mfma32(vb[2 * db + 1], pp[3], o[db]);
        }
      }
    };
    auto dma_next = [&](int s) {   // the DMA issued in interval s: step s+1
      if (s + 1 < nsteps) dma_step(cur, s + 1, bufi(g0 + s + 1));
    };

    f32x16 sa, sb = f32x16{};
    bf16x8 pp[4];
    float alpha;
    bool resc;
    if (!STAG || w < NW / 2) {
      // interval s: S(s) | softmax(s) | PV(s); the DMA is issued behind the first MFMAs, so its
      // block-table lookups (scalar loads waited in place) overlap the matrix pipe
      for (int s = 0; s < nsteps; ++s) {
        scores(s, sa, sb);
        if (s < ns) load_q(cur, qf, p.q);   // the main steps score against q
        dma_next(s);
        softmax(s, sa, sb, pp, alpha, resc);
        pv(s, pp, alpha, resc);
        if (F8 && s + 1 < nsteps) f8_commit();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA (and Q) landed
        __syncthreads();
      }
    } else {
      // the stagger (MI355X_MICROARCH.md "Two waves per SIMD", item 9): waves NW/2.. (one per
      // SIMD, paired with a wave of the first half) run interval s as softmax(s-1) | PV(s-1) |
      // S(s), so each SIMD's two waves put vector work beside matrix work instead of both
      // computing, then both exponentiating.  S(s-1) stays in registers across the barrier and
      // V(s-1) in its buffer (three buffers: the DMA of interval s writes step s+1's).
      for (int s = 0; s < nsteps; ++s) {
        if (s > 0) {
          softmax(s - 1, sa, sb, pp, alpha, resc);
          pv(s - 1, pp, alpha, resc);
        }
        dma_next(s);
        scores(s, sa, sb);
        if (s < ns) load_q(cur, qf, p.q);
        if (F8 && s + 1 < nsteps) f8_commit();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      softmax(nsteps - 1, sa, sb, pp, alpha, resc);
      pv(nsteps - 1, pp, alpha, resc);
    }

    // ---- normalise and store through LDS, so that the stores leave as whole rows: the register
    // layout has each lane hold 4 d values (d = 32 db + (r & 3) + 8 (r >> 2) + 4 hh) of ONE row,
    // and direct per-lane 8-byte stores touched 32 rows (lines) per instruction - store-issue
    // bound, the tail of every workgroup (MI355X_MICROARCH.md constants 'attention epilogue store
    // tail').  Staging image: row R = 32 w + c (= head R / TQ, token R % TQ) of 128 d, 16-byte
    // chunk j at j ^ (R & 15), in the buffer of this tile's last step (all of it read by now; the
    // next tile's first step lands in the other) - or, 8-wave workgroups, buffers 0-1 (64 KB, no
    // prefetch in flight); then each wave-instruction stores 4 whole rows of one token (adjacent
    // heads: 1 KB contiguous in [token][head][d]).
    const float lsum = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = lsum > 0.f ? (F8 ? p.v_scale : 1.f) / lsum : 0.f;
    if (STAG) __syncthreads();                  // every wave is past its last V^T read
    // persistent: the next tile's Q (into qf, dead now) and its first K / V^T step (into the
    // buffer after this tile's last one) are in flight while this tile's output is staged and
    // stored; the block-table, q_start and seq_lens lookups for it too
    const int wi_next = item_of(n + 1);
    Item nxt;
    const bool more = PF && wi_next < wi_end && decode(wi_next, nxt);
    if (more) {
      dma_step(nxt, 0, bufi(g0 + nsteps));
      load_q(nxt, qf, nxt.ns ? p.q_sink : p.q);
    }
    // (8-wave workgroups stage 64 KB: buffers 0-1, nothing in flight; 4-wave ones 32 KB)
    bf16* stg = NW == 8 ? &smem[0][0][0] : kbuf(bufi(g0 + nsteps - 1));
    {
      bf16* srow = stg + (size_t)R * D + 4 * hh;
#pragma unroll
      for (int db = 0; db < D / 32; ++db)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[db][4 * a + r] * inv);
          *reinterpret_cast<bf16x4*>(srow + ((4 * db + a) ^ (R & 15)) * 8) = v;
        }
    }
    __syncthreads();
    constexpr int PER = TQ * GW * (D / 8) / 64 / NW;   // store instructions per wave
    const int nvalid = min(TQ, cur.qlen - cur.t0);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = (k * NW + w) * 64 + lane;
      const int chunk = i & 15, rr = i >> 4;
      const int head = rr % GW, token = rr / GW;
      const int R2 = head * TQ + token;
#if P32_KO_OUT
      if (token < nvalid && lsum == 12345.f) {
#else
      if (token < nvalid) {
#endif
        const bf16x8 v =
            *reinterpret_cast<const bf16x8*>(stg + (size_t)R2 * D + (chunk ^ (R2 & 15)) * 8);
        *reinterpret_cast<bf16x8*>(p.out + ((size_t)(cur.qs0 + cur.t0 + token) * p.nh + cur.h0 +
                                            head) * D + chunk * 8) = v;
      }
    }
    if (!more) break;
    // the next tile's first step (and Q) landed; the staging buffer is its step-1 buffer: every
    // wave's reads of it first
    if constexpr (F8) f8_commit();   // (its buffer is not the staging one)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    g0 += nsteps;
    ++n;
    wi = wi_next;
    cur = nxt;
  }
}

// Eligible: head_dim 128, bf16 or fp8 caches, full or windowed (sinks up to 64 slots), no custom
// mask, power-of-two block size; any GQA
// group (a workgroup takes GW = 8, 4, 2 or 1 of its heads, the largest that divides it) - but a
// group that is not a multiple of 4 only with the long-chunk tiles (prefill_qb 2): its short
// tiles make 2-wave workgroups, and attention.hip's kernel is faster there (512-token prompts,
// MHA 355 vs 309 TF; long chunks 571-620 vs 780-920: profiles/r6/gqa/).
bool attn_prefill32_eligible(const AttnParams& p, int D) {
  const int G = p.nh / p.nkv;
  // fp8 caches widen through registers: 4- and 8-wave workgroups only (a 2-wave one would hold
  // 32 registers of fp8 runs per lane and spill) - all long-chunk tiles, and 16-token tiles of
  // groups of 8
  if (p.kv_fp8 && !(p.prefill_qb == 2 || G % 8 == 0)) return false;
  return p.prefill_m32 && D == P32_D && p.mask == nullptr &&
         (p.ring == 0 || (p.window > p.n_sink && p.ring % 32 == 0 && p.sink_pad % 32 == 0 &&
                          p.sink_pad <= 64 && (p.n_sink == 0 || p.q_sink != nullptr))) &&
         p.bs % 32 == 0 && (p.bs & (p.bs - 1)) == 0 && (G % 4 == 0 || p.prefill_qb == 2);
}

// The instance for (heads per workgroup, tile size, cache dtype, window mode); fp8 caches take
// 4- and 8-wave workgroups only (eligibility), so their 2-wave instances are never built.
template <bool F8, bool WIN>
static void p32_dispatch(const AttnParams& p, int gw, bool big, dim3 grid, int nw,
                         hipStream_t stream) {
  const dim3 block(64 * nw);
  if (gw == 8) {
    if (big) attn_prefill32_kernel<32, 8, F8, WIN><<<grid, block, 0, stream>>>(p);
    else attn_prefill32_kernel<16, 8, F8, WIN><<<grid, block, 0, stream>>>(p);
  } else if (gw == 4) {
    if (big) attn_prefill32_kernel<32, 4, F8, WIN><<<grid, block, 0, stream>>>(p);
    else if constexpr (!F8) attn_prefill32_kernel<16, 4, F8, WIN><<<grid, block, 0, stream>>>(p);
  } else if (gw == 2) {
    if (big) attn_prefill32_kernel<64, 2, F8, WIN><<<grid, block, 0, stream>>>(p);
    else if constexpr (!F8) attn_prefill32_kernel<32, 2, F8, WIN><<<grid, block, 0, stream>>>(p);
  } else {
    if (big) attn_prefill32_kernel<128, 1, F8, WIN><<<grid, block, 0, stream>>>(p);
    else if constexpr (!F8) attn_prefill32_kernel<64, 1, F8, WIN><<<grid, block, 0, stream>>>(p);
  }
}

// Tile = the one attention.hip's kernel uses (16 * (4 / min(GW, 4)) * prefill_qb query tokens:
// 16 or 32 for groups of 4 and 8 heads, 32 or 64 for pairs, 64 or 128 for single heads - MHA or
// an odd group such as Qwen2's 7), so one (sequence, tile) map serves both.
int launch_attn_prefill32(const AttnParams& p, int B, int max_q, hipStream_t stream) {
  const int G = p.nh / p.nkv;
  const int gw = G % 8 == 0 ? 8 : G % 4 == 0 ? 4 : G % 2 == 0 ? 2 : 1;
  const int TQ = 16 * (4 / std::min(gw, 4)) * p.prefill_qb;
  const int nw = gw * TQ / 32;
  dim3 grid((max_q + TQ - 1) / TQ, p.nkv * (G / gw), B);
  if (p.tile_map) {
    const long total = (long)p.n_tiles * p.nkv * (G / gw);
    long per = (total + 7) / 8;              // workgroups per XCD: one tile each ...
    if (P32_PERSIST && nw != 8) {            // ... or persistent: the two a CU holds (64 KB LDS)
      static int cus = 0;
      if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
          cus = 0;
        if (cus <= 0) cus = 256;
      }
      per = std::min(per, (long)(2 * cus / 8));
    }
    grid = dim3((unsigned)(per * 8), 1, 1);
  }
  if (grid.x == 0) return 0;
  const bool big = p.prefill_qb == 2;
  if (p.kv_fp8) {
    if (p.ring > 0) p32_dispatch<true, true>(p, gw, big, grid, nw, stream);
    else p32_dispatch<true, false>(p, gw, big, grid, nw, stream);
  } else {
    if (p.ring > 0) p32_dispatch<false, true>(p, gw, big, grid, nw, stream);
    else p32_dispatch<false, false>(p, gw, big, grid, nw, stream);
  }
  return 0;
}

}  // namespace dli
