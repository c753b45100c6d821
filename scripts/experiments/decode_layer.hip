// One Llama decoder layer for ONE decode row in ONE launch (batch-1 / single-session decode).
//
// At batch 1 a layer is a pure weight stream (70B fp8: 0.86 GB per layer, ~125 us at HBM rate)
// cut into six dependent kernels (QKV + RoPE, attention, merge, O, gate|up + SwiGLU, down); each
// boundary costs a launch plus the latency ramp of the next kernel's first loads (~3.5 us
// measured per GEMV, scripts/gemv_bw.py) -- ~15 % of the fp8 step.  Here the six phases run in
// one persistent grid (one 512-thread workgroup per CU, all co-resident) separated by grid
// barriers, and every wave issues its first weight loads of the next phase BEFORE it waits at the
// barrier, so the barrier's latency hides under the weight fetch instead of adding to it.
//
//   P1  x = rmsnorm(h + r) * w1 (LDS, per workgroup); QKV GEMV, RoPE, k / v -> paged cache, q
//   P2  attention: 4-wave groups run attn_decode_item over consecutive splits and merge them
//       in LDS (attention.hip's grouped path), partials -> part_o / part_ml
//   P4  every workgroup merges the partials into its LDS x (attn_combine_kernel's arithmetic);
//       O GEMV -> o_out
//   P5  res2 = o_out + (h + r); x = rmsnorm(res2) * w2 (LDS); gate|up GEMV + SwiGLU -> act
//   P6  down GEMV -> out
//
// Every phase uses the arithmetic of the kernel it replaces (GEMV per-lane k order and wave
// reduction, the 256-thread norm reduction, the grouped attention merge and the combine), so the
// layer output is bit-identical to the six-kernel path (tests/test_decode_layer_gpu.py).
//
// Grid barrier: 64-bit arrival counters (8, summed) per stream of layer launches, never reset: a
// launch's base is their sum rounded down to a multiple of kDlBarriers * grid (every earlier launch
// added exactly that many), read before the first arrival.  Arrivals are agent-scope atomics
// after a release fence; waiting is a bounded spin (an error count, never a hang: co-residency
// of all workgroups is required, so the host launches grid = CUs and only when no other kernel
// can hold CUs -- ops.decode_layer_ok).
#include "kernels.h"
#include "attn_core.h"
#include "gemv_core.h"

namespace dli {

namespace {

constexpr int kDlThreads = 512;   // 8 waves, 2 per SIMD: 256 VGPRs for the attention phase
constexpr int kDlWaves = kDlThreads / 64;
constexpr int kDlBarriers = 4;
constexpr int kDlUnroll = 4;      // k-steps of weight loads in flight per GEMV wave (8 spills)

constexpr int kDlCounters = 8, kDlCounterStride = 16;   // u64s: one 128-B line per counter
constexpr int kDlMergeCounters = 64;   // attention merge arrivals, one per (kv head, head group)

__device__ __forceinline__ unsigned long long dl_arrivals(unsigned long long* bar) {
  unsigned long long v[kDlCounters];
#pragma unroll
  for (int i = 0; i < kDlCounters; ++i)
    v[i] = __hip_atomic_load(bar + i * kDlCounterStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long t = 0;
#pragma unroll
  for (int i = 0; i < kDlCounters; ++i) t += v[i];
  return t;
}

// diagnostics (DecodeLayerParams::stamps, [grid][24]): slot 0 = start, 2k-1 = arrival at barrier
// k, 12+k = its L2 write-back done, 2k = its release, 9 = end
__device__ __forceinline__ void dl_stamp(unsigned long long* st, int slot) {
  if (st != nullptr && threadIdx.x == 0) st[(size_t)blockIdx.x * 24 + slot] = __builtin_amdgcn_s_memrealtime();
}

// Grid barrier k.  Order inside: every wave's stores complete (vmcnt(0): nothing else is in
// flight yet), one L2 write-back by thread 0, its arrival; THEN the next phase's first weight
// loads (`prefetch`) go out, so they overlap the wait instead of delaying the arrival (vmcnt is
// in order on CDNA: a wait for the stores would also wait for loads issued before it); the
// acquire is a bare L2 / L1 invalidate, which waits for nothing.
template <typename F>
__device__ __forceinline__ void dl_grid_sync(unsigned long long* bar, unsigned long long target,
                                             unsigned* err, unsigned long long* st, int k,
                                             F&& prefetch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores have reached L2
  __syncthreads();
  dl_stamp(st, 2 * k - 1);
  if (threadIdx.x == 0) {
    // arrivals spread over kDlCounters counters in separate 128-B lines (workgroup b -> counter
    // b % kDlCounters): 256 arrivals on ONE address serialise (~6 us measured when they all come
    // at once); pollers sum the counters.
    // Every cross-workgroup value of a phase is stored write-through at device scope (gst<true>),
    // so its completion (vmcnt(0) above) is the release: no L2 write-back (measured 1.3-3.4 us
    // median per workgroup and barrier when it was one); the acquire below invalidates this CU's
    // L1 / the XCD's L2 (no stale line of a buffer another workgroup wrote this launch)
    dl_stamp(st, 12 + k);
    __hip_atomic_fetch_add(bar + (blockIdx.x % kDlCounters) * kDlCounterStride, 1ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  prefetch();
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (dl_arrivals(bar) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins == (1u << 21)) {   // ~0.2 s: count it and go on (never hang the GPU)
        atomicAdd(err, 1u);
        break;
      }
    }
    asm volatile("buffer_inv sc1" ::: "memory");
  }
  dl_stamp(st, 2 * k);
  __syncthreads();
}

// x staging: rmsnorm(a + b) * w for one row of K <= 8192 (b optional), by threads 0..255 with
// gemv_norm_prologue_regs' vector assignment and fma order (the other waves contribute 0 to the
// block sum, which leaves it unchanged): bit-identical to the 256-thread fused norm.  `sum_out`
// (optional, workgroup 0 only): a + b.
__device__ __forceinline__ void dl_norm_stage(bf16x8* xs, const bf16* a, const bf16* b,
                                              const bf16* w, float eps, int K, bf16* sum_out,
                                              float* scratch) {
  constexpr int VPT = 4;
  const int nvec = K >> 3;
  const int t = threadIdx.x;
  const bool act = t < 256;
  auto vidx = [&](int i) { const int idx = t + i * 256; return idx < nvec ? idx : nvec - 1; };
  auto vok = [&](int i) { return act && t + i * 256 < nvec; };
  bf16x8 wv[VPT], av[VPT], rv[VPT];
  if (act) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      wv[i] = reinterpret_cast<const bf16x8*>(w)[vidx(i)];
      av[i] = reinterpret_cast<const bf16x8*>(a)[vidx(i)];
      if (b != nullptr) rv[i] = reinterpret_cast<const bf16x8*>(b)[vidx(i)];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    if (!vok(i)) continue;
    if (b != nullptr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) av[i][j] = (bf16)((float)av[i][j] + (float)rv[i][j]);
      if (sum_out != nullptr) gst<true>(reinterpret_cast<bf16x8*>(sum_out) + t + i * 256, av[i]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)av[i][j];
      ss = __builtin_fmaf(v, v, ss);
    }
  }
  ss = block_reduce_sum(ss, scratch);
  const float rstd = rsqrtf(ss / (float)K + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    if (!vok(i)) continue;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)av[i][j] * rstd * (float)wv[i][j]);
    xs[t + i * 256] = o;
  }
}

// plain x staging (global -> LDS), K % 8 == 0
__device__ __forceinline__ void dl_copy_stage(bf16x8* xs, const bf16* x, int K) {
  for (int i = threadIdx.x; i < (K >> 3); i += kDlThreads) xs[i] = reinterpret_cast<const bf16x8*>(x)[i];
}

// One GEMV phase over tasks (2 weight rows each).  A wave runs TP tasks at once (t, t + nw, ...)
// and walks them in chunks of 4 k-steps (TP x 4 x 2 rows of 16-B weight loads per lane); the
// loads of chunk c + 1 are issued before chunk c is consumed (two register sets), so every wave
// keeps a full chunk in flight without a bubble -- the 8 waves of a CU have to cover the HBM
// latency that ~20 resident waves cover in the standalone kernel.  Each task's per-lane k order,
// dot order, wave reduction and scaling are skinny_gemm_kernel's / skinny_gemm_fp8_kernel's
// (M = 1, bf16 activations): every output is bit-identical to the standalone GEMV.  x in LDS.
// Chunk 0 may have been issued before the phase's barrier (prefetch / pre).
template <int WQ, int TP>   // WQ: 0 bf16, 1 fp8 e4m3, 2 int8
struct DlGemv {
  static constexpr int E = WQ == 0 ? 8 : 16;        // elements per lane per k-step (16 B)
  static constexpr int kStep = 64 * E;
  static constexpr int U = kDlUnroll;
  u32x4n wv[2][TP][U][kRows];
  const unsigned char* wrow[2][TP][kRows];

  template <int EP>
  __device__ __forceinline__ static int ntask(const DecodeProj& g) {
    return EP != kEpPlain ? g.N / 2 : (g.N + kRows - 1) / kRows;
  }
  __device__ __forceinline__ static int iters(const DecodeProj& g) {
    return (g.K + kStep * U - 1) / (kStep * U);
  }
  // issue chunk c (round c / iters, k-chunk c % iters) into register set B
  template <int EP, int B>
  __device__ __forceinline__ void issue(const DecodeProj& g, int gw, int nw, const GemvRope& rp,
                                        int c) {
    const int esz = WQ == 0 ? 2 : 1;
    const int it = iters(g), r = c / it, kc = c - r * it;
    const int nt = ntask<EP>(g);
    const int t0 = gw + r * nw * TP;
    bool live[TP];
#pragma unroll
    for (int i = 0; i < TP; ++i) {
      live[i] = t0 + i * nw < nt;   // idle slots load nothing (their results are never stored)
      const int t = min(t0 + i * nw, nt - 1);
#pragma unroll
      for (int q = 0; q < kRows; ++q)
        wrow[B][i][q] = static_cast<const unsigned char*>(g.w) +
                        (size_t)min(gemv_row<EP>(t, q, rp), g.N - 1) * g.K * esz;
    }
    const int k0 = (threadIdx.x & 63) * E + kc * kStep * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * kStep;
#pragma unroll
      for (int i = 0; i < TP; ++i)
#pragma unroll
        for (int q = 0; q < kRows; ++q)
          wv[B][i][u][q] = live[i] && k < g.K
                               ? __builtin_nontemporal_load(reinterpret_cast<const u32x4n*>(
                                     wrow[B][i][q] + (size_t)k * esz))
                               : u32x4n{0u, 0u, 0u, 0u};
    }
  }
  template <int EP>
  __device__ __forceinline__ int chunks(const DecodeProj& g, int gw, int nw) const {
    const int nt = ntask<EP>(g);
    return gw < nt ? (nt - gw + nw * TP - 1) / (nw * TP) * iters(g) : 0;
  }
  // chunk 0 of this wave (before a barrier)
  template <int EP>
  __device__ __forceinline__ void prefetch(const DecodeProj& g, int gw, int nw, const GemvRope& rp) {
    if (chunks<EP>(g, gw, nw) > 0) issue<EP, 0>(g, gw, nw, rp, 0);
  }

  float acc[TP][kRows];
  float sx;

  // consume chunk c from register set B; the last chunk of a round reduces and stores its tasks
  template <int EP, int B>
  __device__ __forceinline__ void consume(const DecodeProj& g, const bf16* xs, bf16* y, int gw,
                                          int nw, const GemvRope& rp, int c) {
    const int lane = threadIdx.x & 63;
    const int K = g.K, N = g.N, nt = ntask<EP>(g);
    const int it = iters(g), r = c / it, kc = c - r * it;
    if (kc == 0) {
#pragma unroll
      for (int i = 0; i < TP; ++i) acc[i][0] = acc[i][1] = 0.f;
      sx = 0.f;
    }
    const int k0 = lane * E + kc * kStep * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * kStep;
      if constexpr (WQ == 0) {
        const bf16x8 xv = k < K ? *reinterpret_cast<const bf16x8*>(xs + k) : bf16x8{};
#pragma unroll
        for (int i = 0; i < TP; ++i) {
          const bf16x8 w0 = __builtin_bit_cast(bf16x8, wv[B][i][u][0]);
          const bf16x8 w1 = __builtin_bit_cast(bf16x8, wv[B][i][u][1]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bf16x2 xp = {xv[2 * j], xv[2 * j + 1]};
            acc[i][0] = __builtin_amdgcn_fdot2_f32_bf16(xp, bf16x2{w0[2 * j], w0[2 * j + 1]}, acc[i][0], false);
            acc[i][1] = __builtin_amdgcn_fdot2_f32_bf16(xp, bf16x2{w1[2 * j], w1[2 * j + 1]}, acc[i][1], false);
          }
        }
      } else {
        bf16x8 xv[2];
        if (k < K) {
          xv[0] = *reinterpret_cast<const bf16x8*>(xs + k);
          xv[1] = *reinterpret_cast<const bf16x8*>(xs + k + 8);
        } else {
          xv[0] = xv[1] = bf16x8{};
        }
        if constexpr (WQ == 2) {
          const bf16x2 ones = {(bf16)1.f, (bf16)1.f};
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              sx = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{xv[h][2 * j], xv[h][2 * j + 1]}, ones,
                                                   sx, false);
#pragma unroll
          for (int i = 0; i < TP; ++i)
#pragma unroll
            for (int q = 0; q < kRows; ++q)
#pragma unroll
              for (int d = 0; d < 4; ++d) {
                const unsigned ub = wv[B][i][u][q][d] ^ 0x80808080u;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                  const bf16x2 wp = u8pair_to_bf16x2(ub, j);
                  const int e = (d & 1) * 4 + 2 * j;
                  acc[i][q] = __builtin_amdgcn_fdot2_f32_bf16(
                      bf16x2{xv[d >> 1][e], xv[d >> 1][e + 1]}, wp, acc[i][q], false);
                }
              }
        } else {
#pragma unroll
          for (int i = 0; i < TP; ++i)
#pragma unroll
            for (int q = 0; q < kRows; ++q) {
              const bf16x8 w0 = fp8x8_to_bf16x8(uint2{wv[B][i][u][q][0], wv[B][i][u][q][1]});
              const bf16x8 w1 = fp8x8_to_bf16x8(uint2{wv[B][i][u][q][2], wv[B][i][u][q][3]});
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const bf16x2 x0 = {xv[0][2 * j], xv[0][2 * j + 1]};
                const bf16x2 x1 = {xv[1][2 * j], xv[1][2 * j + 1]};
                acc[i][q] = __builtin_amdgcn_fdot2_f32_bf16(x0, bf16x2{w0[2 * j], w0[2 * j + 1]}, acc[i][q], false);
                acc[i][q] = __builtin_amdgcn_fdot2_f32_bf16(x1, bf16x2{w1[2 * j], w1[2 * j + 1]}, acc[i][q], false);
              }
            }
        }
      }
    }
    if (kc != it - 1) return;
    const int t0 = gw + r * nw * TP;
#pragma unroll
    for (int i = 0; i < TP; ++i) {
      const int t = t0 + i * nw;
      if (t >= nt) break;
      if constexpr (WQ == 2) {
#pragma unroll
        for (int q = 0; q < kRows; ++q) acc[i][q] -= 128.f * sx;
      }
      float v[1][kRows];
#pragma unroll
      for (int q = 0; q < kRows; ++q) {
        const int n = min(gemv_row<EP>(t, q, rp), N - 1);
        const float sm = wave_reduce_sum(acc[i][q]);
        v[0][q] = WQ == 0 ? sm + (g.bias ? (float)g.bias[n] : 0.f)
                          : sm * g.ws[n] + (g.bias ? (float)g.bias[n] : 0.f);
      }
      gemv_store<EP, 1, true>(v, t, lane, N, y, rp);
    }
  }

  template <int EP>
  __device__ __forceinline__ void run(const DecodeProj& g, const bf16* xs, bf16* y, int gw, int nw,
                                      const GemvRope& rp, bool pre) {
    const int C = chunks<EP>(g, gw, nw);
    if (C == 0) return;
    if (!pre) issue<EP, 0>(g, gw, nw, rp, 0);
    for (int c = 0; c < C; c += 2) {
      if (c + 1 < C) issue<EP, 1>(g, gw, nw, rp, c + 1);
      consume<EP, 0>(g, xs, y, gw, nw, rp, c);
      if (c + 1 >= C) break;
      if (c + 2 < C) issue<EP, 0>(g, gw, nw, rp, c + 2);
      consume<EP, 1>(g, xs, y, gw, nw, rp, c + 1);
    }
  }
};

template <int WQ, bool KV8>
__global__ void __launch_bounds__(kDlThreads) decode_layer_kernel(DecodeLayerParams a) {
  constexpr int D = 128;
  constexpr int LROW = D + 4;
  // LDS: the staged x of the current GEMV phase (<= 64 KB: I <= 32768), the attention groups'
  // merge images, reduction scratch
  __shared__ __attribute__((aligned(16))) bf16x8 xs[4096];
  __shared__ __attribute__((aligned(16))) float alds[4 * 16 * (LROW + 2)];
  __shared__ float scratch[kDlWaves];
  const int G = gridDim.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // GEMV task order: wave-major across workgroups, so a phase whose task count is not a multiple
  // of the wave count (70B QKV: 2.5 per wave) gives every CU the same number of tasks
  const int gw = __builtin_amdgcn_readfirstlane(wave * (int)gridDim.x + (int)blockIdx.x);
  const int nw = G * kDlWaves;
  const bf16* xsb = reinterpret_cast<const bf16*>(xs);

  // this launch's barrier base (see the header)
  __shared__ unsigned long long base_s;
  if (threadIdx.x == 0) {
    const unsigned long long v = dl_arrivals(a.bar);
    const unsigned long long per = (unsigned long long)kDlBarriers * G;
    base_s = v / per * per;
  }
  // (the norm stage's block reduction below synchronises the workgroup before base_s is read)

  dl_stamp(a.stamps, 0);
  // ---- P1: norm 1 + QKV GEMV + RoPE / cache write ----
  DlGemv<WQ, 3> g1;   // 70B: ~2.5 QKV tasks per wave, one round
  g1.template prefetch<kEpRope>(a.qkv, gw, nw, a.rp);
  dl_norm_stage(xs, a.h, a.r, a.ln1, a.eps1, a.qkv.K, blockIdx.x == 0 ? a.res1 : nullptr, scratch);
  __syncthreads();
  const unsigned long long base = base_s;
  g1.template run<kEpRope>(a.qkv, xsb, nullptr, gw, nw, a.rp, true);
  if (blockIdx.x == 0 && threadIdx.x < kDlMergeCounters && a.merge_cnt != nullptr)   // P2's merge
    __hip_atomic_store(a.merge_cnt + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  dl_grid_sync(a.bar, base + 1ull * G, a.err, a.stamps, 1, [] {});

  // ---- P2: attention partials (4-wave groups, attention.hip's grouped merge) ----
  const AttnParams& p = a.ap;
  const int items = p.nkv * ((p.nh / p.nkv + 15) >> 4) * p.num_splits;   // B = 1
  const bool last_merge = a.merge_cnt != nullptr && a.gs == 4 &&
                          p.nkv * ((p.nh / p.nkv + 15) >> 4) <= kDlMergeCounters;
  // one 4-wave group (the standalone kernel's workgroup) per workgroup, on as many CUs as there
  // are groups: the latency-bound key loop runs one wave per SIMD, as it does standalone; waves
  // 4..7 only join the merge barrier
  for (int gidx = blockIdx.x; gidx * 4 < items; gidx += G) {   // workgroup-uniform
    const bool aw = wave < 4;
    const int wig = wave & 3;
    // gidx: the standalone kernel's blockIdx
    const int item_raw = gidx * 4 + wig;
    const bool live = item_raw < items;
    const int item = __builtin_amdgcn_readfirstlane(live ? item_raw : items - 1);
    WaveState<D> st;
    DecodeItem di{};
    const int col = lane & 15, h4 = lane >> 4;
    float* lds = alds;
    float* lml = lds + 4 * 16 * LROW;
    if (aw) {
      di = attn_decode_item<D, false, KV8, false>(p, item, live, st);
      float lsum = st.l;
      lsum += __shfl_xor(lsum, 16, 64);
      lsum += __shfl_xor(lsum, 32, 64);
      float* lo = lds + (wig * 16 + col) * LROW;
#pragma unroll
      for (int u = 0; u < D / 16; ++u) {
        int d;
        f32x4 o;
        o_unit<D, KV8>(st, u, h4, d, o);
        *reinterpret_cast<f32x4*>(lo + d) = o;
      }
      if (h4 == 0) {
        lml[(wig * 16 + col) * 2] = st.m;
        lml[(wig * 16 + col) * 2 + 1] = lsum;
      }
    }
    __syncthreads();
    const int gs = a.gs;
    const int gq = wig / gs, w0 = gq * gs;   // merge group of this wave inside its 4-wave group
    const int gitem = gidx * 4 + w0;
    if (aw && gitem < items) {
      const int S2 = p.num_splits / gs;
      const int s2 = (gitem % p.num_splits) / gs;
      const int tg = (wig - w0) * 64 + lane;
      constexpr int V4 = 16 * D / 4;
      const int Gq = di.G;
      for (int u = tg; u < V4; u += gs * 64) {
        const int c = u / (D / 4), d4 = (u % (D / 4)) * 4;
        if (di.g0 + c >= Gq) continue;
        float M = -1e30f;
        for (int w = w0; w < w0 + gs; ++w) M = fmaxf(M, lml[(w * 16 + c) * 2]);
        float Lt = 0.f;
        f32x4 O = {0.f, 0.f, 0.f, 0.f};
        for (int w = w0; w < w0 + gs; ++w) {
          const float f = __builtin_amdgcn_exp2f(lml[(w * 16 + c) * 2] - M);
          Lt += f * lml[(w * 16 + c) * 2 + 1];
          O += f * *reinterpret_cast<const f32x4*>(lds + (w * 16 + c) * LROW + d4);
        }
        const int head = di.kvh * Gq + di.g0 + c;
        if (S2 == 1) {
          const float inv = Lt > 0.f ? di.vsc / Lt : 0.f;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(O[r] * inv);
          gst<true>(reinterpret_cast<bf16x4*>(a.attn + (size_t)head * D + d4), v);
        } else {
          const size_t r0 = (size_t)s2 * p.nh + head;
          gst<true>(reinterpret_cast<f32x4*>(p.part_o + r0 * D + d4), O * di.vsc);
          if (d4 == 0) {
            gst<true>(p.part_ml + r0 * 2, M);
            gst<true>(p.part_ml + r0 * 2 + 1, Lt);
          }
        }
      }
    }
    // The last of the S2 merge groups of a (kv head, head group) to finish merges all S2
    // partials into the attention output itself (gs == 4: one merge group per workgroup; the
    // counter was zeroed by workgroup 0 before barrier 1): no merge phase after the barrier.
    // Partials are stored write-through and the arrival follows their completion; the merging
    // group reads them at device scope (sc1), past any stale L2 line.
    const int S2g = p.num_splits / a.gs;
    if (last_merge && S2g > 1 && gidx * 4 < items) {   // workgroup-uniform
      __shared__ int is_last;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int hg = (gidx * 4 / p.num_splits);   // (kv head, head group) index of this group
      if (threadIdx.x == 0)
        is_last = __hip_atomic_fetch_add(a.merge_cnt + hg, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S2g - 1);
      __syncthreads();
      if (is_last) {
        const int Gq = p.nh / p.nkv, hgroups = (Gq + 15) >> 4;
        const int kvh = hg / hgroups, g0 = (hg % hgroups) * 16;
        const int nheads = min(16, Gq - g0);
        constexpr int NG = 256 / (D / 4);
        const auto rso = __builtin_amdgcn_make_buffer_rsrc(p.part_o, 0, 0x7fffffff, 0x00020000);
        const auto rsm = __builtin_amdgcn_make_buffer_rsrc(p.part_ml, 0, 0x7fffffff, 0x00020000);
        for (int idx = threadIdx.x; idx < nheads * (D / 4); idx += kDlThreads) {
          const int head = kvh * Gq + g0 + idx / (D / 4), l4 = idx % (D / 4);
          float gm[NG], gsum[NG];
          f32x4 go[NG];
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            gm[g] = -1e30f;
            gsum[g] = 0.f;
            go[g] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
          for (int base = 0; base < S2g; base += NG) {
#pragma unroll
            for (int half = 0; half < NG; half += 4) {   // 4 partials in flight at a time
              float mi[4], li[4];
              f32x4 oi[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                if (base + half + j < S2g) {
                  const int r = (base + half + j) * p.nh + head;
                  // sc1 (device scope): the value another workgroup stored write-through
                  mi[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsm, r * 8, 0, 16));
                  li[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsm, r * 8 + 4, 0, 16));
                  oi[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                        rso, (r * D + 4 * l4) * 4, 0, 16));
                }
              }
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int g = half + j;
                if (base + g < S2g) {
                  const float mn = fmaxf(gm[g], mi[j]);
                  const float e0 = __builtin_amdgcn_exp2f(gm[g] - mn), e1 = __builtin_amdgcn_exp2f(mi[j] - mn);
                  go[g] = go[g] * e0 + oi[j] * e1;
                  gsum[g] = gsum[g] * e0 + li[j] * e1;
                  gm[g] = mn;
                }
              }
            }
          }
          float M = -1e30f;
#pragma unroll
          for (int g = 0; g < NG; ++g) M = fmaxf(M, gm[g]);
          float Lt = 0.f;
          f32x4 O = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            const float f = __builtin_amdgcn_exp2f(gm[g] - M);
            Lt += f * gsum[g];
            O += f * go[g];
          }
          const float inv = Lt > 0.f ? 1.f / Lt : 0.f;
          bf16x4 v;
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = (bf16)(O[q] * inv);
          gst<true>(reinterpret_cast<bf16x4*>(a.attn + (size_t)head * D + 4 * l4), v);
        }
      }
    }
    __syncthreads();   // the LDS images are rewritten by the next group of this workgroup
  }
  DlGemv<WQ, 2> g4;
  const bool o_early = (a.flags & 1) != 0;   // O weights in flight during the attention tail
  dl_grid_sync(a.bar, base + 2ull * G, a.err, a.stamps, 2, [&] {
    if (o_early) g4.template prefetch<kEpPlain>(a.o, gw, nw, a.rp);
  });

  // ---- P3 + P4: merge the partials into the O GEMV's x (LDS), O GEMV ----
  const int S2 = p.num_splits / a.gs;
  if (S2 > 1 && last_merge) {
    dl_copy_stage(xs, a.attn, a.o.K);   // merged by the last attention group of each head group
  } else if (S2 > 1 && S2 <= 4 && p.nh * (D / 4) <= 4 * kDlThreads) {
    // short contexts (<= 4 partials per head, every item of the workgroup in one pass): all
    // loads of a thread's 4 items first, one round trip; the combine kernel's groups 4..7 are
    // empty here (their merge terms are exact zeros) and are skipped
    constexpr int IPT = 4;
    float mi[IPT][4], li[IPT][4];
    f32x4 oi[IPT][4];
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
      const int idx = threadIdx.x + it * kDlThreads;
      const int head = idx / (D / 4), l4 = idx % (D / 4);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (g < S2 && idx < p.nh * (D / 4)) {
          const size_t r = (size_t)g * p.nh + head;
          mi[it][g] = p.part_ml[r * 2];
          li[it][g] = p.part_ml[r * 2 + 1];
          oi[it][g] = *reinterpret_cast<const f32x4*>(p.part_o + r * D + 4 * l4);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
      const int idx = threadIdx.x + it * kDlThreads;
      if (idx >= p.nh * (D / 4)) break;
      const int head = idx / (D / 4), l4 = idx % (D / 4);
      float gm[4], gsum[4];
      f32x4 go[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // the combine kernel's first merge into an empty group
        if (g >= S2) break;
        // its running state is a loop-carried value there, not a constant: keep it opaque so the
        // same multiply-adds (and contractions) are emitted
        float m0 = -1e30f, s0 = 0.f;
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+v"(m0), "+v"(s0), "+v"(o0));
        const float mn = fmaxf(m0, mi[it][g]);
        const float e0 = __builtin_amdgcn_exp2f(m0 - mn), e1 = __builtin_amdgcn_exp2f(mi[it][g] - mn);
        go[g] = o0 * e0 + oi[it][g] * e1;
        gsum[g] = s0 * e0 + li[it][g] * e1;
        gm[g] = mn;
      }
      float M = -1e30f;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (g < S2) M = fmaxf(M, gm[g]);
      float Lt = 0.f;
      f32x4 O = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (g >= S2) break;
        const float f = __builtin_amdgcn_exp2f(gm[g] - M);
        Lt += f * gsum[g];
        O += f * go[g];
      }
      const float inv = Lt > 0.f ? 1.f / Lt : 0.f;
      bf16x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = (bf16)(O[q] * inv);
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(xs) + (size_t)head * D + 4 * l4) = v;
    }
  } else if (S2 > 1) {
    // every workgroup merges all heads itself (the partials are a few tens of KB, L2-resident
    // after the first reader of each XCD) instead of a merge phase and a barrier; thread ->
    // (head, 4 consecutive d); attn_combine_kernel's 8 lane groups take partials g, g + 8, ...:
    // its per-group running merge and the in-order merge of the 8 group states are reproduced
    // with the same operations
    constexpr int NG = 256 / (D / 4);
    for (int idx = threadIdx.x; idx < p.nh * (D / 4); idx += kDlThreads) {
      const int head = idx / (D / 4), l4 = idx % (D / 4);
      float gm[NG], gsum[NG];
      f32x4 go[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        gm[g] = -1e30f;
        gsum[g] = 0.f;
        go[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      // partials base + g go to group g (the combine kernel's order); each round's loads are
      // issued together, then merged
      for (int base = 0; base < S2; base += NG) {
        float mi[NG], li[NG];
        f32x4 oi[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          if (base + g < S2) {
            const size_t r = (size_t)(base + g) * p.nh + head;
            mi[g] = p.part_ml[r * 2];
            li[g] = p.part_ml[r * 2 + 1];
            oi[g] = *reinterpret_cast<const f32x4*>(p.part_o + r * D + 4 * l4);
          }
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          if (base + g < S2) {
            const float mn = fmaxf(gm[g], mi[g]);
            const float e0 = __builtin_amdgcn_exp2f(gm[g] - mn), e1 = __builtin_amdgcn_exp2f(mi[g] - mn);
            go[g] = go[g] * e0 + oi[g] * e1;
            gsum[g] = gsum[g] * e0 + li[g] * e1;
            gm[g] = mn;
          }
        }
      }
      float M = -1e30f;
#pragma unroll
      for (int g = 0; g < NG; ++g) M = fmaxf(M, gm[g]);
      float Lt = 0.f;
      f32x4 O = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float f = __builtin_amdgcn_exp2f(gm[g] - M);
        Lt += f * gsum[g];
        O += f * go[g];
      }
      const float inv = Lt > 0.f ? 1.f / Lt : 0.f;
      bf16x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = (bf16)(O[q] * inv);
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(xs) + (size_t)head * D + 4 * l4) = v;
    }
  } else {
    dl_copy_stage(xs, a.attn, a.o.K);
  }
  __syncthreads();
  dl_stamp(a.stamps, 20);   // merge / staging done
  g4.template run<kEpPlain>(a.o, xsb, a.o_out, gw, nw, a.rp, o_early);
  DlGemv<WQ, 2> g5;   // 70B: 14 gate|up tasks per wave, 7 full rounds
  dl_grid_sync(a.bar, base + 3ull * G, a.err, a.stamps, 3,
               [&] { g5.template prefetch<kEpSwiGLU>(a.gu, gw, nw, a.rp); });

  // ---- P5: residual + norm 2 + gate|up GEMV + SwiGLU ----
  dl_norm_stage(xs, a.o_out, a.res1, a.ln2, a.eps2, a.gu.K, blockIdx.x == 0 ? a.res2 : nullptr,
                scratch);
  __syncthreads();
  g5.template run<kEpSwiGLU>(a.gu, xsb, a.act, gw, nw, a.rp, true);
  DlGemv<WQ, 2> g6;
  dl_grid_sync(a.bar, base + 4ull * G, a.err, a.stamps, 4,
               [&] { g6.template prefetch<kEpPlain>(a.down, gw, nw, a.rp); });

  // ---- P6: down GEMV ----
  dl_copy_stage(xs, a.act, a.down.K);
  __syncthreads();
  g6.template run<kEpPlain>(a.down, xsb, a.out, gw, nw, a.rp, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  dl_stamp(a.stamps, 9);
}

template <int WQ, bool KV8>
int launch_dl(const DecodeLayerParams& p, hipStream_t stream) {
  const int grid = decode_layer_grid();
  if (grid <= 0) return -20;
  static int fits = -1;   // every workgroup must be co-resident (grid barriers)
  if (fits < 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_layer_kernel<WQ, KV8>, kDlThreads, 0) != hipSuccess)
      return -21;
    fits = n >= 1 ? 1 : 0;
  }
  if (!fits) return -22;
  decode_layer_kernel<WQ, KV8><<<grid, kDlThreads, 0, stream>>>(p);
  return 0;
}

}  // namespace

int decode_layer_grid() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  return n;
}

// wq: 0 bf16, 1 fp8 e4m3, 2 int8 weights (per-row scales in DecodeProj::ws)
int launch_decode_layer(const DecodeLayerParams& p, int wq, hipStream_t stream) {
  const int K = p.qkv.K;
  if (K % 8 != 0 || K > 8 * 4 * 256) return -1;                 // norm staging: 4 vectors / thread
  if (p.o.N != K || p.gu.K != K || p.down.N != K || p.o.K != p.ap.nh * 128) return -2;
  if (p.gu.N != 2 * p.down.K || p.down.K % 8 != 0 || p.down.K > 8 * 4096) return -3;   // LDS x
  if (p.rp.D != 128 || p.ap.num_splits < 1 || p.gs < 1 || p.ap.num_splits % p.gs != 0 ||
      4 % p.gs != 0)
    return -4;
  if (p.ap.n_sink != 0 || p.ap.ring != 0) return -5;             // full cache only
  if (wq != 0 && (p.qkv.ws == nullptr || p.o.ws == nullptr || p.gu.ws == nullptr || p.down.ws == nullptr))
    return -6;
  if (p.bar == nullptr || p.err == nullptr || p.attn == nullptr || p.o_out == nullptr ||
      p.act == nullptr || p.res2 == nullptr || p.res1 == nullptr || p.out == nullptr)
    return -7;
  if (p.ap.num_splits / p.gs > 1 && (p.ap.part_o == nullptr || p.ap.part_ml == nullptr)) return -8;
  const bool kv8 = p.ap.kv_fp8 != 0;
  switch (wq) {
    case 0: return kv8 ? launch_dl<0, true>(p, stream) : launch_dl<0, false>(p, stream);
    case 1: return kv8 ? launch_dl<1, true>(p, stream) : launch_dl<1, false>(p, stream);
    case 2: return kv8 ? launch_dl<2, true>(p, stream) : launch_dl<2, false>(p, stream);
  }
  return -9;
}

}  // namespace dli
