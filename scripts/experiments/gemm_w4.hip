// Projection GEMM for CDNA4, 4-wave variant:  C[M, N] = A[M, K] . B[N, K]^T  (bf16, fp32 acc)
//
// Why a second tile kernel: the decode GEMMs run power-bound.  Clock stamps of gemm_tile.hip
// (scripts/gemm_stamps.hip) show ~2950 shader cycles per 256x256x64 k-tile whatever the number of
// busy CUs, while the clock falls from 1.83 to 1.57 GHz as more CUs run — time is energy / power
// cap, so the lever is energy per FLOP, and the largest avoidable energy item is LDS read traffic.
// gemm_tile's 8 waves own 128 x 64 output each and read 192 KB of LDS fragments per k-tile per CU;
// here 4 waves own 128 x 128 each (one wave per SIMD, 256 fp32 accumulators in AGPRs) and read
// 128 KB, a third less, for the same MFMA work — the same geometry hipBLASLt's MT256x256x64 MI16x16
// kernels use (their MIWT8_8 / WG 256 threads).
//
//   * workgroup = 4 waves as 2 (M) x 2 (N); wave tile 128 x 128 = 8 x 8 fragments of
//     v_mfma_f32_16x16x32_bf16; the weight fragment is the MFMA A operand, so each lane owns 4
//     consecutive output columns of one row (vector stores), as in gemm_tile.hip;
//   * k-tile = 128 bytes of every row (64 bf16); LDS stage = A [256][128 B] + B [256][128 B]
//     = 64 KB, two stages (tile t in stage t & 1);
//   * staging by `buffer_load_dwordx4 ... lds` (LDS-DMA) from a buffer resource per operand: the
//     per-lane VGPR offset is fixed for the whole loop and the per-instruction part (row block,
//     k-tile) is a scalar offset, so the DMA costs no vector ALU; rows past M read as zeros (the
//     resource's range), no clamping.  The XOR swizzle chunk ^ ((row >> 1) & 7) is applied on the
//     per-lane source address (LDS-DMA writes lane-linearly) and on the fragment reads: every
//     ds_read_b128 is conflict-free (docs/kernels.md);
//   * software pipeline, ONE barrier per k-tile: the fragments of k-step kk = 0 of tile t are in
//     registers when iteration t starts; the wave reads kk = 1 while its kk = 0 MFMAs run, waits
//     for its own DMA of tile t+1 and its reads, barriers, re-stages the freed stage with tile t+2
//     and reads kk = 0 of tile t+1 while the kk = 1 MFMAs run.  The DMA of a tile has one whole
//     iteration (128 MFMAs) to land;
//   * epilogues as gemm_tile: bf16 store, fp32 split-K partials (reduced by the consumer), fused
//     SwiGLU with gate/up rows interleaved per 16-row fragment pair (ops.swiglu_interleave,
//     wave column width 128).
#include "kernels.h"

namespace dli {

namespace {

constexpr int kW4Threads = 256;
constexpr int kW4Stage = 65536;   // A [256][128 B] + B [256][128 B]

enum W4Epi { kW4Bf16 = 0, kW4F32 = 1, kW4SwiGLU = 2 };

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void w4_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float w4_silu(float x) { return x / (1.f + __expf(-x)); }

// Buffer descriptor from read-first-laned inputs: uniformity the compiler can prove (otherwise
// every DMA through it becomes a waterfall loop, cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t w4_rsrc(const void* base, int bytes) {
  const unsigned long long p = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// NS = 2: 64-wide k-tiles (128-B rows) in two 64 KB slots, DMA lead one k-tile.
// NS >= 3: 32-wide k-steps (64-B rows) in NS 32 KB slots, DMA lead NS - 1 k-steps.
template <int EPI, int NS>
__global__ void __launch_bounds__(kW4Threads, 1)
gemm_w4_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* __restrict__ C,
               int M, int N, int K, int tiles_m, int tiles_n, int kps) {
  __shared__ __attribute__((aligned(1024))) char smem[NS == 2 ? 2 * kW4Stage : NS * 32768];
  const int tid = threadIdx.x, lane = tid & 63;
#ifdef GEMM_STAMPS   // diagnostic build only (g_stamp_blk: gemm_tile.hip, scripts/gemm_w4_bench.hip)
  if (tid == 0) {
    unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
    st[0] = __builtin_amdgcn_s_memrealtime();
    st[1] = __builtin_amdgcn_s_memtime();
  }
#endif
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: SGPR LDS bases
  const int wr = wave >> 1, wc = wave & 1, fr = lane & 15;

  // XCD-aware bijective remap (consecutive logical ids share an XCD and its L2)
  const int nb = gridDim.x;
  const int bx = blockIdx.x, x8 = bx & 7, q = nb >> 3, r8 = nb & 7;
  const int lid = __builtin_amdgcn_readfirstlane(
      (x8 < r8 ? x8 * (q + 1) : r8 * (q + 1) + (x8 - r8) * q) + (bx >> 3));
  const int tiles = tiles_m * tiles_n;
  const int tile = lid % tiles, split = lid / tiles;
  const int tm = tile % tiles_m, tn = tile / tiles_m;   // M tiles of one weight panel adjacent
  const int m0 = tm * 256, n0 = tn * 256;
  const int Kb = K * 2;
  const int kt0 = split * kps;
  const int T = __builtin_amdgcn_readfirstlane(min(kps, Kb / 128 - kt0));

  // ---- DMA sources: unit u = j * 256 + tid (j = 0..7) of a 32 KB operand tile -> row
  // lr = j * 32 + (tid >> 3), LDS slot tid & 7, global chunk (tid & 7) ^ ((tid >> 4) & 7) ----
  const auto rsA = w4_rsrc(A + (size_t)m0 * K, min(256, M - m0) * Kb);
  const auto rsB = w4_rsrc(B + (size_t)n0 * K, 256 * Kb);
  const int voff = (tid >> 3) * Kb + (((tid & 7) ^ ((tid >> 4) & 7)) << 4) + kt0 * 128;
  // ---- fragment reads (conflict-free: chunk ^ (row >> 1) & 7 with row & 15 == fr) ----
  const int a_lane = (wr * 128 + fr) * 128;
  const int b_lane = 32768 + (wc * 128 + fr) * 128;
  int sch[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) sch[kk] = ((kk * 4 + (lane >> 4)) ^ (fr >> 1)) << 4;

  // Accumulators live in AGPRs through inline-asm MFMAs ("+a"): with the builtin the register
  // allocator cannot keep 256 fp32 accumulators in place across the loop and copies ~200 of them
  // between AGPRs and VGPRs every k-tile.  The MFMA statements are volatile, so they keep their
  // program order relative to the LDS reads and DMA issues written between them: that order IS
  // the schedule (per 8-MFMA row: two fragment reads, or two DMA pieces + two reads).  hipcc still
  // counts the ds_reads and inserts the lgkmcnt waits before each MFMA that consumes one.
  f32x4 acc[8][8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  // read step s (0..7) of a k-step's 16 fragments: the 8 weight fragments first (every MFMA row
  // needs all of them), then the activation fragments in row order — so the rows of the next
  // half find their operands landed well before they issue
  auto rd = [&](int t, int kk, int s, bf16x8 (&af)[8], bf16x8 (&bf)[8]) {
    const char* base = smem + (t & 1) * kW4Stage;
    if (s < 4) {
      bf[2 * s] = *reinterpret_cast<const bf16x8*>(base + b_lane + (2 * s) * 2048 + sch[kk]);
      bf[2 * s + 1] = *reinterpret_cast<const bf16x8*>(base + b_lane + (2 * s + 1) * 2048 + sch[kk]);
    } else {
      const int i = 2 * (s - 4);
      af[i] = *reinterpret_cast<const bf16x8*>(base + a_lane + i * 2048 + sch[kk]);
      af[i + 1] = *reinterpret_cast<const bf16x8*>(base + a_lane + (i + 1) * 2048 + sch[kk]);
    }
  };
  auto row = [&](int i, const bf16x8 (&af)[8], const bf16x8 (&bf)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                   : "+a"(acc[i][j]) : "v"(bf[j]), "v"(af[i]));
  };
  auto row0 = [&](int i, const bf16x8 (&af)[8], const bf16x8 (&bf)[8]) {   // C = 0
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                   : "=a"(acc[i][j]) : "v"(bf[j]), "v"(af[i]));
  };
  auto dma = [&](int slot, int t, int j) {   // piece j (rows j*32 ..) of both operands
    char* dst = smem + slot * kW4Stage + wave * 1024 + j * 4096;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)dst, 16, voff, j * 32 * Kb + t * 128,
                                             0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)(dst + 32768), 16, voff,
                                             j * 32 * Kb + t * 128, 0, 0);
  };

  // ---- prologue: tiles 0 and 1 in flight, tile 0 landed; kk = 0 of tile 0 read, then the
  // first half of tile 0 (kk = 1 reads beside the kk = 0 MFMAs, which start from C = 0).
  // Past the last k-tile the re-stage index is clamped (re-loads tile T-1 into the freed slot,
  // which nothing reads) so the loop body is branch-free; the last half-iteration is peeled. ----
  if (T <= 0) return;   // uniform: never taken for a valid launch (every split owns >= 1 k-tile)
  if constexpr (NS >= 3) {
    // ---- 32-wide k-steps: step x lives in slot x % NS as A [256][64 B] | B [256][64 B]; a
    // 1 KB DMA piece p (0..15) of an operand = rows 16p .. 16p+15, wave w issues p = 4j + w.
    // Source chunk (l & 3) ^ ((l >> 4) & 3) (= chunk ^ (row >> 2) & 3): conflict-free reads.
    // Iteration s: wait own DMA(s+1) -> barrier -> DMA(s+NS-1) into the slot of step s-1 (read
    // in iteration s-2, consumed by MFMAs of s-1) -> read fragments of step s+1 -> MFMAs of s.
    const int S = 2 * T;
    const int voff2 = (lane >> 2) * Kb + (((lane & 3) ^ ((lane >> 4) & 3)) << 4) + kt0 * 128;
    const int a2 = (wr * 128 + fr) * 64, b2 = 16384 + (wc * 128 + fr) * 64;
    const int sw2 = (((lane >> 4) ^ (fr >> 2)) & 3) << 4;
    auto dma2 = [&](int x, int j) {   // piece 4j + wave of both operands of step min(x, S-1)
      const int xs = min(x, S - 1);
      char* dst = smem + (x % NS) * 32768 + (4 * j + wave) * 1024;
      const int so = (4 * j + wave) * 16 * Kb + xs * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_t*)dst, 16, voff2, so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void_t*)(dst + 16384), 16, voff2, so, 0, 0);
    };
    auto rd2 = [&](int x, int st, bf16x8 (&af)[8], bf16x8 (&bf)[8]) {   // read step st of 8
      const char* base = smem + (min(x, S - 1) % NS) * 32768;
      if (st < 4) {
        bf[2 * st] = *reinterpret_cast<const bf16x8*>(base + b2 + (2 * st) * 1024 + sw2);
        bf[2 * st + 1] = *reinterpret_cast<const bf16x8*>(base + b2 + (2 * st + 1) * 1024 + sw2);
      } else {
        const int i = 2 * (st - 4);
        af[i] = *reinterpret_cast<const bf16x8*>(base + a2 + i * 1024 + sw2);
        af[i + 1] = *reinterpret_cast<const bf16x8*>(base + a2 + (i + 1) * 1024 + sw2);
      }
    };
    auto iter = [&](int x, bool first, const bf16x8 (&ac)[8], const bf16x8 (&bc)[8],
                    bf16x8 (&an)[8], bf16x8 (&bn)[8]) {
      // own DMA(x+1) landed: DMA(x+2 .. x+NS-2) (8 loads per step) may stay in flight
      if (NS == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (NS == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      if (NS == 5) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      w4_barrier();
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i < 4) dma2(x + NS - 1, i);
        rd2(x + 1, i, an, bn);
        if (first) row0(i, ac, bc); else row(i, ac, bc);
      }
    };
#pragma unroll
    for (int x = 0; x < NS - 1; ++x)
#pragma unroll
      for (int j = 0; j < 4; ++j) dma2(x, j);
    // step 0 landed (NS - 2 later steps stay in flight)
    if (NS == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    if (NS == 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    if (NS == 5) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    w4_barrier();
#pragma unroll
    for (int st = 0; st < 8; ++st) rd2(0, st, a0, b0);
    iter(0, true, a0, b0, a1, b1);
    iter(1, false, a1, b1, a0, b0);
    for (int t = 1; t < T; ++t) {
      iter(2 * t, false, a0, b0, a1, b1);
      iter(2 * t + 1, false, a1, b1, a0, b0);
    }
  } else {
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, 0, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, min(1, T - 1), j);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  w4_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) rd(0, 0, i, a0, b0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    rd(0, 1, i, a1, b1);
    row0(i, a0, b0);
  }
  for (int t = 0; t < T - 1; ++t) {
    // own DMA of tile t+1 landed and own reads of slot t & 1 done -> after the barrier every
    // wave's part of tile t+1 is visible and slot t & 1 is free for tile t+2
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    w4_barrier();
    const int tn2 = min(t + 2, T - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // second half of tile t: kk = 1 MFMAs
      dma(t & 1, tn2, i);
      rd(t + 1, 0, i, a0, b0);
      row(i, a1, b1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // first half of tile t+1: kk = 0 MFMAs
      rd(t + 1, 1, i, a1, b1);
      row(i, a0, b0);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) row(i, a1, b1);
  }
  // the last MFMAs' results -> compiler-issued reads: 8-pass XDL needs 12 wait states before
  // any reader; the fence statements take every accumulator "+a" so no read is hoisted above
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]),
                 "+a"(acc[i][4]), "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));

#ifdef GEMM_STAMPS
  if (tid == 0) {
    unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
    st[6] = __builtin_amdgcn_s_memrealtime();
    st[7] = __builtin_amdgcn_s_memtime();
  }
#endif
  // ---- epilogue: fragment (i, j) element e of lane l is C[m0 + wr*128 + 16 i + (l & 15)]
  //      [n0 + wc*128 + 16 j + 4 (l >> 4) + e] ----
  const int crow = m0 + wr * 128 + fr;
  const int cq = 4 * (lane >> 4);
  if (EPI == kW4SwiGLU) {
    bf16* out = reinterpret_cast<bf16*>(C);
    const int I = N >> 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float g = (float)(bf16)acc[i][2 * p][e];   // round like GEMM -> silu_mul
          const float u = (float)(bf16)acc[i][2 * p + 1][e];
          o[e] = (bf16)(w4_silu(g) * u);
        }
        *reinterpret_cast<bf16x4*>(out + (size_t)row * I + (n0 >> 1) + wc * 64 + p * 16 + cq) = o;
      }
    }
  } else if (EPI == kW4F32) {
    float* out = reinterpret_cast<float*>(C) + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<f32x4*>(out + (size_t)row * N + n0 + wc * 128 + j * 16 + cq) = acc[i][j];
    }
  } else {
    bf16* out = reinterpret_cast<bf16*>(C);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)acc[i][j][e];
        *reinterpret_cast<bf16x4*>(out + (size_t)row * N + n0 + wc * 128 + j * 16 + cq) = o;
      }
    }
  }
#ifdef GEMM_STAMPS
  if (tid == 0) {
    unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
    st[2] = __builtin_amdgcn_s_memrealtime();
    st[3] = __builtin_amdgcn_s_memtime();
  }
#endif

}

}  // namespace

// C = A . B^T on the 4-wave kernel.  splits > 1: fp32 partials [splits, M, N] into `workspace`
// (epilogue must be 1 = partials only: the consumer reduces them); epilogue 2 = fused SwiGLU
// (B rows in swiglu_interleave order for wave column width 128, C is [M, N / 2]).
template <int NS>
int launch_w4(void* C, const void* A, const void* B, float* workspace, int M, int N, int K,
              int splits, int epilogue, hipStream_t stream) {
  if (M <= 0 || N % 256 != 0 || (K * 2) % 128 != 0 || splits < 1) return -1;
  const int kt = K * 2 / 128;
  if (splits > kt) return -2;
  const int kps = (kt + splits - 1) / splits;
  if ((splits - 1) * kps >= kt) return -2;
  if ((size_t)256 * K * 2 >= (1ull << 31)) return -3;   // 32-bit buffer offsets
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256;
  const int grid = tiles_m * tiles_n * splits;
  if (splits > 1) {
    if (workspace == nullptr || epilogue != kW4F32) return -4;
    gemm_w4_kernel<kW4F32, NS><<<grid, kW4Threads, 0, stream>>>(
        (const bf16*)A, (const bf16*)B, workspace, M, N, K, tiles_m, tiles_n, kps);
  } else if (epilogue == kW4SwiGLU) {
    gemm_w4_kernel<kW4SwiGLU, NS><<<grid, kW4Threads, 0, stream>>>(
        (const bf16*)A, (const bf16*)B, C, M, N, K, tiles_m, tiles_n, kps);
  } else if (epilogue == kW4Bf16) {
    gemm_w4_kernel<kW4Bf16, NS><<<grid, kW4Threads, 0, stream>>>(
        (const bf16*)A, (const bf16*)B, C, M, N, K, tiles_m, tiles_n, kps);
  } else {
    return -4;
  }
  return 0;
}

int launch_gemm_w4(void* C, const void* A, const void* B, float* workspace, int M, int N, int K,
                   int splits, int epilogue, hipStream_t stream, int pipe) {
  switch (pipe) {
    case 2: return launch_w4<2>(C, A, B, workspace, M, N, K, splits, epilogue, stream);
    case 3: return launch_w4<3>(C, A, B, workspace, M, N, K, splits, epilogue, stream);
    case 4: return launch_w4<4>(C, A, B, workspace, M, N, K, splits, epilogue, stream);
    case 5: return launch_w4<5>(C, A, B, workspace, M, N, K, splits, epilogue, stream);
  }
  return -9;
}

}  // namespace dli
