// Projection GEMM for CDNA4:  C[M, N] = A[M, K] . B[N, K]^T   (bf16 in, fp32 accumulate)
//
// The decode step of a pipeline stage multiplies a micro-batch of activations (M = 256..512 rows)
// by each weight matrix (fused QKV, O, gate|up, down).  This kernel is the 8-wave, LDS-DMA-staged,
// 8-phase MFMA structure of cdna_hip_programming.md §5 ("The 256² 8-phase template"), written for
// the NT layout both operands have here (A = activations [M, K] and B = nn.Linear weight [N, K],
// both K-contiguous), with a variable tile width:
//
//   * tile 256 (M) x BN (N), BN = 32 NF for NF = 4..8 n-fragments per wave (BN 128..256).  The
//     width is a per-shape choice (ops.tile_gemm_plan): the decode GEMMs are power-bound, and the
//     lever is whole waves of tiles — Llama-3-70B gate|up at M = 512 has 448 256-wide tiles
//     (1.75 waves on 256 CUs) but 512 224-wide ones (2 full waves), which is also the tile
//     hipBLASLt picks for that shape;
//   * workgroup = 8 waves as 4 (M) x 2 (N); wave tile 64 x 16 NF = 4 x NF fragments of
//     v_mfma_f32_16x16x32_bf16 (16 NF fp32 accumulators per lane);
//   * each 256 x 64 operand tile is staged as two 128-row HALF-TILES; half h of A holds the rows
//     the waves' m-quadrant h uses, half q of B the rows of their n-quadrant q (NF odd: the second
//     one is shorter).  One half-tile = 16 KB = two `global_load_lds_dwordx4` per thread,
//     lane-linear in LDS; the XOR swizzle chunk ^ ((row >> 1) & 7) is applied to the per-lane
//     GLOBAL address (LDS-DMA cannot scatter) and makes every fragment `ds_read_b128`
//     conflict-free (docs/kernels.md derivation);
//   * per k-tile 4 phases, one output quadrant each:
//        phase 0: read A-half 0 + B-half 0 fragments | DMA A-half 1 of tile t+1
//        phase 1: read B-half 1                      |
//        phase 2: read A-half 1                      | DMA A-half 0 of tile t+2 (same buffer)
//        phase 3: (reuse B-half 0 registers)         | DMA B-halves 0, 1 of tile t+2; vmcnt(6)
//     so three half-tiles stay in flight across every barrier (counted `s_waitcnt vmcnt(6)`,
//     never 0 in the steady state);
//   * the two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one barrier apart
//     (§5 "if (wr == 1) s_barrier"): each SIMD alternates one wave's MFMA segment with the other
//     wave's ds_reads and DMA issue.  With that stagger a half-tile is restaged >= 2 phases after
//     its last ds_read (WAR across the lagging group) and read >= 1 phase after the vmcnt that
//     retired its DMA (RAW across the leading group);
//   * raw `s_barrier` (no __syncthreads: its fence would drain the DMA queue) and one __shared__
//     array (a second one makes hipcc wait vmcnt(0) before the first ds_read of every phase);
//   * blockIdx is remapped so the blocks of one XCD run neighbouring tiles (§5.5 T1, bijective);
//   * the MFMAs take the weight fragment as the A operand, so the accumulator holds the tile
//     transposed and every lane owns 4 consecutive output columns (vector stores);
//   * split-K partials are reduced by the consumer (rms_norm_splitk, rope_cache) or by a separate
//     full-chip pass; an in-launch fix-up was measured 20-70 % slower on these shapes, and a
//     stream-K tail for the partial last wave was neutral inside the decode step (both removed;
//     profiles/stream_k_decode_ab.txt);
//   * 1-byte operands (same staging: a k-tile is 128 bytes of every row): fp8 e4m3 on the
//     block-scaled K=128 MFMA (2x the bf16 rate, unit block scales) and int8 on
//     v_mfma_i32_16x16x64_i8 (LLM.int8 weights); per-row / per-channel scales in the epilogue;
//   * epilogues: bf16 store, fp32 split-K slab, or fused SwiGLU: with B's rows pairwise
//     interleaved by `swiglu_interleave` (row 2c = gate c, row 2c+1 = up c) every lane holds gate
//     and up of two output columns in adjacent accumulator registers and stores silu(g) * u.
//
// A 4-wave variant (128 x 128 per wave, 256 AGPR accumulators, one wave per SIMD) was built and
// measured bit-identical but 1-23 % slower: a single wave per SIMD cannot hide its own LDS-DMA
// issue behind its MFMAs (~3150 vs 2900 cycles per k-tile; profiles/gemm_w4_ab.txt).
#include "kernels.h"

namespace dli {

namespace {

constexpr int kTM = 256, kTN = 256, kTK = 64, kThreads = 512;
constexpr int kHalf = 128 * 128;       // bytes of one half-tile (128 rows x 64 bf16)
constexpr int kBuf = 4 * kHalf;        // A0 A1 B0 B1
constexpr int kLds = 2 * kBuf;         // double buffer: 128 KB

enum Epilogue { kStoreBf16 = 0, kStoreF32 = 1, kSwiGLU = 2 };


typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void dma16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

typedef int i32x8 __attribute__((ext_vector_type(8)));

// fp8 e4m3 x fp8 e4m3 -> fp32, K = 128, through the block-scaled MFMA (2x the bf16 rate on
// gfx950; the plain fp8 16x16x32 form only runs at the bf16 rate).  Block scales are all 1.0
// (e8m0 127): the per-row activation and per-channel weight scales are applied in the epilogue.
// Both operands are read with the same lane/byte pattern, so the products pair the same k.
__device__ __forceinline__ f32x4 mfma_fp8(const bf16x8& a0, const bf16x8& a1, const bf16x8& b0,
                                          const bf16x8& b1, const f32x4& c) {
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  const i32x4_t al = __builtin_bit_cast(i32x4_t, a0), ah = __builtin_bit_cast(i32x4_t, a1);
  const i32x4_t bl = __builtin_bit_cast(i32x4_t, b0), bh = __builtin_bit_cast(i32x4_t, b1);
  const i32x8 a = {al[0], al[1], al[2], al[3], ah[0], ah[1], ah[2], ah[3]};
  const i32x8 b = {bl[0], bl[1], bl[2], bl[3], bh[0], bh[1], bh[2], bh[3]};
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// int8 x int8 -> int32, K = 64 (2x the bf16 rate); the accumulator registers hold int32 bits.
__device__ __forceinline__ f32x4 mfma_i8(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(
      __builtin_bit_cast(i32x4_t, a), __builtin_bit_cast(i32x4_t, b),
      __builtin_bit_cast(i32x4_t, c), 0, 0, 0));
}

enum Prec { kBf16 = 0, kFp8 = 1, kInt8 = 2 };

#ifdef GEMM_STAMPS
// Diagnostic build only (scripts/gemm_stamps.hip, scripts/gemm_w4_bench.hip): per-workgroup clock
// stamps (begin/end shader cycles and 100 MHz wall ticks, end of the main loop).  Never compiled
// into the extension.
__device__ unsigned long long* g_stamp_blk;   // [grid][8]
#endif

// FP8 / INT8: A and B are 1-byte elements (K counted in elements = bytes) with fp32 a_scale[M]
// (per row) and b_scale[N] (per output channel).  Staging is byte-identical to bf16: a k-tile is
// 128 bytes of every row (64 bf16, 128 fp8 / int8).
//
// NF = n-fragments per wave: tile 256 x BN with BN = 32 * NF; n-quadrant 0 holds fragments
// [0, NF0), n-quadrant 1 [NF0, NF), NF0 = ceil(NF / 2).
template <int EPI, int PREC, int NF>
__global__ void __launch_bounds__(kThreads, 1)
gemm_tile_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, void* __restrict__ C,
                 const float* __restrict__ a_scale, const float* __restrict__ b_scale,
                 int M, int N, int K, int tiles_m, int tiles_n, int k_tiles_per_split) {
  constexpr bool FP8 = PREC == kFp8;
  constexpr bool BYTES = PREC != kBf16;   // 1-byte operands
  constexpr int NF0 = (NF + 1) / 2, NF1 = NF - NF0;
  constexpr int BN = 32 * NF;
  const char* A = reinterpret_cast<const char*>(Av);
  const char* B = reinterpret_cast<const char*>(Bv);
  const size_t Kb = (size_t)K * (BYTES ? 1 : 2);   // row stride in bytes
  const int kt_all = (int)(Kb / 128);              // k-tiles of a whole tile
  __shared__ __attribute__((aligned(1024))) char smem[kLds];

  const int tid = threadIdx.x;
#ifdef GEMM_STAMPS
  if (tid == 0) {
    unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
    st[0] = __builtin_amdgcn_s_memrealtime();
    st[1] = __builtin_amdgcn_s_memtime();
  }
#endif
  const int lane = tid & 63, wave = tid >> 6, fr = lane & 15;
  const int wr = wave >> 1, wc = wave & 1;   // 4 (M) x 2 (N) waves
  const int grp = wave >> 2;                 // stagger group: one wave of each per SIMD

  // ---- XCD-aware, bijective block remap (consecutive logical ids share an XCD / its L2) ----
  const int nb = gridDim.x, bx = blockIdx.x, x8 = bx & 7, q8 = nb >> 3, r8 = nb & 7;
  const int lid = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bx >> 3);
  const int tile = lid % (tiles_m * tiles_n);
  const int split = lid / (tiles_m * tiles_n);
  const int kt0 = split * k_tiles_per_split;
  const int T = min(k_tiles_per_split, kt_all - kt0);
  const int tm = tile % tiles_m;              // the M tiles of one N panel are neighbours:
  const int tn = tile / tiles_m;              // they share the streamed weight panel via L2
  const int m0 = tm * kTM, n0 = tn * BN;

  int sch[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) sch[kk] = ((kk * 4 + (lane >> 4)) ^ (fr >> 1)) << 4;
  const int a_lane = (wr * 32 + fr) * 128;
  const int b_lane0 = (wc * 16 * NF0 + fr) * 128;
  const int b_lane1 = (wc * 16 * NF1 + fr) * 128;

  // ---- DMA source rows: thread stages LDS units u = j*512 + tid (j = 0, 1) of each half-tile ----
  // unit u -> local row lr = u >> 3, LDS slot s = u & 7, global chunk s ^ ((lr >> 1) & 7).
  // A half h: local row lr -> tile row (lr >> 5) * 64 + h * 32 + (lr & 31) (the rows of m-quadrant
  // h of every wave row).  B half q: local row lr -> (lr / (16 NFq)) * 16 NF + q * 16 NF0 +
  // lr % (16 NFq); local rows past 32 NFq (NF odd: the short half) re-load a valid row into the
  // unused end of the slot, so every thread issues the same count (uniform vmcnt).
  const char* srcA[2][2];
  const char* srcB[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int u = j * kThreads + tid;
    const int lr = u >> 3, ch = (u & 7) ^ ((lr >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ga = (lr >> 5) * 64 + h * 32 + (lr & 31);
      const int ra = min(m0 + ga, M - 1);       // rows past M are computed, never stored
      srcA[h][j] = A + (size_t)ra * Kb + (size_t)kt0 * 128 + ch * 16;
      const int nfq = h == 0 ? NF0 : NF1;
      const int lrc = min(lr, 32 * nfq - 1);
      const int gb = (lrc / (16 * nfq)) * 16 * NF + h * 16 * NF0 + lrc % (16 * nfq);
      srcB[h][j] = B + (size_t)(n0 + gb) * Kb + (size_t)kt0 * 128 + ch * 16;
    }
  }
  // stage half `which` (0 = A0, 1 = A1, 2 = B0, 3 = B1) of k-tile t into buffer t & 1
  auto stage = [&](int which, int t) {
    char* dst = smem + (t & 1) * kBuf + which * kHalf + wave * 1024;
    const size_t koff = (size_t)t * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const char* src = which < 2 ? srcA[which][j] : srcB[which - 2][j];
      dma16(src + koff, dst + j * 8192);
    }
  };

  f32x4 acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[2][2], b0[NF0][2], b1[NF1][2];
  auto read_a = [&](const char* buf, int h) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[i][kk] = *reinterpret_cast<const bf16x8*>(buf + h * kHalf + a_lane + i * 2048 + sch[kk]);
  };
  auto read_b0 = [&](const char* buf) {
#pragma unroll
    for (int j = 0; j < NF0; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        b0[j][kk] = *reinterpret_cast<const bf16x8*>(buf + 2 * kHalf + b_lane0 + j * 2048 + sch[kk]);
  };
  auto read_b1 = [&](const char* buf) {
#pragma unroll
    for (int j = 0; j < NF1; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        b1[j][kk] = *reinterpret_cast<const bf16x8*>(buf + 3 * kHalf + b_lane1 + j * 2048 + sch[kk]);
  };
  auto quadrant = [&](int mq, auto& bf, auto nq_tag) {
    constexpr int NQ = decltype(nq_tag)::value;
    constexpr int NFQ = NQ == 0 ? NF0 : NF1;
    constexpr int J0 = NQ == 0 ? 0 : NF0;
    // the computing wave outranks its SIMD partner for the segment: 13-15 % faster than a
    // static priority for the lagging group or none (profiles/gemm_variants_ab.txt)
    __builtin_amdgcn_s_setprio(1);
    if (FP8) {
      // one K=128 MFMA per fragment pair: the two 16-B chunks (g, g+4) of the 128-B k-tile row
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NFQ; ++j)
          acc[mq * 2 + i][J0 + j] = mfma_fp8(bf[j][0], bf[j][1], af[i][0], af[i][1],
                                             acc[mq * 2 + i][J0 + j]);
    } else if (PREC == kInt8) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NFQ; ++j)
            acc[mq * 2 + i][J0 + j] = mfma_i8(bf[j][kk], af[i][kk], acc[mq * 2 + i][J0 + j]);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NFQ; ++j)
            acc[mq * 2 + i][J0 + j] = mfma(bf[j][kk], af[i][kk], acc[mq * 2 + i][J0 + j]);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;

  // ---- prologue: tile 0 complete, three halves of tile 1 in flight ----
  if (T > 0) {
    stage(0, 0); stage(2, 0); stage(3, 0); stage(1, 0);
    if (T > 1) {
      stage(0, 1); stage(2, 1); stage(3, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  barrier();

  // the two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one barrier apart, so every
  // SIMD alternates one wave's MFMA segment with the other's LDS reads
  if (grp == 1) barrier();
  for (int t = 0; t < T; ++t) {
    const char* buf = smem + (t & 1) * kBuf;
    const bool more1 = t + 1 < T, more2 = t + 2 < T;
    // phase 0: quadrant (0, 0)
    read_a(buf, 0);
    read_b0(buf);
    if (more1) stage(1, t + 1);
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    quadrant(0, b0, Q0{});
    barrier();
    // phase 1: quadrant (0, 1)
    read_b1(buf);
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    quadrant(0, b1, Q1{});
    barrier();
    // phase 2: quadrant (1, 1); A-half 0 was last read two phases ago
    read_a(buf, 1);
    if (more2) stage(0, t + 2);
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    quadrant(1, b1, Q1{});
    barrier();
    // phase 3: quadrant (1, 0); restage both B halves; retire tile t+1 (all but 3 newest halves)
    if (more2) {
      stage(2, t + 2);
      stage(3, t + 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    quadrant(1, b0, Q0{});
    barrier();
  }
  if (grp == 0) barrier();
#ifdef GEMM_STAMPS
  if (tid == 0) {
    unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
    st[6] = __builtin_amdgcn_s_memrealtime();
    st[7] = __builtin_amdgcn_s_memtime();
  }
#endif

  // ---- epilogue ----
  // The MFMAs compute the transposed tile (A operand = weight rows): fragment (i, j) element e of
  // lane l is C[row = m0 + 64 wr + 16 i + (l & 15)][col = n0 + 16 NF wc + 16 j + 4 (l >> 4) + e],
  // so each lane owns 4 consecutive output columns of one row -> 8-B (bf16) / 16-B (fp32) stores.
  const int crow = m0 + wr * 64 + fr;
  const int ccol = n0 + wc * 16 * NF + 4 * (lane >> 4);
  if (BYTES) {  // dequantise: per-row activation scale x per-output-channel weight scale
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float sa = a_scale[min(crow + i * 16, M - 1)];
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const f32x4 sb = *reinterpret_cast<const f32x4*>(b_scale + ccol + j * 16);
        f32x4 v = acc[i][j];
        if (PREC == kInt8) {
          typedef int i32x4_t __attribute__((ext_vector_type(4)));
          const i32x4_t iv = __builtin_bit_cast(i32x4_t, v);
          v = f32x4{(float)iv[0], (float)iv[1], (float)iv[2], (float)iv[3]};
        }
        acc[i][j] = v * sb * sa;
      }
    }
  }
  if (EPI == kSwiGLU) {
    // B rows pairwise interleaved (ops.swiglu_interleave): columns (2c, 2c+1) = (gate, up) of
    // output column c, so elements (0, 1) and (2, 3) of every fragment are one output each
    bf16* out = reinterpret_cast<bf16*>(C);
    const int I = N >> 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        bf16x2 o;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          // round gate and up to bf16 first: matches the unfused GEMM -> silu_mul path
          const float g = (float)(bf16)acc[i][j][2 * e];
          const float u = (float)(bf16)acc[i][j][2 * e + 1];
          o[e] = (bf16)(silu(g) * u);
        }
        *reinterpret_cast<bf16x2*>(out + (size_t)row * I + ((ccol + j * 16) >> 1)) = o;
      }
    }
  } else if (EPI == kStoreF32) {
    float* out = reinterpret_cast<float*>(C) + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < NF; ++j)
        *reinterpret_cast<f32x4*>(out + (size_t)row * N + ccol + j * 16) = acc[i][j];
    }
  } else {
    bf16* out = reinterpret_cast<bf16*>(C);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)acc[i][j][e];
        *reinterpret_cast<bf16x4*>(out + (size_t)row * N + ccol + j * 16) = o;
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

__global__ void __launch_bounds__(256) tile_splitk_reduce_kernel(bf16* __restrict__ C,
                                                                 const float* __restrict__ part,
                                                                 int splits, size_t MN) {
  for (size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * 8; i < MN;
       i += (size_t)gridDim.x * blockDim.x * 8) {
    f32x4 s0 = *reinterpret_cast<const f32x4*>(part + i);
    f32x4 s1 = *reinterpret_cast<const f32x4*>(part + i + 4);
    for (int k = 1; k < splits; ++k) {
      s0 += *reinterpret_cast<const f32x4*>(part + k * MN + i);
      s1 += *reinterpret_cast<const f32x4*>(part + k * MN + i + 4);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (bf16)s0[j];
      o[j + 4] = (bf16)s1[j];
    }
    *reinterpret_cast<bf16x8*>(C + i) = o;
  }
}

template <int PREC, int NF>
int launch_tile_nf(void* C, const void* A, const void* B, const float* sa, const float* sb,
                   float* workspace, int M, int N, int K, int splits, int epilogue,
                   hipStream_t stream) {
  constexpr int esz = PREC == kBf16 ? 2 : 1;
  constexpr int BN = 32 * NF;
  const int kt = (int)((size_t)K * esz / 128);
  if (M <= 0 || N % BN != 0 || (size_t)K * esz % 128 != 0 || splits < 1) return -1;
  if (splits > kt) return -2;
  if (PREC != kBf16 && (sa == nullptr || sb == nullptr)) return -5;
  const int tiles_m = (M + kTM - 1) / kTM, tiles_n = N / BN;
  const int kps = (kt + splits - 1) / splits;
  if ((splits - 1) * kps >= kt) return -2;   // every split owns at least one k-tile
  // kStoreF32 with splits > 1: partials only, the consumer reduces them (rms_norm_splitk)
  if (splits > 1 && (workspace == nullptr || epilogue == kSwiGLU)) return -3;
  if (splits == 1 && epilogue == kStoreF32) return -3;
  const int grid = tiles_m * tiles_n * splits;
  if (splits > 1) {
    gemm_tile_kernel<kStoreF32, PREC, NF><<<grid, kThreads, 0, stream>>>(
        A, B, workspace, sa, sb, M, N, K, tiles_m, tiles_n, kps);
    if (epilogue == kStoreF32) return 0;
    const size_t MN = (size_t)M * N;
    size_t blocks = (MN / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    tile_splitk_reduce_kernel<<<(int)blocks, 256, 0, stream>>>(reinterpret_cast<bf16*>(C),
                                                               workspace, splits, MN);
  } else if (epilogue == kSwiGLU) {
    gemm_tile_kernel<kSwiGLU, PREC, NF><<<grid, kThreads, 0, stream>>>(
        A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kps);
  } else if (epilogue == kStoreBf16) {
    gemm_tile_kernel<kStoreBf16, PREC, NF><<<grid, kThreads, 0, stream>>>(
        A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kps);
  } else {
    return -4;
  }
  return 0;
}

template <int PREC>
int launch_tile(void* C, const void* A, const void* B, const float* sa, const float* sb,
                float* workspace, int M, int N, int K, int splits, int epilogue, int bn,
                hipStream_t stream) {
  switch (bn) {
    case 128: return launch_tile_nf<PREC, 4>(C, A, B, sa, sb, workspace, M, N, K, splits, epilogue, stream);
    case 160: return launch_tile_nf<PREC, 5>(C, A, B, sa, sb, workspace, M, N, K, splits, epilogue, stream);
    case 192: return launch_tile_nf<PREC, 6>(C, A, B, sa, sb, workspace, M, N, K, splits, epilogue, stream);
    case 224: return launch_tile_nf<PREC, 7>(C, A, B, sa, sb, workspace, M, N, K, splits, epilogue, stream);
    case 256: return launch_tile_nf<PREC, 8>(C, A, B, sa, sb, workspace, M, N, K, splits, epilogue, stream);
  }
  return -11;
}

}  // namespace

int launch_splitk_reduce(bf16* C, const float* parts, int splits, size_t MN, hipStream_t stream) {
  if (splits < 1 || MN % 8 != 0) return -1;
  if (MN == 0) return 0;
  size_t blocks = (MN / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  tile_splitk_reduce_kernel<<<(int)blocks, 256, 0, stream>>>(C, parts, splits, MN);
  return 0;
}

int launch_gemm_tile(void* C, const void* A, const void* B, const float* a_scale,
                     const float* b_scale, float* workspace, int M, int N, int K, int splits,
                     int epilogue, int precision, hipStream_t stream, int bn) {
  switch (precision) {
    case kBf16:
      return launch_tile<kBf16>(C, A, B, nullptr, nullptr, workspace, M, N, K, splits, epilogue, bn,
                                stream);
    case kFp8:
      return launch_tile<kFp8>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue, bn,
                               stream);
    case kInt8:
      return launch_tile<kInt8>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue, bn,
                                stream);
  }
  return -6;
}

}  // namespace dli
