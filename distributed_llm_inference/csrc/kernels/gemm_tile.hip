// Projection GEMM for CDNA4:  C[M, N] = A[M, K] . B[N, K]^T   (bf16 in, fp32 accumulate)
//
// The decode step of a pipeline stage multiplies a micro-batch of activations (M = 256..512 rows)
// by each weight matrix (fused QKV, O, gate|up, down).  This kernel is the 256 x 256 x 64,
// 8-wave, LDS-DMA-staged, 8-phase MFMA structure of cdna_hip_programming.md §5 ("The 256² 8-phase
// template"), written for the NT layout both operands have here (A = activations [M, K] and
// B = nn.Linear weight [N, K], both K-contiguous):
//
//   * workgroup = 8 waves as 2 (M) x 4 (N); wave tile 128 x 64 = 8 x 4 fragments of
//     v_mfma_f32_16x16x32_bf16 (128 fp32 accumulators per lane);
//   * each 256 x 64 operand tile is staged as two 128-row HALF-TILES; half h of A holds the rows
//     the waves' m-quadrant h uses (tile rows {r : (r % 128) / 64 == h}), half h of B the columns
//     of their n-quadrant h ({c : (c % 64) / 32 == h}).  One half-tile = 16 KB = two
//     `global_load_lds_dwordx4` per thread, lane-linear in LDS; the XOR swizzle
//     chunk ^ ((row >> 1) & 7) is applied to the per-lane GLOBAL address (LDS-DMA cannot scatter)
//     and makes every fragment `ds_read_b128` conflict-free (docs/kernels.md derivation);
//   * per k-tile 4 phases, one output quadrant (64 x 32, 16 MFMAs) each:
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
//   * split-K partials are reduced by a separate full-chip pass: an in-launch stream-K fix-up
//     (last-arriving workgroup sums the other partials) was measured 20-70 % slower on these
//     shapes — a 256 KB fp32 partial tile is far past what one CU's ~100 GB/s read path
//     reduces cheaply (§5 "In-launch split-K reduction": worth it at tens of KB per tile);
//   * 1-byte operands (same staging: a k-tile is 128 bytes per row): fp8 e4m3 on the block-scaled
//     K=128 MFMA (2x the bf16 rate, unit block scales) and int8 on v_mfma_i32_16x16x64_i8 (LLM.int8
//     weights); per-row / per-channel scales are applied in the epilogue;
//   * epilogues: bf16 store, fp32 split-K slab (summed by `splitk_reduce`), or fused SwiGLU:
//     with B's rows interleaved by `swiglu_interleave` (gate and up rows of the same output
//     column land in n-fragments 2p and 2p+1 of one wave) the wave holds gate and up of an output
//     element in the same lane and register, and stores silu(gate) * up directly.
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

// FP8 / INT8: A and B are 1-byte elements (K counted in elements = bytes) with fp32 a_scale[M]
// (per row) and b_scale[N] (per output channel).  Staging is byte-identical to bf16: a k-tile is
// 128 bytes of every row (64 bf16, 128 fp8 / int8).
template <int EPI, int PREC>
__global__ void __launch_bounds__(kThreads, 1)
gemm_tile_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, void* __restrict__ C,
                 const float* __restrict__ a_scale, const float* __restrict__ b_scale,
                 int M, int N, int K, int tiles_m, int tiles_n, int k_tiles_per_split) {
  constexpr bool FP8 = PREC == kFp8;
  constexpr bool BYTES = PREC != kBf16;   // 1-byte operands
  const char* A = reinterpret_cast<const char*>(Av);
  const char* B = reinterpret_cast<const char*>(Bv);
  const size_t Kb = (size_t)K * (BYTES ? 1 : 2);   // row stride in bytes
  __shared__ __attribute__((aligned(1024))) char smem[kLds];

  // ---- XCD-aware, bijective block remap (consecutive logical ids share an XCD / its L2) ----
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = lid % tiles_m;               // the M tiles of one N panel are neighbours:
  const int tn = (lid / tiles_m) % tiles_n;   // they share the streamed weight panel via L2
  const int split = lid / (tiles_m * tiles_n);
  const int m0 = tm * kTM, n0 = tn * kTN;
  const int kt0 = split * k_tiles_per_split;
  const int T = min(k_tiles_per_split, (int)(Kb / 128) - kt0);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  // ---- DMA source rows: thread stages LDS units u = j*512 + tid (j = 0, 1) of each half-tile ----
  // unit u -> local row lr = u >> 3, LDS slot s = u & 7, global chunk s ^ ((lr >> 1) & 7)
  const char* srcA[2][2];
  const char* srcB[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int u = j * kThreads + tid;
    const int lr = u >> 3, ch = (u & 7) ^ ((lr >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ga = (lr >> 6) * 128 + h * 64 + (lr & 63);
      const int gb = (lr >> 5) * 64 + h * 32 + (lr & 31);
      const int ra = min(m0 + ga, M - 1);       // rows past M are computed, never stored
      srcA[h][j] = A + (size_t)ra * Kb + (size_t)kt0 * 128 + ch * 16;
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

  // ---- fragment read offsets (lane constant part; ds_read immediates do the rest) ----
  const int fr = lane & 15;
  int sch[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) sch[kk] = ((kk * 4 + (lane >> 4)) ^ (fr >> 1)) << 4;
  const int a_lane = (wr * 64 + fr) * 128;
  const int b_lane = (wc * 32 + fr) * 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  auto read_a = [&](const char* buf, int h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[i][kk] = *reinterpret_cast<const bf16x8*>(buf + h * kHalf + a_lane + i * 16 * 128 + sch[kk]);
  };
  auto read_b = [&](const char* buf, int h, bf16x8 (&bf)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bf[j][kk] = *reinterpret_cast<const bf16x8*>(buf + (2 + h) * kHalf + b_lane + j * 16 * 128 + sch[kk]);
  };
  auto quadrant = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
    if (FP8) {
      // one K=128 MFMA per fragment pair: the two 16-B chunks (g, g+4) of the 128-B k-tile row
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + i][nq * 2 + j] = mfma_fp8(bf[j][0], bf[j][1], af[i][0], af[i][1],
                                                 acc[mq * 4 + i][nq * 2 + j]);
    } else if (PREC == kInt8) {
      // two K=64 int8 MFMAs per k-tile (16-B chunks g and g+4), like the two bf16 k-steps
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq * 4 + i][nq * 2 + j] = mfma_i8(bf[j][kk], af[i][kk], acc[mq * 4 + i][nq * 2 + j]);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq * 4 + i][nq * 2 + j] = mfma(bf[j][kk], af[i][kk], acc[mq * 4 + i][nq * 2 + j]);
    }
    __builtin_amdgcn_s_setprio(0);
  };

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

  // the two wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7, one of each per SIMD) run one
  // barrier apart, so every SIMD alternates one wave's MFMA segment with the other's LDS reads
  if (wr == 1) barrier();
  for (int t = 0; t < T; ++t) {
    const char* buf = smem + (t & 1) * kBuf;
    const bool more1 = t + 1 < T, more2 = t + 2 < T;
    // phase 0: quadrant (0, 0)
    read_a(buf, 0);
    read_b(buf, 0, b0);
    if (more1) stage(1, t + 1);
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    quadrant(0, 0, b0);
    barrier();
    // phase 1: quadrant (0, 1)
    read_b(buf, 1, b1);
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    quadrant(0, 1, b1);
    barrier();
    // phase 2: quadrant (1, 1); A-half 0 was last read two phases ago
    read_a(buf, 1);
    if (more2) stage(0, t + 2);
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    quadrant(1, 1, b1);
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
    quadrant(1, 0, b0);
    barrier();
  }
  if (wr == 0) barrier();

  // ---- epilogue ----
  // The MFMAs compute the transposed tile (A operand = weight rows): fragment (i, j) element e of
  // lane l is C[row = 16 i + (l & 15)][col = 16 j + 4 (l >> 4) + e], so each lane owns 4
  // consecutive output columns of one row -> 8-B (bf16) / 16-B (fp32) vector stores.
  const int crow = m0 + wr * 128 + fr;
  const int cq = 4 * (lane >> 4);
  if (BYTES) {  // dequantise: per-row activation scale x per-output-channel weight scale
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sa = a_scale[min(crow + i * 16, M - 1)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 sb = *reinterpret_cast<const f32x4*>(b_scale + n0 + wc * 64 + j * 16 + cq);
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
    // n-fragments (2p, 2p+1) = (gate, up) of output columns n0/2 + wc*32 + p*16 + cq + e
    bf16* out = reinterpret_cast<bf16*>(C);
    const int I = N >> 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // round gate and up to bf16 first: matches the unfused GEMM -> silu_mul path
          const float g = (float)(bf16)acc[i][2 * p][e];
          const float u = (float)(bf16)acc[i][2 * p + 1][e];
          o[e] = (bf16)(silu(g) * u);
        }
        *reinterpret_cast<bf16x4*>(out + (size_t)row * I + (n0 >> 1) + wc * 32 + p * 16 + cq) = o;
      }
    }
  } else if (EPI == kStoreF32) {
    float* out = reinterpret_cast<float*>(C) + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(out + (size_t)row * N + n0 + wc * 64 + j * 16 + cq) = acc[i][j];
    }
  } else {
    bf16* out = reinterpret_cast<bf16*>(C);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = crow + i * 16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)acc[i][j][e];
        *reinterpret_cast<bf16x4*>(out + (size_t)row * N + n0 + wc * 64 + j * 16 + cq) = o;
      }
    }
  }
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

template <int PREC>
int launch_tile(void* C, const void* A, const void* B, const float* sa, const float* sb,
                float* workspace, int M, int N, int K, int splits, int epilogue,
                hipStream_t stream) {
  constexpr int esz = PREC == kBf16 ? 2 : 1;
  const int kt = (int)((size_t)K * esz / 128);
  if (M <= 0 || N % kTN != 0 || (size_t)K * esz % 128 != 0 || splits < 1) return -1;
  if (splits > kt) return -2;
  const int kps = (kt + splits - 1) / splits;
  if ((splits - 1) * kps >= kt) return -2;   // every split owns at least one k-tile
  if (splits > 1 && (workspace == nullptr || epilogue != kStoreBf16)) return -3;
  if (PREC != kBf16 && (sa == nullptr || sb == nullptr)) return -5;
  const int tiles_m = (M + kTM - 1) / kTM, tiles_n = N / kTN;
  const int grid = tiles_m * tiles_n * splits;
  if (splits > 1) {
    gemm_tile_kernel<kStoreF32, PREC><<<grid, kThreads, 0, stream>>>(A, B, workspace, sa, sb, M, N,
                                                                    K, tiles_m, tiles_n, kps);
    const size_t MN = (size_t)M * N;
    size_t blocks = (MN / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    tile_splitk_reduce_kernel<<<(int)blocks, 256, 0, stream>>>(reinterpret_cast<bf16*>(C),
                                                               workspace, splits, MN);
  } else if (epilogue == kSwiGLU) {
    gemm_tile_kernel<kSwiGLU, PREC><<<grid, kThreads, 0, stream>>>(A, B, C, sa, sb, M, N, K, tiles_m,
                                                                  tiles_n, kps);
  } else if (epilogue == kStoreBf16) {
    gemm_tile_kernel<kStoreBf16, PREC><<<grid, kThreads, 0, stream>>>(A, B, C, sa, sb, M, N, K,
                                                                     tiles_m, tiles_n, kps);
  } else {
    return -4;
  }
  return 0;
}

}  // namespace

int launch_gemm_tile(void* C, const void* A, const void* B, const float* a_scale,
                     const float* b_scale, float* workspace, int M, int N, int K, int splits,
                     int epilogue, int precision, hipStream_t stream) {
  switch (precision) {
    case kBf16:
      return launch_tile<kBf16>(C, A, B, nullptr, nullptr, workspace, M, N, K, splits, epilogue,
                                stream);
    case kFp8:
      return launch_tile<kFp8>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue,
                               stream);
    case kInt8:
      return launch_tile<kInt8>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue,
                                stream);
  }
  return -6;
}

}  // namespace dli
