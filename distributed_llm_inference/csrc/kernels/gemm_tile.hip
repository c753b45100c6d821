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
//     element in the same lane and register, and stores silu(gate) * up directly;
//   * fp8 MX activations (kSwiGLUMx -> kFp8Mx): the fp8 gate|up SwiGLU epilogue quantises its
//     output itself, with one power-of-two (e8m0) scale per (row, 128-column block) — a block is
//     exactly one workgroup's 128 output columns, so the amax needs only an LDS reduction over its
//     4 n-waves — and the down projection feeds those scales to the block-scaled MFMA's per-lane
//     scale operand (each lane scales the 32 K-values it holds, opsel picks the byte), since a
//     128-column block is exactly one of its k-tiles.  That removes the separate per-row
//     quantisation pass over h and halves the epilogue's store bytes (fp8 instead of bf16).
#include "kernels.h"

namespace dli {

namespace {

constexpr int kTM = 256, kTN = 256, kTK = 64, kThreads = 512;
constexpr int kHalf = 128 * 128;       // bytes of one half-tile (128 rows x 64 bf16)
constexpr int kBuf = 4 * kHalf;        // A0 A1 B0 B1
constexpr int kLds = 2 * kBuf;         // double buffer: 128 KB

// kStoreBf16Part: split-K partials rounded to bf16 (half the partial bytes of kStoreF32 for the
// consumers that sum them; the default for every precision)
enum Epilogue { kStoreBf16 = 0, kStoreF32 = 1, kSwiGLU = 2, kSwiGLUMx = 3, kStoreBf16Part = 4 };

// stream-K workspace header: flags [0, kSkMaxWgs), error counter at kSkErrWord, slabs after
constexpr int kSkMaxWgs = 1020, kSkErrWord = 1023, kSkHeaderFloats = 1024;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void dma16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// non-temporal (cache policy NT): data streamed through once
__device__ __forceinline__ void dma16_nt(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 2);
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

enum Prec { kBf16 = 0, kFp8 = 1, kInt8 = 2, kFp8Mx = 3 };

// fp8 x fp8 with per-lane e8m0 scales on the activation operand: lane l's byte SEL of `sc` scales
// the 32 K-values it holds (row l & 15, K-block l >> 4) — mx_scale_probe.hip pins that mapping
template <int SEL>
__device__ __forceinline__ f32x4 mfma_fp8_mx(const bf16x8& a0, const bf16x8& a1, const bf16x8& b0,
                                             const bf16x8& b1, const f32x4& c, int sc) {
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  const i32x4_t al = __builtin_bit_cast(i32x4_t, a0), ah = __builtin_bit_cast(i32x4_t, a1);
  const i32x4_t bl = __builtin_bit_cast(i32x4_t, b0), bh = __builtin_bit_cast(i32x4_t, b1);
  const i32x8 a = {al[0], al[1], al[2], al[3], ah[0], ah[1], ah[2], ah[3]};
  const i32x8 b = {bl[0], bl[1], bl[2], bl[3], bh[0], bh[1], bh[2], bh[3]};
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, SEL, sc);
}

// e8m0 activation scales (MX): common.h mx_off layout (a k-tile of 128 fp8 = one scale block)
constexpr int kMxMaxKt = 64;             // k-tiles of scales a kFp8Mx workgroup keeps in LDS
constexpr int kMxLds = kMxMaxKt * 256;   // [k-tile][256 tile rows] bytes

struct MxArgs {
  const uint8_t* a_sc;   // kFp8Mx: the A operand's scales (mx_off layout)
  uint8_t* out_sc;       // kSwiGLUMx: scales of the quantised output (mx_off layout, kt = n-tile)
  int nb;                // ceil(M / 64)
};

// Stream-K tail (splits == 1, bf16 / SwiGLU epilogues).  With more tiles than CUs the last wave
// of whole tiles leaves CUs idle (Llama-3-70B gate|up at M = 512: 448 tiles = 1.75 waves on 256
// CUs).  Workgroups [0, n_dp) compute tiles [0, n_dp) whole (data-parallel part, a multiple of the
// CU count); workgroups [n_dp, n_dp + sk_wgs) split the k-tiles of the remaining tiles evenly
// (sk_wgs = CU count, so they are co-resident).  A tile whose k-range spans several workgroups is
// finished by the one holding its last k-tile: every other holder publishes its fp32 partial
// (write-through `sc1` slab stores, drained, then one relaxed agent-scope flag store) and the
// finisher polls each flag, acquires, and adds the slab to its accumulators before the epilogue
// (cdna_hip_programming.md §6 Guideline 16, R1 form).  Each workgroup runs its publishing piece
// FIRST and its finishing piece LAST, and never waits before it has published, so every wait is
// on a co-resident workgroup that is already past its own publish point (no deadlock, whatever
// the dispatch order).
struct SkArgs {
  int n_dp;          // workgroups computing whole tiles; == grid when the tail is off
  int sk_wgs;        // stream-K workgroups (0 = off)
  unsigned* flags;   // [sk_wgs] publish flags, zeroed by a memset node before every launch
  unsigned* err;     // spin-timeout counter (diagnostic; tests zero it once)
  float* slabs;      // [sk_wgs][256 * 256] fp32 partials in accumulator (register) order
  int gm = 8;        // M-tiles per group of the grouped tile order (measured best: 4-8)
};

// LLM.int8 outlier columns (int8 precision only): the bf16 product x_out [M, J] . w_out [N, J]^T
// of the J feature columns held out of the int8 quantisation is added to the dequantised tile in
// the epilogue (split 0 only, so a split-K sum counts it once), one bf16 MFMA k-step per 32
// columns with the fragments loaded straight from global memory (J <= 64: a few KB per tile).
struct OutlierArgs {
  const bf16* x;   // [M, J] activations of the outlier columns (zero-padded past the used ones)
  const bf16* w;   // [N, J] dequantised weight columns (zero-padded likewise)
  int J;           // multiple of 32; 0 = none
  // optional device count of the outlier columns actually selected (llm_int8_select): only the
  // first ceil(cnt / 32) k-steps are multiplied; columns past them may hold stale data
  const int* cnt;
};

typedef __attribute__((address_space(1))) unsigned gu32;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifdef GEMM_STAMPS
// Diagnostic builds only (scripts/experiments/gemm_stamps.hip, gemm_w4_bench.hip): per-workgroup
// clock stamps (begin / end shader cycles and 100 MHz wall ticks, end of the main loop).  Never
// compiled into the extension.
__device__ unsigned long long* g_stamp_blk;   // [grid][8]
#endif

// FP8 / INT8: A and B are 1-byte elements (K counted in elements = bytes) with fp32 a_scale[M]
// (per row) and b_scale[N] (per output channel).  Staging is byte-identical to bf16: a k-tile is
// 128 bytes of every row (64 bf16, 128 fp8 / int8).
// VAR bit 0 (whole-tile / split-K launches with tiles_m <= 2, i.e. decode micro-batches of
// <= 512 rows): the weight (B) half-tiles are loaded non-temporal — each weight byte is read by
// at most the two M-tiles of its panel, so keep the L2 for the re-read activation panels
// (down projection 203 -> 194 us, gate|up -0.6 %; at 8192^3, where B is re-read by 32 M-tiles,
// it costs 3 %: profiles/gemm_var_nt_group_ab.json)
template <int EPI, int PREC, bool SKT, int VAR = 0>
__global__ void __launch_bounds__(kThreads, 1)
gemm_tile_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, void* __restrict__ C,
                 const float* __restrict__ a_scale, const float* __restrict__ b_scale,
                 int M, int N, int K, int tiles_m, int tiles_n, int k_tiles_per_split, SkArgs sk,
                 OutlierArgs ol, MxArgs mx) {
  constexpr bool MX = PREC == kFp8Mx;
  constexpr bool FP8 = PREC == kFp8 || MX;
  constexpr bool BYTES = PREC != kBf16;   // 1-byte operands
  const char* A = reinterpret_cast<const char*>(Av);
  const char* B = reinterpret_cast<const char*>(Bv);
  const size_t Kb = (size_t)K * (BYTES ? 1 : 2);   // row stride in bytes
  const int kt_all = (int)(Kb / 128);              // k-tiles of a whole tile
  __shared__ __attribute__((aligned(1024))) char smem[kLds + (MX ? kMxLds : 0)];

  const int tid0 = threadIdx.x;
#ifdef GEMM_STAMPS
  if (tid0 == 0) {
    unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
    st[0] = __builtin_amdgcn_s_memrealtime();
    st[1] = __builtin_amdgcn_s_memtime();
  }
#endif

  // ---- XCD-aware, bijective block remap (consecutive logical ids share an XCD / its L2) ----
  auto remap = [](int b, int n) {
    const int x = b & 7, q = n >> 3, r = n & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  };
  // the stream-K hand-off is a separate instantiation: compiled into the whole-tile kernels it
  // pushed the allocator to 256 VGPRs + 104 B/lane of scratch spills in the main loop (bf16 store
  // and SwiGLU variants), which cost the plain kernels ~10 % (bf16 only: in the 1-byte variants
  // the hand-off code spills even on its own)
  constexpr bool kSk = SKT && PREC == kBf16 && EPI != kStoreF32;
  const bool is_sk = kSk && (int)blockIdx.x >= sk.n_dp;
  const int lid = is_sk ? remap(blockIdx.x - sk.n_dp, sk.sk_wgs) : remap(blockIdx.x, sk.n_dp);

  // ---- segments: one (tile, k-range) for data-parallel / split-K blocks; for a stream-K block
  // the tiles its k-iteration range [lo, hi) touches: the last one first (it may be a partial
  // that others wait for), the first one last (it may wait for its predecessors' partials) ----
  long long sk_total = 0, lo = 0, hi = 0;
  int first_t = 0, nseg = 1;
  if (is_sk) {
    sk_total = (long long)(tiles_m * tiles_n - sk.n_dp) * kt_all;
    lo = sk_total * lid / sk.sk_wgs;
    hi = sk_total * (lid + 1) / sk.sk_wgs;
    first_t = (int)(lo / kt_all);
    nseg = (int)((hi - 1) / kt_all) - first_t + 1;
  }

  for (int seg = 0; seg < nseg; ++seg) {
    // re-derive the lane-dependent addressing in every segment instead of keeping it live
    // across the loop (hoisted, it costs ~20 VGPRs the accumulators need)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = tid >> 6, wr = wave >> 2, wc = wave & 3, fr = lane & 15;
    int sch[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) sch[kk] = ((kk * 4 + (lane >> 4)) ^ (fr >> 1)) << 4;
    const int a_lane = (wr * 64 + fr) * 128;
    const int b_lane = (wc * 32 + fr) * 128;
    int tile, kt0, T, split = 0;
    bool publish = false, finish = false;
    long long tile_k0 = 0;
    if (!is_sk) {
      tile = lid % (tiles_m * tiles_n);
      split = lid / (tiles_m * tiles_n);
      kt0 = split * k_tiles_per_split;
      T = min(k_tiles_per_split, kt_all - kt0);
    } else {
      const int t = first_t + (nseg == 1 ? 0 : seg == 0 ? nseg - 1 : seg == nseg - 1 ? 0 : seg);
      tile_k0 = (long long)t * kt_all;
      const long long s0 = max(lo, tile_k0), s1 = min(hi, tile_k0 + kt_all);
      kt0 = (int)(s0 - tile_k0);
      T = (int)(s1 - s0);
      publish = s1 < tile_k0 + kt_all;   // stops short of the tile's end: hand the partial on
      finish = !publish && s0 > tile_k0; // ends the tile but did not start it: add predecessors'
      tile = sk.n_dp + t;
    }
    // grouped tile order: groups of (up to) 8 M-tiles x all N panels, M fastest inside a group,
    // so the 32 consecutive tiles an XCD runs share 8 activation and 4 weight panels through its
    // L2 (the M tiles of one N panel stay neighbours).  Identical to M-fastest order for
    // tiles_m <= 8 (every decode shape); 8192^3: 1296 -> 1386 TF (profiles/gemm_var_nt_group_ab.json)
    const int GM = sk.gm;
    const int gper = GM * tiles_n, grp = tile / gper, grem = tile % gper;
    const int gm = min(GM, tiles_m - grp * GM);
    const int tm = grp * GM + grem % gm;
    const int tn = grem / gm;
    const int m0 = tm * kTM, n0 = tn * kTN;

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
        if ((VAR & 1) != 0 && which >= 2)
          dma16_nt(src + koff, dst + j * 8192);
        else
          dma16(src + koff, dst + j * 8192);
      }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    bf16x8 af[4][2], b0[2][2], b1[2][2];
    int s_mx[2] = {0, 0};   // kFp8Mx: this lane's 4 row scales of A-half 0 / 1, current k-tile
    const char* sls = smem + kLds;   // kFp8Mx: [k-tile][256 rows] e8m0 scales
    int mx_t = 0;                    // kFp8Mx: k-tile (within this split) read_a is reading
    auto read_a = [&](const char* buf, int h) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          af[i][kk] = *reinterpret_cast<const bf16x8*>(buf + h * kHalf + a_lane + i * 16 * 128 + sch[kk]);
      if constexpr (MX)
        s_mx[h] = *reinterpret_cast<const int*>(sls + mx_t * 256 + wr * 128 + h * 64 + fr * 4);
    };
    auto read_b = [&](const char* buf, int h, bf16x8 (&bf)[2][2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          bf[j][kk] = *reinterpret_cast<const bf16x8*>(buf + (2 + h) * kHalf + b_lane + j * 16 * 128 + sch[kk]);
    };
    auto quadrant = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
      // the computing wave outranks its SIMD partner for the segment: 13-15 % faster than a
      // static priority for the lagging group or none; triple-buffering the weight half-tiles
      // (160 KB LDS, twice the DMA lead) buys nothing (profiles/gemm_variants_ab.txt)
      __builtin_amdgcn_s_setprio(1);
      if constexpr (MX) {
        // per-lane e8m0 activation scales: byte i of the half's dword = row block i
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int sc = s_mx[mq];
          acc[mq * 4 + 0][nq * 2 + j] = mfma_fp8_mx<0>(bf[j][0], bf[j][1], af[0][0], af[0][1], acc[mq * 4 + 0][nq * 2 + j], sc);
          acc[mq * 4 + 1][nq * 2 + j] = mfma_fp8_mx<1>(bf[j][0], bf[j][1], af[1][0], af[1][1], acc[mq * 4 + 1][nq * 2 + j], sc);
          acc[mq * 4 + 2][nq * 2 + j] = mfma_fp8_mx<2>(bf[j][0], bf[j][1], af[2][0], af[2][1], acc[mq * 4 + 2][nq * 2 + j], sc);
          acc[mq * 4 + 3][nq * 2 + j] = mfma_fp8_mx<3>(bf[j][0], bf[j][1], af[3][0], af[3][1], acc[mq * 4 + 3][nq * 2 + j], sc);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[mq * 4 + i][nq * 2 + j]));
      } else if (FP8) {
        // one K=128 MFMA per fragment pair: the two 16-B chunks (g, g+4) of the 128-B k-tile row
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq * 4 + i][nq * 2 + j] = mfma_fp8(bf[j][0], bf[j][1], af[i][0], af[i][1],
                                                   acc[mq * 4 + i][nq * 2 + j]);
        // pin the segment here: without a use the compiler sank all 32 MFMAs of the k-tile past
        // the phase barriers to the loop's end, which serialised them against the partner wave's
        // reads (one 1024-cycle MFMA burst per wave instead of four interleaved segments)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[mq * 4 + i][nq * 2 + j]));
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

    if constexpr (MX) {
      // this split's activation scales -> LDS, before any LDS-DMA is in flight (plain loads):
      // k-tile t, 64-row block w >> 2 of the tile (clamped: rows past M are never stored)
      for (int u = tid; u < T * 16; u += kThreads) {
        const int t = u >> 4, w = u & 15;
        const int blk = min((m0 >> 6) + (w >> 2), mx.nb - 1);
        const uint4 v = *reinterpret_cast<const uint4*>(
            mx.a_sc + ((size_t)(kt0 + t) * mx.nb + blk) * 64 + (w & 3) * 16);
        *reinterpret_cast<uint4*>(smem + kLds + t * 256 + w * 16) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // ---- prologue: tile 0 complete, three halves of tile 1 in flight ----
    // (LDS is free here: every wave passed the realigning barrier after its last ds_read)
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
      mx_t = t;
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
#ifdef GEMM_STAMPS
    if (tid0 == 0) {
      unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
      st[6] = __builtin_amdgcn_s_memrealtime();
      st[7] = __builtin_amdgcn_s_memtime();
    }
#endif

    // ---- stream-K hand-off ----
    if (kSk && publish) {
      // slab layout = register order: element (i, j) of thread tid at f32x4 index (i*4+j)*512+tid
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(sk.slabs + (size_t)lid * (kTM * kTN), 0,
                                                        kTM * kTN * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                 tid * 16, (i * 4 + j) * kThreads * 16,
                                                 16 /* sc1: write-through */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store((gu32*)(sk.flags + lid), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;   // nothing to store: the finisher owns the epilogue
    }
    // predecessors lid-1, lid-2, ... hold the earlier k-tiles of this tile; the last of them is
    // the one whose range starts at or before the tile's first k-tile (counted first, on scalars:
    // a `break` out of the accumulating loop makes the compiler copy and spill the accumulators)
    int npred = 0;
    if (kSk && finish)
      for (int p = lid - 1; p >= 0; --p) {
        ++npred;
        if (sk_total * p / sk.sk_wgs <= tile_k0) break;
      }
    {
      for (int q = 1; q <= npred; ++q) {
        const int p = lid - q;
        if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {   // wave 0 polls (uniform loop)
          unsigned spins = 0;
          while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(
                     (gu32*)(sk.flags + p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins == (1u << 20)) {   // bounded: count the timeout, never hang the GPU
              if (tid == 0) atomicAdd(sk.err, 1u);
              break;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        // buffer loads: one VGPR offset (tid * 16) + a constant SGPR offset per fragment, and 4
        // loads in flight at a time (all 32 at once would need 128 more VGPRs)
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(sk.slabs + (size_t)p * (kTM * kTN), 0,
                                                          kTM * kTN * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          f32x4 v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rs, tid * 16, (i * 4 + j) * kThreads * 16, 0));
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] += v[j];
          __builtin_amdgcn_sched_barrier(0);   // keep the chunks apart (no batching of 32 loads)
        }
      }
    }

    // ---- epilogue ----
    // The MFMAs compute the transposed tile (A operand = weight rows): fragment (i, j) element e of
    // lane l is C[row = 16 i + (l & 15)][col = 16 j + 4 (l >> 4) + e], so each lane owns 4
    // consecutive output columns of one row -> 8-B (bf16) / 16-B (fp32) vector stores.
    const int crow = m0 + wr * 128 + fr;
    const int cq = 4 * (lane >> 4);
    if (BYTES) {  // dequantise: per-row activation scale x per-output-channel weight scale
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float sa = MX ? 1.f : a_scale[min(crow + i * 16, M - 1)];
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
    if constexpr (PREC == kInt8) {
      if (ol.J > 0 && split == 0) {
        // weight fragment = MFMA A operand, as in the main loop: lane l holds w_out row
        // n0 + 64 wc + 16 j + (l & 15) and x_out row crow + 16 i, k = 8 (l >> 4) .. + 7
        const int jl = ol.cnt ? min(ol.J, (*ol.cnt + 31) & ~31) : ol.J;
        for (int kk = 0; kk < jl; kk += 32) {
          bf16x8 wf[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            wf[j] = *reinterpret_cast<const bf16x8*>(
                ol.w + (size_t)(n0 + wc * 64 + j * 16 + fr) * ol.J + kk + 8 * (lane >> 4));
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int m = min(crow + i * 16, M - 1);
            const bf16x8 xf = *reinterpret_cast<const bf16x8*>(ol.x + (size_t)m * ol.J + kk +
                                                               8 * (lane >> 4));
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma(wf[j], xf, acc[i][j]);
          }
        }
      }
    }
    if constexpr (EPI == kSwiGLUMx) {
      // h = silu(gate) * up rounded to bf16 (what the bf16 epilogue stores), kept in the gate
      // fragments; amax per row over the wave's 32 columns (shuffles), then over the 4 n-waves
      // of the workgroup = the row's 128-column block (LDS; free: every wave is past the loop)
      float* red = reinterpret_cast<float*>(smem);   // [wr][wc][128 rows]
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float a = 0.f;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float g = (float)(bf16)acc[i][2 * p][e];
            const float u = (float)(bf16)acc[i][2 * p + 1][e];
            const float h = (float)(bf16)(silu(g) * u);
            acc[i][2 * p][e] = h;
            a = fmaxf(a, fabsf(h));
          }
        a = fmaxf(a, __shfl_xor(a, 16, 64));
        a = fmaxf(a, __shfl_xor(a, 32, 64));
        if (lane < 16) red[(wr * 4 + wc) * 128 + i * 16 + fr] = a;
      }
      __syncthreads();
      uint8_t* out = reinterpret_cast<uint8_t*>(C);
      const int I = N >> 1;
      const int tn = n0 / kTN;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = crow + i * 16;
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) a = fmaxf(a, red[(wr * 4 + w) * 128 + i * 16 + fr]);
        const int k = mx_exponent(a);
        const float inv = mx_inv_scale(k);
        if (row < M) {
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const f32x4 v = acc[i][2 * p] * inv;
            *reinterpret_cast<unsigned*>(out + (size_t)row * I + (n0 >> 1) + wc * 32 + p * 16 + cq) =
                pack4_fp8(v[0], v[1], v[2], v[3]);
          }
        }
        // one byte per (row, block); rows in [M, 64 nb) get 2^0 so the consumer's dword loads
        // never read an unwritten scale
        if (wc == 0 && lane < 16 && row < mx.nb * 64)
          mx.out_sc[mx_off(tn, row, mx.nb)] = (uint8_t)(row < M ? k + 127 : 127);
      }
    } else if (EPI == kSwiGLU) {
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
    } else if (EPI == kStoreBf16Part) {
      bf16* out = reinterpret_cast<bf16*>(C) + (size_t)split * M * N;
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
#ifdef GEMM_STAMPS
  if (tid0 == 0) {
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

int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cus[dev] = n;
  }
  return cus[dev];
}

template <int VAR, int PREC>
int launch_whole_impl(void* C, const void* A, const void* B, const float* sa, const float* sb,
                      float* workspace, int M, int N, int K, int splits, int kps, int epilogue,
                      int tiles, int tiles_m, int tiles_n, hipStream_t stream, OutlierArgs ol,
                      MxArgs mx) {
  SkArgs sk{0, 0, nullptr, nullptr, nullptr};
  if (epilogue == kStoreBf16Part) {   // bf16 partials into C [splits, M, N]; the consumer sums
    if (splits < 2) return -3;
    sk.n_dp = tiles * splits;   // the block remap covers the whole grid
    gemm_tile_kernel<kStoreBf16Part, PREC, false, VAR><<<tiles * splits, kThreads, 0, stream>>>(
        A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kps, sk, ol, mx);
    return 0;
  }
  // kStoreF32 with splits > 1: partials only, the consumer reduces them (rms_norm_splitk)
  if (splits > 1 && (workspace == nullptr || epilogue == kSwiGLU)) return -3;
  if (splits == 1 && epilogue == kStoreF32) return -3;
  const int grid = tiles * splits;
  sk.n_dp = grid;
  if (splits > 1) {
    gemm_tile_kernel<kStoreF32, PREC, false, VAR><<<grid, kThreads, 0, stream>>>(
        A, B, workspace, sa, sb, M, N, K, tiles_m, tiles_n, kps, sk, ol, mx);
    if (epilogue == kStoreF32) return 0;
    const size_t MN = (size_t)M * N;
    size_t blocks = (MN / 8 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    tile_splitk_reduce_kernel<<<(int)blocks, 256, 0, stream>>>(reinterpret_cast<bf16*>(C),
                                                               workspace, splits, MN);
  } else if (epilogue == kSwiGLUMx) {
    if constexpr (PREC == kFp8)
      gemm_tile_kernel<kSwiGLUMx, PREC, false, VAR><<<grid, kThreads, 0, stream>>>(
          A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kps, sk, ol, mx);
  } else if (epilogue == kSwiGLU) {
    if constexpr (PREC == kFp8Mx) return -4;   // MX activations come from the SwiGLU epilogue
    else
      gemm_tile_kernel<kSwiGLU, PREC, false, VAR><<<grid, kThreads, 0, stream>>>(
          A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kps, sk, ol, mx);
  } else if (epilogue == kStoreBf16) {
    gemm_tile_kernel<kStoreBf16, PREC, false, VAR><<<grid, kThreads, 0, stream>>>(
        A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kps, sk, ol, mx);
  } else {
    return -4;
  }
  return 0;
}

// non-temporal weight loads (gemm_tile_kernel VAR bit 0) for tiles_m <= 2: each weight byte is
// read at most twice (profiles/gemm_var_nt_group_ab.json)
bool weights_nt(int tiles_m) { return tiles_m <= 2; }

// splits == 0: data-parallel whole tiles + stream-K tail (SkArgs); workspace = the
// gemm_tile_sk_workspace_floats() layout: [flags | err | pad] 4 KB, then sk_wgs fp32 slabs.
template <int PREC>
int launch_tile(void* C, const void* A, const void* B, const float* sa, const float* sb,
                float* workspace, int M, int N, int K, int splits, int epilogue,
                hipStream_t stream, OutlierArgs ol, MxArgs mx) {
  constexpr int esz = PREC == kBf16 ? 2 : 1;
  const int kt = (int)((size_t)K * esz / 128);
  if (M <= 0 || N % kTN != 0 || (size_t)K * esz % 128 != 0 || splits < 0) return -1;
  if (splits > kt) return -2;
  if (PREC != kBf16 && ((sa == nullptr && PREC != kFp8Mx) || sb == nullptr)) return -5;
  if (PREC == kFp8Mx && (mx.a_sc == nullptr || mx.nb != (M + 63) / 64)) return -13;
  if (epilogue == kSwiGLUMx && (PREC != kFp8 || mx.out_sc == nullptr || mx.nb != (M + 63) / 64 ||
                                splits != 1))
    return -14;
  const int tiles_m = (M + kTM - 1) / kTM, tiles_n = N / kTN;
  const int tiles = tiles_m * tiles_n;
  SkArgs sk{0, 0, nullptr, nullptr, nullptr};
  if constexpr (PREC != kBf16) {
    if (splits == 0) return -10;   // the stream-K tail is compiled for bf16 operands only
  } else if (splits == 0) {
    const int cus = device_cus();
    if (cus <= 0 || cus > kSkMaxWgs) return -7;
    if (workspace == nullptr || epilogue == kStoreF32) return -3;
    sk.sk_wgs = cus;
    sk.n_dp = tiles / cus * cus;
    // needs a tail and >= 1 k-tile per stream-K workgroup
    if (tiles == sk.n_dp || (long long)(tiles - sk.n_dp) * kt < cus) return -8;
    sk.flags = reinterpret_cast<unsigned*>(workspace);
    sk.err = reinterpret_cast<unsigned*>(workspace) + kSkErrWord;
    sk.slabs = workspace + kSkHeaderFloats;
    // zero the flags (a memset node under graph capture); 16-byte multiple from the allocation start
    if (hipMemsetAsync(workspace, 0, ((size_t)cus * 4 + 15) / 16 * 16, stream) != hipSuccess) return -9;
    const int grid = sk.n_dp + sk.sk_wgs;
    if (epilogue == kSwiGLU)
      gemm_tile_kernel<kSwiGLU, PREC, true><<<grid, kThreads, 0, stream>>>(A, B, C, sa, sb, M, N, K,
                                                                          tiles_m, tiles_n, kt, sk, ol, mx);
    else if (epilogue == kStoreBf16)
      gemm_tile_kernel<kStoreBf16, PREC, true><<<grid, kThreads, 0, stream>>>(
          A, B, C, sa, sb, M, N, K, tiles_m, tiles_n, kt, sk, ol, mx);
    else
      return -4;
    return 0;
  }
  const int kps = (kt + splits - 1) / splits;
  if ((splits - 1) * kps >= kt) return -2;   // every split owns at least one k-tile
  if (PREC == kFp8Mx && kps > kMxMaxKt) return -15;   // its scales must fit the LDS slot
  if (weights_nt(tiles_m))
    return launch_whole_impl<1, PREC>(C, A, B, sa, sb, workspace, M, N, K, splits, kps, epilogue, tiles, tiles_m, tiles_n, stream, ol, mx);
  return launch_whole_impl<0, PREC>(C, A, B, sa, sb, workspace, M, N, K, splits, kps, epilogue, tiles, tiles_m, tiles_n, stream, ol, mx);
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

long long gemm_tile_sk_workspace_floats() {
  const int cus = device_cus();
  return cus <= 0 ? -1 : kSkHeaderFloats + (long long)cus * kTM * kTN;
}

int launch_gemm_tile(void* C, const void* A, const void* B, const float* a_scale,
                     const float* b_scale, float* workspace, int M, int N, int K, int splits,
                     int epilogue, int precision, hipStream_t stream, const bf16* x_out,
                     const bf16* w_out, int J, const uint8_t* a_mx, uint8_t* out_mx,
                     const int* ol_cnt) {
  if (J < 0 || J % 32 != 0 || (J > 0 && (precision != kInt8 || !x_out || !w_out))) return -12;
  const OutlierArgs ol{x_out, w_out, J, ol_cnt};
  const MxArgs mx{a_mx, out_mx, (M + 63) / 64};
  switch (precision) {
    case kBf16:
      return launch_tile<kBf16>(C, A, B, nullptr, nullptr, workspace, M, N, K, splits, epilogue,
                                stream, ol, mx);
    case kFp8:
      return launch_tile<kFp8>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue,
                               stream, ol, mx);
    case kFp8Mx:
      return launch_tile<kFp8Mx>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue,
                                 stream, ol, mx);
    case kInt8:
      return launch_tile<kInt8>(C, A, B, a_scale, b_scale, workspace, M, N, K, splits, epilogue,
                                stream, ol, mx);
  }
  return -6;
}

}  // namespace dli
