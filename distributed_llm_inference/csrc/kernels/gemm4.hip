// Projection GEMM for CDNA4, one wave per SIMD:  C[M, N] = A[M, K] . B[N, K]^T  (bf16, fp32 acc)
//
// Same contract as gemm_tile.hip (256 x 256 x 64 tiles, NT operands, the weight fragment as the
// MFMA A operand so every lane owns 4 consecutive output columns, the same SwiGLU interleave and
// split-K partial layouts), different machine shape:
//
//   * workgroup = 4 waves as 2 (M) x 2 (N), ONE wave per SIMD; wave tile 128 x 128 = 8 x 8
//     fragments of v_mfma_f32_16x16x32_bf16, 256 fp32 accumulators per lane in AGPRs.  Per
//     k-tile a wave reads 16 + 16 fragments (32 KB per wave, 128 KB per CU) for 128 MFMAs -- a
//     third less LDS traffic per FLOP than the 8-wave kernel's 128 x 64 wave tiles (192 KB per
//     CU per k-tile).  The decode GEMMs run at the power cap, so LDS energy is clock;
//   * the k-loop is written instruction by instruction: every MFMA, fragment read, barrier and
//     wait is an `asm volatile` statement (the LDS-DMA issues are builtins pinned between them
//     by the statements' memory clobbers), so the source order IS the issue order, and the
//     compiler only allocates registers.  The schedule is the one hipBLASLt's hand-written
//     MT256x256x64 MI16x16 kernel uses (profiles/gemm4_isa_vs_hipblaslt.md):
//
//       seg 1 (64 MFMAs of k-step 0, fragments P):  read k-step 1 fragments Q of tile t, one
//             ds_read_b128 per 2 MFMAs; lgkmcnt(0) + barrier B1 (stage t&1 is free);
//       seg 2 (64 MFMAs of k-step 1, fragments Q):  LDS-DMA tile t+2 into stage t&1, one
//             buffer_load ... lds per 2 MFMAs; after 8 of them vmcnt(8) + barrier B2 (tile t+1
//             has landed in stage (t+1)&1 for every wave); read k-step 0 fragments P of tile
//             t+1, one per 2 MFMAs; lgkmcnt(0) at the segment's end.
//
//     Two barriers per k-tile, no wait on a fragment inside a segment (each segment's
//     fragments were read and retired during the previous one), the DMA of a tile has one
//     whole k-tile of MFMAs to land;
//   * LDS: two stages of A [256][128 B] + B [256][128 B] = 128 KB; XOR swizzle chunk ^ ((row >> 1)
//     & 7) on the DMA source address (LDS-DMA writes lane-linearly) and on the fragment reads
//     (conflict-free ds_read_b128, docs/kernels.md).  Rows of A past M are clamped to row M-1
//     (computed, never stored), so no load leaves the tensor;
//   * persistent grid: with more tiles than CUs each workgroup runs several whole tiles in turn
//     (gate|up at M = 512: 448 tiles on 224 workgroups, 2 each -- at the power cap fewer busy CUs
//     clock higher, which is why hipBLASLt picks that grid); blockIdx is remapped so the
//     workgroups of one XCD take neighbouring work items (shared A / B panels in its L2).
//   * fp8 (e4m3) operands run gemm_tile.hip's block-scaled 16x16x128 MFMA with its fragment
//     pairing (halves = 16-B chunks g and g+4 of the 128-B k-tile row), so sums, epilogues and
//     split-K partials are bit-identical to gemm_tile's fp8 path.  A k-tile is 64 MFMAs of 32
//     cycles (the bf16 k-tile's 2048), but each needs a whole 32-B fragment pair, so the k-loop
//     has its own schedule (G4S8): weight fragments double-buffered, activation fragments
//     re-read one row block behind the MFMAs.  Per-row activation x per-channel weight scales in
//     the epilogue (PREC 1), or MX activations (PREC 2: one e8m0 scale per (row, 128-column
//     block), common.h mx_off layout) on the MFMA's per-lane scale operand -- a k-tile is exactly
//     one scale block, read once per k-tile from an LDS copy of the tile's scales; and the
//     gate|up SwiGLU epilogue can quantise its output to MX itself (kG4SwiGLUMx: the 128 output
//     columns of a 256-wide weight tile are one block, so the row amax is two shuffles plus one
//     LDS exchange between the tile's two n-waves).
#include "kernels.h"

#include <type_traits>
#include <utility>

namespace dli {

namespace {

// cache-policy bits of the activation / weight LDS-DMA (experiment builds override them)
#ifndef GEMM4_A_AUX
#define GEMM4_A_AUX 0
#endif
#ifndef GEMM4_B_AUX
#define GEMM4_B_AUX 0
#endif

constexpr int kG4Threads = 256;
constexpr int kG4Stage = 65536;   // A [256][128 B] | B [256][128 B]

enum G4Epi { kG4Bf16 = 0, kG4F32 = 1, kG4SwiGLU = 2, kG4SwiGLUMx = 3, kG4Bf16Part = 4 };

constexpr int kG4MxKt = 64;                // k-tiles of MX scales a workgroup keeps in LDS
constexpr int kG4MxLds = kG4MxKt * 256;    // [k-tile][256 tile rows] e8m0 bytes
static_assert(kG4MxLds == 4 * 256 * 16, "the MX slab load: 4 x 16 B per lane of 256 lanes");
constexpr int kG4RedLds = 2 * 256 * 4;     // kG4SwiGLUMx row amax exchange [wc][256 rows]

struct G4Mx {
  const uint8_t* a_sc;   // PREC 2: the activations' e8m0 scales (mx_off layout)
  uint8_t* out_sc;       // kG4SwiGLUMx: scales of the quantised output (mx_off, kt = n-tile)
  int nb;                // ceil(M / 64)
};

typedef __attribute__((address_space(3))) void g4_lds_t;

template <bool V>
struct G4B { static constexpr bool value = V; };

// compile-time loop: f(std::integral_constant<int, i>) for i in the sequence, fully unrolled
// (a 128-step #pragma unroll loop of this size is not unrolled by the compiler)
template <typename F, int... I>
__device__ __forceinline__ void g4_static_for(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

// k-loop schedules (MFMA positions 0..127 of a k-tile): Q reads at q0 + qs*n, lgkmcnt(0) + B1
// after MFMA b1, DMA piece j at d0 + ds*j, vmcnt(vm) + B2 after b2 (vm = DMA pieces issued
// before b2), P reads at p0 + ps*n.  Constraints: Q reads < b1 < d0, pieces before b2 == vm,
// b2 < p0, the last P read leaves the tail of the k-tile to retire it.
template <int V> struct G4Sched;
template <> struct G4Sched<4> {   // late wait, DMA spread thin (1 per 4 MFMAs), dense P reads
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 4, b2 = 104, vm = 16, p0 = 105, ps = 1;
};
template <> struct G4Sched<6> {   // v4 with the DMA spread over B2 (1 per 6 MFMAs, 12 before it)
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 6, b2 = 104, vm = 12, p0 = 105, ps = 1;
};
// v4 / v6 with the weight DMA non-temporal (cache policy NT, aux 2: gemm_tile's decode weight
// stream) -- each weight byte is read by at most two workgroups at decode M
template <> struct G4Sched<8> : G4Sched<4> { static constexpr bool nt = true; };
template <> struct G4Sched<9> : G4Sched<6> { static constexpr bool nt = true; };
// (the other eight schedules of the round-4 A/B, profiles/r4/gemm4_ab_v0-7.txt, are in
// scripts/experiments/gemm4_sched_variants.h)
template <typename S, typename = void> struct G4BFirst { static constexpr bool value = false; };
template <typename S> struct G4BFirst<S, std::void_t<decltype(S::bfirst)>> {
  static constexpr bool value = S::bfirst;
};
template <int V, typename = void> struct G4Nt { static constexpr bool value = false; };
template <int V> struct G4Nt<V, std::void_t<decltype(G4Sched<V>::nt)>> {
  static constexpr bool value = G4Sched<V>::nt;
};
// Default schedules: decode-sized M (<= 2 row tiles, the activations stay L2 / MALL-resident and
// only the weight stream misses) takes v8 = v4 with the weight stream non-temporal (round 5,
// profiles/r5/gemm4_sched_nt.md: gate|up 400 vs 431 us for v6, down 191 vs 216, +1.4 % tok/s
// in-step; round 4 had picked v6 over plain v4, profiles/r4/gemm4_ab_v0-7.txt); larger M, where
// both operands stream from HBM and are re-read by many row tiles, takes v4 (8192^3: v6 1074 us).
constexpr int kG4Default = 4, kG4DecodeDefault = 8;

__device__ __forceinline__ float g4_silu(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ void g4_mfma(f32x4& acc, const bf16x8& w, const bf16x8& x) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(x) : "memory");
}

typedef int g4_i32x4 __attribute__((ext_vector_type(4)));
typedef int g4_i32x8 __attribute__((ext_vector_type(8)));
typedef float g4_f32x16 __attribute__((ext_vector_type(16)));

// fp8 e4m3 x fp8 e4m3 -> fp32, 16 x 16 x 128, block scales 1.0 (e8m0 127 in `sc`): the per-row /
// per-channel scales are applied in the epilogue -- gemm_tile.hip's mfma_fp8, same operand order
// (weights = A, activations = B).  The two 16-B halves of each operand come from two
// ds_read_b128 into adjacent registers (the register coalescer places them; no copies).
__device__ __forceinline__ void g4_mfma8(f32x4& acc, const g4_i32x4& w0, const g4_i32x4& w1,
                                         const g4_i32x4& x0, const g4_i32x4& x1, int sc) {
  const g4_i32x8 w = __builtin_shufflevector(w0, w1, 0, 1, 2, 3, 4, 5, 6, 7);
  const g4_i32x8 x = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
               : "+a"(acc) : "v"(w), "v"(x), "v"(sc) : "memory");
}

// MX activations: the weight block scale stays 1.0 (e8m0 127), the activation scale is byte SEL
// of `sx` (lane l: row l & 15 of activation fragment SEL of a 64-row half, mx_off's byte order)
template <int SEL>
__device__ __forceinline__ void g4_mfma8mx(f32x4& acc, const g4_i32x4& w0, const g4_i32x4& w1,
                                           const g4_i32x4& x0, const g4_i32x4& x1, int sc, int sx) {
  const g4_i32x8 w = __builtin_shufflevector(w0, w1, 0, 1, 2, 3, 4, 5, 6, 7);
  const g4_i32x8 x = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  if constexpr (SEL == 0)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]"
                 : "+a"(acc) : "v"(w), "v"(x), "v"(sc), "v"(sx) : "memory");
  else if constexpr (SEL == 1)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,1,0] op_sel_hi:[0,0,0]"
                 : "+a"(acc) : "v"(w), "v"(x), "v"(sc), "v"(sx) : "memory");
  else if constexpr (SEL == 2)
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,1,0]"
                 : "+a"(acc) : "v"(w), "v"(x), "v"(sc), "v"(sx) : "memory");
  else
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,1,0] op_sel_hi:[0,1,0]"
                 : "+a"(acc) : "v"(w), "v"(x), "v"(sc), "v"(sx) : "memory");
}

// fp8 k-loop schedules, in MFMA slots 0..63 of a k-tile (32 cycles each; MFMA g = activation
// fragment g / 8 x weight fragment g % 8).  Activation fragments la..7 of the tile are read at
// slots 1.. (two halves each), then lgkmcnt(0) + B1 after slot b1; DMA piece j after slot
// d0 + ds*j; vmcnt(vm) + B2 after b2; then the next tile's reads -- MX dwords with activation
// fragment 0, weight fragments 0..7 (into the other weight buffer), activation fragments
// 1..la-1 -- spread evenly over slots p0..63, each at least two MFMAs after its register's last
// use; lgkmcnt(2 (la - 1)) at the tile's end (weights and fragment 0 landed).  Weights are double
// buffered (128 VGPRs), activations single (64): with the 256 accumulators in AGPRs a second
// activation set would not fit.
template <int V> struct G4S8;
template <> struct G4S8<0> {   // late activation reads, DMA before B2 (1 per 2 MFMAs)
  static constexpr int la = 7, b1 = 5, d0 = 6, ds = 2, b2 = 37, vm = 16, p0 = 38;
};
template <> struct G4S8<1> {   // three activation fragments read at the tile's start
  static constexpr int la = 5, b1 = 8, d0 = 9, ds = 2, b2 = 40, vm = 16, p0 = 41;
};
template <> struct G4S8<2> {   // v0 with the DMA spread over B2 (1 per 3 MFMAs, 12 before it)
  static constexpr int la = 7, b1 = 5, d0 = 6, ds = 3, b2 = 40, vm = 12, p0 = 41;
};
constexpr int kG8Default = 0, kG8Variants = 3;
template <typename S> struct G4S8Reads {
  static constexpr int n = 16 + 2 * S::la;   // post-B2 reads per k-tile
  static constexpr int len = 64 - S::p0;
  // first post-B2 read issued after MFMA slot g (reads [lo(g), lo(g + 1)) go there)
  static constexpr int lo(int g) { return g < S::p0 ? 0 : ((g - S::p0) * n + len - 1) / len; }
  static constexpr int pos(int r) { return S::p0 + r * len / n; }
  static constexpr bool ok() {
    for (int i = 1; i < S::la; ++i)   // activation fragment i's last MFMA is slot 8 i + 7
      if (pos(18 + 2 * (i - 1)) < 8 * i + 9) return false;
    return S::b1 >= 2 * (8 - S::la) && S::d0 > S::b1 && S::d0 + (S::vm - 1) * S::ds <= S::b2 &&
           (S::vm == 16 || S::d0 + S::vm * S::ds > S::b2) && S::p0 > S::b2 &&
           S::d0 + 15 * S::ds <= 63 && 2 * (S::la - 1) <= 15;
  }
};
static_assert(G4S8Reads<G4S8<0>>::ok() && G4S8Reads<G4S8<1>>::ok() && G4S8Reads<G4S8<2>>::ok(),
              "fp8 k-loop schedule violates a hazard / count constraint");

typedef unsigned g4_u32x2 __attribute__((ext_vector_type(2)));

// the two dwords of this lane's MX scales of one k-tile (rows wr*128 + (l & 15) + {0..63 step
// 16} and + 64: mx_off packs rows r, r+16, r+32, r+48 of a 64-row block in one dword; byte i of
// dword h scales activation fragment 4 h + i)
__device__ __forceinline__ void g4_read_mx(g4_u32x2& dst, int addr) {
  asm volatile("ds_read2_b32 %0, %1 offset1:16" : "=v"(dst) : "v"(addr) : "memory");
}

template <int OFF>
__device__ __forceinline__ void g4_read8(g4_i32x4& dst, int addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF) : "memory");
}

template <int OFF>
__device__ __forceinline__ void g4_read(bf16x8& dst, int addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF) : "memory");
}

__device__ __forceinline__ void g4_sync_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void g4_barrier() { asm volatile("s_barrier" ::: "memory"); }

#ifdef GEMM_PROBE
// diagnostic builds only (scripts/experiments/gemm4_probe.hip): per wave, shader cycles stalled
// at the k-loop's waits (s_memtime, an SMEM read, before and after each; the read after B2 is
// waited for at once -- no LDS read is in flight there -- the others ride the next lgkmcnt(0)).
// g_probe[(block * 4 + wave) * 8 + k]: k = 0 B1 (lgkmcnt(0) + barrier), 1 B2 (vmcnt + barrier),
// 2 end-of-tile LDS wait, 3 k-loop cycles, 4 k-tiles
__device__ unsigned long long* g_probe;
struct G4Probe {
  unsigned long long b1 = 0, b2 = 0, ew = 0, t0 = 0, t1 = 0, t4 = 0, t5 = 0, loop0 = 0, loop = 0;
  unsigned long long kt = 0;
};
#define G4P_TIME(v) asm volatile("s_memtime %0" : "=s"(v) :: "memory")
#define G4P_FENCE(v) asm volatile("" : "+s"(v) :: "memory")
#endif

template <int N>
__device__ __forceinline__ void g4_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t g4_rsrc(const void* base, int bytes) {
  const unsigned long long p = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// PREC 0: bf16 operands (16x16x32 MFMAs, 128 per wave per k-tile, G4Sched<VAR>).  PREC 1: fp8
// e4m3 operands (a k-tile = 128 bytes = 128 elements of every row, the same LDS image and DMA):
// 16x16x128 block-scaled MFMAs, 64 per wave per k-tile (G4S8<VAR>); per-row a_scale x
// per-channel b_scale in the epilogue, as gemm_tile.hip's fp8 path.  PREC 2: PREC 1 with MX
// activation scales (G4Mx) on the MFMA's scale operand instead of a_scale.
template <int EPI, int VAR, int PREC = 0>
__global__ void __launch_bounds__(kG4Threads, 1)
gemm4_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, void* __restrict__ C,
             int M, int N, int K, int tiles_m, int tiles_n, int kps, int splits,
             const float* __restrict__ a_scale, const float* __restrict__ b_scale, G4Mx mx) {
  constexpr bool F8 = PREC >= 1;
  constexpr bool MXIN = PREC == 2;
  constexpr int kBAux = (!F8 && G4Nt<VAR>::value) ? 2 : GEMM4_B_AUX;   // weight DMA cache policy
  constexpr int kMxOff = 2 * kG4Stage;                              // MX scale slab
  constexpr int kRedOff = kMxOff + (MXIN ? kG4MxLds : 0);           // kG4SwiGLUMx exchange
  constexpr int kSmem = kRedOff + (EPI == kG4SwiGLUMx ? kG4RedLds : 0);
  const char* A = reinterpret_cast<const char*>(Av);
  const char* B = reinterpret_cast<const char*>(Bv);
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  const int tid = threadIdx.x, lane = tid & 63;
#ifdef GEMM_STAMPS
  // diagnostic builds only (scripts/experiments/gemm4_bench.hip): begin / end-of-last-k-loop /
  // end stamps per workgroup, shader cycles and 100 MHz wall ticks (g_stamp_blk: gemm_tile.hip)
  unsigned long long* st = g_stamp_blk + (size_t)blockIdx.x * 8;
  if (tid == 0) {
    st[0] = __builtin_amdgcn_s_memrealtime();
    st[1] = __builtin_amdgcn_s_memtime();
  }
#endif
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1, fr = lane & 15;
  const int Kb = K * (F8 ? 1 : 2);
  const int kt_all = Kb / 128;
  const int items = tiles_m * tiles_n * splits;
  const int lds0 = (int)(size_t)smem;
#ifdef GEMM_PROBE
  G4Probe pr;
#endif

  // XCD-aware bijective remap of the workgroup index: blocks b, b+8, ... share an XCD
  const int G = gridDim.x, bx = blockIdx.x, x8 = bx & 7, q8 = G >> 3, r8 = G & 7;
  const int lid = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bx >> 3);

  // per-lane constants: fragment read addresses of (operand, k-step, stage) and DMA offsets
  const int sw = fr >> 1;   // (row >> 1) & 7 of every row this lane reads
  int rdA[2][2], rdB[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = ((kk * 4 + (lane >> 4)) ^ sw) << 4;
      rdA[kk][s] = lds0 + s * kG4Stage + (wr * 128 + fr) * 128 + ch;
      rdB[kk][s] = lds0 + s * kG4Stage + 32768 + (wc * 128 + fr) * 128 + ch;
    }
  // (fp8: a fragment's two 16-B halves are the bf16 k-step 0 / 1 chunks, rdX[0] / rdX[1]: chunks
  // l >> 4 and 4 + (l >> 4) of the 128-B row, gemm_tile.hip's fp8 pairing)
  // MX scales: this lane's two dwords of a k-tile's 256-byte slab (rows wr*128 + (l & 15) + 16 i)
  const int mxrd = lds0 + kMxOff + wr * 128 + (lane & 15) * 4;
  // DMA: wave-load q = 4j + w covers tile rows 8q .. 8q+7; lane -> row 8q + (lane >> 3), LDS
  // slot lane & 7 holding global chunk (lane & 7) ^ ((row >> 1) & 7) = .. ^ ((q & 1) * 4 + (lane >> 4))
  const int dchunk = ((lane & 7) ^ (((w & 1) * 4 + (lane >> 4)) & 7)) << 4;
  const int drow = 8 * w + (lane >> 3);

  for (int item = lid; item < items; item += G) {
    const int tile = item % (tiles_m * tiles_n), split = item / (tiles_m * tiles_n);
    const int tm = tile % tiles_m, tn = tile / tiles_m;   // M tiles of one weight panel adjacent
    const int m0 = tm * 256, n0 = tn * 256;
    const int kt0 = split * kps;
    const int T = __builtin_amdgcn_readfirstlane(min(kps, kt_all - kt0));
    const int mrows = min(256, M - m0);
    const auto rsA = g4_rsrc(A + (size_t)m0 * Kb, mrows * Kb);
    const auto rsB = g4_rsrc(B + (size_t)n0 * Kb, 256 * Kb);
    int voA[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) voA[j] = min(drow + 32 * j, mrows - 1) * Kb + dchunk;
    const int voB = drow * Kb + dchunk;
#ifdef GEMM_PROBE
    G4P_TIME(pr.loop0);
#endif

    if constexpr (MXIN) {
      // this tile's scales of its k-tiles into LDS, [t][256 rows]: a k-tile's 4 blocks of 64
      // rows are 256 contiguous bytes of mx_off, so 16 B per lane and every load issued before
      // any store -- one round trip (T <= kG4MxKt = 4 x 256 lanes x 16 B / 256 B).  64-row
      // blocks past the array (a partial last M tile) read as 2^0 (computed, never stored).
      // (A dword per lane, each load waited for before its store, cost 14 round trips per
      // workgroup for the 70B down projection: +3 % on its in-step time.)
      const int vb = min(4, mx.nb - (m0 >> 6));
      uint4 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int idx = tid + r * kG4Threads, t = idx >> 4, q = idx & 15;
        v[r] = make_uint4(0x7f7f7f7fu, 0x7f7f7f7fu, 0x7f7f7f7fu, 0x7f7f7f7fu);
        if (t < T && (q >> 2) < vb)
          v[r] = *reinterpret_cast<const uint4*>(
              mx.a_sc + ((size_t)(kt0 + t) * mx.nb + (m0 >> 6)) * 64 + q * 16);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int idx = tid + r * kG4Threads, t = idx >> 4, q = idx & 15;
        if (t < T) *reinterpret_cast<uint4*>(smem + kMxOff + t * 256 + q * 16) = v[r];
      }
      g4_sync_lds();   // written before the prologue's barrier publishes them
    }
    g4_u32x2 mxr = {0x7f7f7f7fu, 0x7f7f7f7fu};   // scale dwords of the next k-tile
    g4_u32x2 mxc = mxr;                          // ... of the current one

    // stage DMA piece j (0..15: A rows 32j' .. for j < 8, B for j >= 8) of k-tile t
    auto dma = [&](int t, int j) {
#ifdef GEMM_PROBE_NODMA
      if (t >= 2) return;   // diagnostic: the k-loop's DMA cost (results are garbage)
#endif
      const int s = t & 1;
      const int koff = __builtin_amdgcn_readfirstlane((kt0 + t) * 128);
      if (j < 8) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsA, (g4_lds_t*)(smem + s * kG4Stage + (4 * j + w) * 1024), 16, voA[j], koff, 0,
            GEMM4_A_AUX);
      } else {
        const int jb = j - 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsB, (g4_lds_t*)(smem + s * kG4Stage + 32768 + (4 * jb + w) * 1024), 16, voB,
            __builtin_amdgcn_readfirstlane(koff + jb * 32 * Kb), 0, kBAux);
      }
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (F8) {
      // ---- fp8 k-loop (G4S8): 64 16x16x128 MFMAs per wave per k-tile ----
      using S = G4S8<(VAR >= 0 && VAR < kG8Variants) ? VAR : kG8Default>;
      using R = G4S8Reads<S>;
      const int sc127 = 127;
      g4_i32x4 W8[2][8][2], A8[8][2];   // [buffer][fragment][half], [fragment][half]
      // prologue: tiles 0 and 1 in flight, tile 0 landed, its weights (buffer 0), activation
      // fragments 0..la-1 and MX scales read
#pragma unroll
      for (int j = 0; j < 16; ++j) dma(0, j);
      if (T > 1) {
#pragma unroll
        for (int j = 0; j < 16; ++j) dma(1, j);
        g4_vmcnt<16>();
      } else {
        g4_vmcnt<0>();
      }
      g4_barrier();
      if constexpr (MXIN) g4_read_mx(mxr, mxrd);
      g4_static_for(std::make_integer_sequence<int, 16>{}, [&](auto N) {
        constexpr int n = decltype(N)::value, f = n >> 1, h = n & 1;
        g4_read8<f * 2048>(W8[0][f][h], rdB[h][0]);
        if constexpr (f < S::la) g4_read8<f * 2048>(A8[f][h], rdA[h][0]);
      });
      g4_sync_lds();

      // one k-tile on stage / weight buffer P (= t & 1).  DMA: issue tile t+2 into stage P; NEXT:
      // read tile t+1's weights into buffer P ^ 1 and its activation fragments 0..la-1
      auto ktile8 = [&](int t, auto p_c, auto dma_c, auto next_c, bool dma_rt, bool next_rt) {
        constexpr int P = decltype(p_c)::value;
        // DMA / NEXT: compile-time "may", dma_rt / next_rt: whether it does (uniform)
        constexpr bool DMA = decltype(dma_c)::value, NEXT = decltype(next_c)::value;
        if constexpr (MXIN) mxc = mxr;
        g4_static_for(std::make_integer_sequence<int, 64>{}, [&](auto G) {
          constexpr int g = decltype(G)::value, i = g >> 3, j = g & 7;
          if constexpr (MXIN)
            g4_mfma8mx<i & 3>(acc[i][j], W8[P][j][0], W8[P][j][1], A8[i][0], A8[i][1], sc127,
                              (int)mxc[i >> 2]);
          else
            g4_mfma8(acc[i][j], W8[P][j][0], W8[P][j][1], A8[i][0], A8[i][1], sc127);
          if constexpr (g >= 1 && g <= 2 * (8 - S::la)) {   // this tile's late activation reads
            constexpr int f = S::la + (g - 1) / 2, h = (g - 1) & 1;
            g4_read8<f * 2048>(A8[f][h], rdA[h][P]);
          }
          if constexpr (g == S::b1) {
#ifdef GEMM_PROBE
            G4P_TIME(pr.t0);
#endif
            g4_sync_lds();
            if (DMA && dma_rt) g4_barrier();
#ifdef GEMM_PROBE
            G4P_FENCE(pr.t4); G4P_FENCE(pr.t5); G4P_FENCE(pr.t0);
            pr.ew += pr.t5 - pr.t4;
            pr.t4 = pr.t5 = 0;
            G4P_TIME(pr.t1);
#endif
          }
          if constexpr (DMA && g >= S::d0 && g <= S::d0 + 15 * S::ds && (g - S::d0) % S::ds == 0)
            if (dma_rt) dma(t + 2, (g - S::d0) / S::ds);
          if constexpr (NEXT && g == S::b2) {
            if (next_rt) {
#ifdef GEMM_PROBE
              unsigned long long t2, t3;
              G4P_TIME(t2);
#endif
              if (DMA && dma_rt) g4_vmcnt<S::vm>(); else g4_vmcnt<0>();
              g4_barrier();
#ifdef GEMM_PROBE
              G4P_TIME(t3);
              g4_sync_lds();
              G4P_FENCE(t2); G4P_FENCE(t3); G4P_FENCE(pr.t1);
              pr.b2 += t3 - t2;
              pr.b1 += pr.t1 - pr.t0;
              pr.t0 = pr.t1 = 0;
#endif
            }
          }
          if constexpr (NEXT) if (next_rt) {
            g4_static_for(std::make_integer_sequence<int, 4>{}, [&](auto K) {
              constexpr int r = R::lo(g) + decltype(K)::value;
              if constexpr (r < R::lo(g + 1)) {
                if constexpr (r < 2) {
                  if constexpr (MXIN && r == 0) g4_read_mx(mxr, mxrd + (t + 1) * 256);
                  g4_read8<0>(A8[0][r], rdA[r][P ^ 1]);
                } else if constexpr (r < 18) {
                  constexpr int f = (r - 2) >> 1, h = r & 1;
                  g4_read8<f * 2048>(W8[P ^ 1][f][h], rdB[h][P ^ 1]);
                } else {
                  constexpr int f = 1 + ((r - 18) >> 1), h = r & 1;
                  g4_read8<f * 2048>(A8[f][h], rdA[h][P ^ 1]);
                }
              }
            });
          }
        });
#ifdef GEMM_PROBE
        if constexpr (NEXT) if (next_rt) G4P_TIME(pr.t4);
#endif
        if constexpr (NEXT)
          if (next_rt) asm volatile("s_waitcnt lgkmcnt(%0)" :: "i"(2 * (S::la - 1)) : "memory");
#ifdef GEMM_PROBE
        if constexpr (NEXT) if (next_rt) G4P_TIME(pr.t5);
        ++pr.kt;
#endif
      };
      // tiles in pairs (stage parity = t & 1 is a compile-time argument), then the 1-3 left
      using B1 = G4B<true>;
      using B0 = G4B<false>;
      using P0 = std::integral_constant<int, 0>;
      using P1 = std::integral_constant<int, 1>;
      int t = 0;
      for (; t + 3 < T; t += 2) {
        ktile8(t, P0{}, B1{}, B1{}, true, true);
        ktile8(t + 1, P1{}, B1{}, B1{}, true, true);
      }
      ktile8(t, P0{}, B1{}, B1{}, t + 2 < T, t + 1 < T);
      if (t + 1 < T) {
        ktile8(t + 1, P1{}, B0{}, B1{}, false, t + 2 < T);
        if (t + 2 < T) ktile8(t + 2, P0{}, B0{}, B0{}, false, false);
      }
    } else {
    // fragment sets: P = k-step 0, Q = k-step 1 ([0..7] weight fragments, [8..15] activation)
    bf16x8 P[16], Q[16];
    // read fragment n of k-step kk of stage s: n < 8 weight rows wc*128 + 16n, else activation
    // rows wr*128 + 16(n-8)
    auto rd = [&](bf16x8 (&F)[16], int n, int kk, int s, bool in_loop = true) {
#ifdef GEMM_PROBE_NOBREAD
      if (n < 8 && in_loop) return;   // diagnostic: no weight-fragment LDS reads in the loop
#endif
      switch (n) {
        case 0: g4_read<0 * 2048>(F[0], rdB[kk][s]); break;
        case 1: g4_read<1 * 2048>(F[1], rdB[kk][s]); break;
        case 2: g4_read<2 * 2048>(F[2], rdB[kk][s]); break;
        case 3: g4_read<3 * 2048>(F[3], rdB[kk][s]); break;
        case 4: g4_read<4 * 2048>(F[4], rdB[kk][s]); break;
        case 5: g4_read<5 * 2048>(F[5], rdB[kk][s]); break;
        case 6: g4_read<6 * 2048>(F[6], rdB[kk][s]); break;
        case 7: g4_read<7 * 2048>(F[7], rdB[kk][s]); break;
        case 8: g4_read<0 * 2048>(F[8], rdA[kk][s]); break;
        case 9: g4_read<1 * 2048>(F[9], rdA[kk][s]); break;
        case 10: g4_read<2 * 2048>(F[10], rdA[kk][s]); break;
        case 11: g4_read<3 * 2048>(F[11], rdA[kk][s]); break;
        case 12: g4_read<4 * 2048>(F[12], rdA[kk][s]); break;
        case 13: g4_read<5 * 2048>(F[13], rdA[kk][s]); break;
        case 14: g4_read<6 * 2048>(F[14], rdA[kk][s]); break;
        default: g4_read<7 * 2048>(F[15], rdA[kk][s]); break;
      }
    };
    // MFMA number k (0..63) of a segment: activation row-block k / 8, weight block k % 8
    auto mf = [&](const bf16x8 (&F)[16], int k) {
      g4_mfma(acc[k >> 3][k & 7], F[k & 7], F[8 + (k >> 3)]);
    };

    // ---- prologue: tiles 0 and 1 in flight, tile 0 landed, k-step 0 fragments of tile 0 read ----
#pragma unroll
    for (int j = 0; j < 16; ++j) dma(0, j);
    if (T > 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dma(1, j);
      g4_vmcnt<16>();
    } else {
      g4_vmcnt<0>();
    }
    g4_barrier();
#pragma unroll
    for (int n = 0; n < 16; ++n) rd(P, n, 0, 0, false);
#ifdef GEMM_PROBE_NOBREAD
#pragma unroll
    for (int n = 0; n < 8; ++n) rd(Q, n, 1, 0, false);   // real (random) weight values throughout
#endif
    g4_sync_lds();

    // one k-tile.  DMA: issue tile t+2 into stage t&1; NEXT: read k-step 0 of tile t+1
    auto ktile = [&](int t, auto dma_c, auto next_c) {
      constexpr bool DMA = decltype(dma_c)::value, NEXT = decltype(next_c)::value;
      using S = G4Sched<VAR>;
      const int s = t & 1;
      // MFMA g of the k-tile (g < 64: k-step 0 on P, else k-step 1 on Q), and after it: the k-step
      // 1 reads of this tile -> Q, B1, the DMA of tile t+2 into stage s, B2, the k-step 0 reads of
      // tile t+1 -> P, at the positions the schedule S gives
      g4_static_for(std::make_integer_sequence<int, 128>{}, [&](auto G) {
        constexpr int g = decltype(G)::value;
        if constexpr (g < 64) mf(P, g); else mf(Q, g - 64);
        if constexpr (g >= S::q0 && g < S::q0 + 16 * S::qs && (g - S::q0) % S::qs == 0)
          rd(Q, (g - S::q0) / S::qs, 1, s);
        if constexpr (g == S::b1) {   // this wave's reads of stage s done -> after B1 every wave's
#ifdef GEMM_PROBE
          G4P_TIME(pr.t0);
#endif
          g4_sync_lds();
          if (DMA) g4_barrier();
#ifdef GEMM_PROBE
          G4P_FENCE(pr.t4); G4P_FENCE(pr.t5); G4P_FENCE(pr.t0);
          pr.ew += pr.t5 - pr.t4;
          pr.t4 = pr.t5 = 0;
          G4P_TIME(pr.t1);
#endif
        }
        if constexpr (DMA && g >= S::d0 && g < S::d0 + 16 * S::ds && (g - S::d0) % S::ds == 0)
          dma(t + 2, G4BFirst<S>::value ? (((g - S::d0) / S::ds) + 8) & 15 : (g - S::d0) / S::ds);
        if constexpr (NEXT && g == S::b2) {   // own DMA of tile t+1 landed (all but t+2's since)
#ifdef GEMM_PROBE
          unsigned long long t2, t3;
          G4P_TIME(t2);
#endif
          if (DMA) g4_vmcnt<S::vm>(); else g4_vmcnt<0>();
          g4_barrier();
#ifdef GEMM_PROBE
          G4P_TIME(t3);
          g4_sync_lds();
          G4P_FENCE(t2); G4P_FENCE(t3); G4P_FENCE(pr.t1);
          pr.b2 += t3 - t2;
          pr.b1 += pr.t1 - pr.t0;
          pr.t0 = pr.t1 = 0;
#endif
        }
        if constexpr (NEXT && g >= S::p0 && g < S::p0 + 16 * S::ps && (g - S::p0) % S::ps == 0)
          rd(P, (g - S::p0) / S::ps, 0, s ^ 1);
      });
#ifdef GEMM_PROBE
      if (NEXT) G4P_TIME(pr.t4);
#endif
      if (NEXT) g4_sync_lds();
#ifdef GEMM_PROBE
      if (NEXT) G4P_TIME(pr.t5);
      ++pr.kt;
#endif
    };
    int t = 0;
    for (; t + 2 < T; ++t) ktile(t, G4B<true>{}, G4B<true>{});
    if (t + 1 < T) ktile(t++, G4B<false>{}, G4B<true>{});
    ktile(t, G4B<false>{}, G4B<false>{});
    }

#ifdef GEMM_STAMPS
    if (tid == 0) {
      st[6] = __builtin_amdgcn_s_memrealtime();
      st[7] = __builtin_amdgcn_s_memtime();
    }
#endif
    // the last MFMAs' results -> compiler-issued AGPR reads: 12+ wait states for an 8-pass XDL
    // write (18+ for the 16-pass fp8 one); the fence takes every accumulator "+a" so no read is
    // hoisted above it
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#ifdef GEMM_PROBE
    {
      unsigned long long e;
      G4P_TIME(e);
      g4_sync_lds();
      G4P_FENCE(e); G4P_FENCE(pr.loop0);
      pr.loop += e - pr.loop0;
    }
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]),
                   "+a"(acc[i][4]), "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));

    // ---- epilogue: fragment (i, j) element e of lane l is
    //      C[m0 + wr*128 + 16i + (l & 15)][n0 + wc*128 + 16j + 4(l >> 4) + e] ----
    const int crow = m0 + wr * 128 + fr;
    const int cq = 4 * (lane >> 4);
    if constexpr (F8) {   // dequantise as gemm_tile.hip: (acc x channel scale) x row scale
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float sa = MXIN ? 1.f : a_scale[min(crow + i * 16, M - 1)];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4 sb = *reinterpret_cast<const f32x4*>(b_scale + n0 + wc * 128 + j * 16 + cq);
          acc[i][j] = acc[i][j] * sb * sa;
        }
      }
    }
    if constexpr (EPI == kG4SwiGLUMx) {
      // h = silu(gate) * up rounded to bf16 (what the bf16 SwiGLU epilogue stores), kept in the
      // gate fragments; the row's amax over its 128-column block = the two n-waves' 64 each (the
      // 4 lanes sharing a row: two shuffles, then one LDS exchange), then e4m3(h * 2^-k) and one
      // e8m0 byte per (row, block) -- ops.mx_quantize's rule, gemm_tile's kSwiGLUMx
      float* red = reinterpret_cast<float*>(smem + kRedOff);   // [wc][256 rows]
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float a = 0.f;
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float g = (float)(bf16)acc[i][2 * p][e];
            const float u = (float)(bf16)acc[i][2 * p + 1][e];
            const float h = (float)(bf16)(g4_silu(g) * u);
            acc[i][2 * p][e] = h;
            a = fmaxf(a, fabsf(h));
          }
        a = fmaxf(a, __shfl_xor(a, 16, 64));
        a = fmaxf(a, __shfl_xor(a, 32, 64));
        if (lane < 16) red[wc * 256 + wr * 128 + i * 16 + fr] = a;
      }
      g4_sync_lds();
      g4_barrier();
      uint8_t* out = reinterpret_cast<uint8_t*>(C);
      const int I = N >> 1, tn = n0 >> 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = wr * 128 + i * 16 + fr, row = m0 + r;
        const int k = mx_exponent(fmaxf(red[r], red[256 + r]));
        const float inv = mx_inv_scale(k);
        if (row < M) {
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const f32x4 v = acc[i][2 * p] * inv;
            *reinterpret_cast<unsigned*>(out + (size_t)row * I + (n0 >> 1) + wc * 64 + p * 16 + cq) =
                pack4_fp8(v[0], v[1], v[2], v[3]);
          }
        }
        // one byte per (row, block); rows in [M, 64 nb) get 2^0 (the consumer reads them)
        if (wc == 0 && lane < 16 && row < mx.nb * 64)
          mx.out_sc[mx_off(tn, row, mx.nb)] = (uint8_t)(row < M ? k + 127 : 127);
      }
      g4_barrier();   // the exchange slab is reused by the next item
      continue;
    }
    if constexpr (EPI == kG4SwiGLU) {
      // n-fragments (2p, 2p+1) = (gate, up) of output columns n0/2 + wc*64 + 16p + cq + e
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
            o[e] = (bf16)(g4_silu(g) * u);
          }
          *reinterpret_cast<bf16x4*>(out + (size_t)row * I + (n0 >> 1) + wc * 64 + p * 16 + cq) = o;
        }
      }
    } else if constexpr (EPI == kG4F32) {
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
      bf16* out = reinterpret_cast<bf16*>(C) + (EPI == kG4Bf16Part ? (size_t)split * M * N : 0);
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
    // the next item's prologue re-stages both LDS stages: every wave's last reads are retired
    // (lgkmcnt(0) in the last k-tile), the barrier makes that hold for all of them
    g4_barrier();
  }
#ifdef GEMM_PROBE
  if (lane == 0) {
    unsigned long long* q = g_probe + ((size_t)blockIdx.x * 4 + w) * 8;
    q[0] = pr.b1; q[1] = pr.b2; q[2] = pr.ew; q[3] = pr.loop; q[4] = pr.kt;
  }
#endif
#ifdef GEMM_STAMPS
  if (tid == 0) {
    st[2] = __builtin_amdgcn_s_memrealtime();
    st[3] = __builtin_amdgcn_s_memtime();
  }
#endif
}

int g4_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return 256;
  return n;
}

}  // namespace

// Persistent grid for `items` work items on `cus` CUs: all of them if they fit, else the
// smallest grid that needs the same number of rounds (448 items on 256 CUs -> 224 x 2).
int gemm4_grid(int items, int cus) {
  if (items <= cus) return items;
  const int rounds = (items + cus - 1) / cus;
  return (items + rounds - 1) / rounds;
}

// C = A . B^T on the one-wave-per-SIMD kernel.  epilogue 0: bf16 [M, N]; 2: fused SwiGLU ([M,
// N/2], B rows in swiglu_interleave order); with splits > 1: 1 = fp32 partials [splits, M, N],
// 4 = bf16 partials [splits, M, N] (into C; the consumer sums them).  grid <= 0: automatic.
template <int VAR, int PREC>
static int launch_gemm4_v(void* C, const void* a, const void* b, int M, int N, int K, int tiles_m,
                          int tiles_n, int kps, int splits, int epilogue, int grid,
                          hipStream_t stream, const float* sa, const float* sb, G4Mx mx) {
  switch (epilogue) {
    case kG4Bf16:
      gemm4_kernel<kG4Bf16, VAR, PREC><<<grid, kG4Threads, 0, stream>>>(a, b, C, M, N, K, tiles_m, tiles_n, kps, splits, sa, sb, mx);
      break;
    case kG4F32:
      gemm4_kernel<kG4F32, VAR, PREC><<<grid, kG4Threads, 0, stream>>>(a, b, C, M, N, K, tiles_m, tiles_n, kps, splits, sa, sb, mx);
      break;
    case kG4SwiGLU:
      if constexpr (PREC == 2) return -4;   // MX activations feed down / O, never gate|up
      else gemm4_kernel<kG4SwiGLU, VAR, PREC><<<grid, kG4Threads, 0, stream>>>(a, b, C, M, N, K, tiles_m, tiles_n, kps, splits, sa, sb, mx);
      break;
    case kG4SwiGLUMx:
      if constexpr (PREC != 1) return -4;   // the MX output of the fp8 gate|up projection
      else gemm4_kernel<kG4SwiGLUMx, VAR, PREC><<<grid, kG4Threads, 0, stream>>>(a, b, C, M, N, K, tiles_m, tiles_n, kps, splits, sa, sb, mx);
      break;
    case kG4Bf16Part:
      gemm4_kernel<kG4Bf16Part, VAR, PREC><<<grid, kG4Threads, 0, stream>>>(a, b, C, M, N, K, tiles_m, tiles_n, kps, splits, sa, sb, mx);
      break;
    default:
      return -4;
  }
  return 0;
}

template <int PREC>
static int launch_gemm4_p(void* C, const void* a, const void* b, int M, int N, int K, int tiles_m,
                          int tiles_n, int kps, int splits, int epilogue, int grid,
                          hipStream_t stream, int variant, const float* sa, const float* sb,
                          G4Mx mx) {
  if constexpr (PREC >= 1) {   // fp8: G4S8 schedules (the others: experiment builds only)
#ifdef GEMM4_FP8_VARIANTS
    if (variant == 1)
      return launch_gemm4_v<1, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
    if (variant == 2)
      return launch_gemm4_v<2, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
#endif
    if (variant != kG8Default) return -5;
    return launch_gemm4_v<kG8Default, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
  } else {
    if (variant == 6)
      return launch_gemm4_v<6, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
    if (variant == 8)
      return launch_gemm4_v<8, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
    if (variant == 9)
      return launch_gemm4_v<9, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
    if (variant != kG4Default) return -5;
    return launch_gemm4_v<kG4Default, PREC>(C, a, b, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream, sa, sb, mx);
  }
}

// C = A . B^T on the one-wave-per-SIMD kernel.  epilogue 0: bf16 [M, N]; 2: fused SwiGLU ([M,
// N/2], B rows in swiglu_interleave order); with splits > 1: 1 = fp32 partials [splits, M, N],
// 4 = bf16 partials [splits, M, N] (into C; the consumer sums them).  grid <= 0: automatic.
// variant < 0: the default k-loop schedule (G4Sched; fp8: G4S8), else that one (A/B experiments).
// precision 1: fp8 e4m3 A [M, K] / B [N, K] (1-byte), results scaled by a_scale[M] * b_scale[N];
// precision 2: fp8 with MX activation scales a_mx (mx_off layout, nb = ceil(M / 64)) instead of
// a_scale.  epilogue 3 (precision 1, one split): SwiGLU quantised to MX fp8 [M, N/2] in C, its
// scales in out_mx.
int launch_gemm4(void* C, const void* A, const void* B, int M, int N, int K, int splits,
                 int epilogue, int grid, hipStream_t stream, int variant, int precision,
                 const float* a_scale, const float* b_scale, const uint8_t* a_mx,
                 uint8_t* out_mx) {
  const int esz = precision >= 1 ? 1 : 2;
  if (precision < 0 || precision > 2) return -6;
  if (precision == 1 && (a_scale == nullptr || b_scale == nullptr)) return -7;
  if (precision == 2 && (a_mx == nullptr || b_scale == nullptr)) return -7;
  if (epilogue == kG4SwiGLUMx && (precision != 1 || out_mx == nullptr)) return -8;
  if (M <= 0 || N % 256 != 0 || (K * esz) % 128 != 0 || splits < 1) return -1;
  const int kt = K * esz / 128;
  if (splits > kt) return -2;
  const int kps = (kt + splits - 1) / splits;
  if ((splits - 1) * kps >= kt) return -2;   // every split owns at least one k-tile
  if (precision == 2 && kps > kG4MxKt) return -9;   // the tile's scales must fit the LDS slab
  if ((splits > 1) != (epilogue == kG4F32 || epilogue == kG4Bf16Part)) return -3;
  const int tiles_m = (M + 255) / 256, tiles_n = N / 256;
  const int items = tiles_m * tiles_n * splits;
  if (grid <= 0) grid = gemm4_grid(items, g4_cus());
  if (grid > items) grid = items;
  if (variant < 0)
    variant = precision >= 1 ? kG8Default : tiles_m <= 2 ? kG4DecodeDefault : kG4Default;
  const G4Mx mx{a_mx, out_mx, (M + 63) / 64};
  if (precision == 2)
    return launch_gemm4_p<2>(C, A, B, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid,
                             stream, variant, nullptr, b_scale, mx);
  if (precision == 1)
    return launch_gemm4_p<1>(C, A, B, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid,
                             stream, variant, a_scale, b_scale, mx);
  return launch_gemm4_p<0>(C, A, B, M, N, K, tiles_m, tiles_n, kps, splits, epilogue, grid, stream,
                           variant, nullptr, nullptr, mx);
}

}  // namespace dli
