// Decode-shaped GEMM for CDNA4:  C[M, N] = A[M, K] . B[N, K]^T   (bf16 in, fp32 accumulate)
//
// The decode projections of a pipeline stage (fused QKV, O, gate|up, down) multiply a small
// activation block (M = micro-batch <= 256 tokens) by a large weight matrix that is streamed
// from HBM exactly once per step.  hipBLASLt's tuned solutions reach ~600-700 TF on the narrow
// ones (N = 8192 / 10240) at M = 256 because too few output tiles exist to fill 256 CUs; this
// kernel always covers all M rows in one 256-row tile (the weight tile is read once) and splits K
// across workgroups so that every CU streams weights:
//   * workgroup = 8 waves (4 along M x 2 along N), tile 256 x BN x 64, wave tile 64 x BN/2;
//   * v_mfma_f32_16x16x32_bf16 (fragment maps: cdna_hip_programming.md §3);
//   * register-staged, double-buffered LDS: the global loads of k-tile t+1 are issued before the
//     MFMAs of tile t and written to the other LDS buffer after them (one barrier per k-tile);
//   * LDS rows of 128 B (64 bf16) with the 16-B chunk c of row r stored at c ^ ((r >> 1) & 7):
//     for the 16x16x32 A/B fragment reads (lane l -> row l&15, chunk l>>4) every ds_read_b128
//     16-lane group {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... touches 16 distinct 16-B bank
//     slots (conflict-free; derivation in docs/kernels.md);
//   * split-K partials go to an fp32 workspace [splits, M, N] and are summed by a small reduce
//     kernel (bf16 out); with one split the bf16 tile is stored directly.
#include "kernels.h"

namespace dli {

namespace {

constexpr int kBM = 256;
constexpr int kBK = 64;
constexpr int kThreads = 512;

__device__ __forceinline__ f32x4 mfma16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// byte offset of (row, 16-B chunk) inside a [rows][64 bf16] swizzled LDS tile
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

typedef int i32x4v __attribute__((ext_vector_type(4)));

template <int BN>
__global__ void __launch_bounds__(kThreads, 1)
gemm_nt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
               float* __restrict__ part, int M, int N, int K, int k_per_split) {
  constexpr int WN = BN / 2;           // wave tile N
  constexpr int NT = WN / 16;          // 16-wide n tiles per wave
  constexpr int A_CHUNKS = kBM * 8;    // 16-B chunks per A tile
  constexpr int B_CHUNKS = BN * 8;
  constexpr int A_PER_T = A_CHUNKS / kThreads;  // 4
  constexpr int B_PER_T = (B_CHUNKS + kThreads - 1) / kThreads;  // 2 (BN=128) / 1 (BN=64)
  constexpr int A_BYTES = kBM * 128;
  constexpr int B_BYTES = BN * 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave & 3;      // 4 waves along M
  const int wn = wave >> 2;     // 2 waves along N
  const int n0 = blockIdx.x * BN;
  const int split = blockIdx.y;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int ntiles = (kend - kbeg) / kBK;

  // stage buffer b: A tile at smem + b*(A+B), B tile right after it
#define As(b) (smem + (b) * (A_BYTES + B_BYTES))
#define Bs(b) (smem + (b) * (A_BYTES + B_BYTES) + A_BYTES)

  i32x4v ra[A_PER_T], rb[B_PER_T];
  const i32x4v zero = {0, 0, 0, 0};

  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * kBK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * kThreads;
      const int row = q >> 3, c = q & 7;
      ra[i] = row < M ? *reinterpret_cast<const i32x4v*>(A + (size_t)row * K + k0 + c * 8) : zero;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * kThreads;
      if (q < B_CHUNKS) {
        const int row = q >> 3, c = q & 7;
        rb[i] = *reinterpret_cast<const i32x4v*>(B + (size_t)(n0 + row) * K + k0 + c * 8);
      }
    }
  };
  auto lwrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * kThreads;
      *reinterpret_cast<i32x4v*>(As(buf) + swz(q >> 3, q & 7)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * kThreads;
      if (q < B_CHUNKS) *reinterpret_cast<i32x4v*>(Bs(buf) + swz(q >> 3, q & 7)) = rb[i];
    }
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;  // fragment row (A: m, B: n)
  const int fch = lane >> 4;   // fragment 16-B chunk within a 32-wide k step

  if (ntiles > 0) {
    gload(0);
    lwrite(0);
  }
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ntiles) gload(kt + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[NT];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As(cur) + swz(wm * 64 + i * 16 + frow, kk * 4 + fch));
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs(cur) + swz(wn * WN + j * 16 + frow, kk * 4 + fch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16x32(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < ntiles) lwrite(cur ^ 1);
    __syncthreads();
  }

#undef As
#undef Bs
  // epilogue: C/D layout of 16x16 MFMA: col = lane&15, row = (lane>>4)*4 + r
  const int ccol = lane & 15;
  const int crow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wn * WN + j * 16 + ccol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + crow + r;
        if (row < M) {
          if (part)
            part[((size_t)split * M + row) * N + col] = acc[i][j][r];
          else
            C[(size_t)row * N + col] = (bf16)acc[i][j][r];
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16* __restrict__ C,
                                                            const float* __restrict__ part,
                                                            int splits, size_t MN) {
  for (size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * 4; i < MN;
       i += (size_t)gridDim.x * blockDim.x * 4) {
    f32x4 s = *reinterpret_cast<const f32x4*>(part + i);
    for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(part + k * MN + i);
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)s[j];
    *reinterpret_cast<bf16x4*>(C + i) = o;
  }
}

}  // namespace

int launch_gemm_nt(bf16* C, const bf16* A, const bf16* B, float* workspace, int M, int N, int K,
                   int splits, int bn, hipStream_t stream) {
  if (M <= 0 || M > kBM || K % kBK != 0 || N % bn != 0 || splits < 1) return -1;
  if ((K / kBK) % splits != 0) return -2;
  const int kps = K / splits;
  if (splits > 1 && workspace == nullptr) return -3;
  dim3 grid(N / bn, splits);
  float* part = splits > 1 ? workspace : nullptr;
  if (bn == 128)
    gemm_nt_kernel<128><<<grid, kThreads, 0, stream>>>(A, B, C, part, M, N, K, kps);
  else if (bn == 64)
    gemm_nt_kernel<64><<<grid, kThreads, 0, stream>>>(A, B, C, part, M, N, K, kps);
  else
    return -4;
  if (splits > 1) {
    const size_t MN = (size_t)M * N;
    if (MN % 4 != 0) return -5;
    size_t blocks = (MN / 4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<<<(int)blocks, 256, 0, stream>>>(C, workspace, splits, MN);
  }
  return 0;
}

}  // namespace dli
