// LLM.int8 outlier bookkeeping on the GPU (reference utils/model.py:93-113 -> bitsandbytes
// Linear8bitLt(threshold)): per product, the activation columns whose magnitude exceeds
// `threshold` anywhere in the batch are multiplied in bf16 with the dequantised weight columns.
// Static shapes for graph capture: at most `max_out` columns (the largest ones passing the
// threshold) are taken.  Four kernels replace a torch chain of abs / amax / topk / scatter /
// gathers / casts:
//   * llm_int8_colmax_kernel     colmax[k] = max_m |x[m, k]|   (LDS row-lane fold, one store)
//   * llm_int8_select_kernel     one workgroup: the <= max_out largest columns above threshold,
//                                in column order -> idx[max_out] (padded), sel[max_out], flags[K]
//   * llm_int8_gather_w_kernel   w_out[n, j] = bf16(wq[n, idx[j]] * ws[n]) * sel[j]
//   * llm_int8_gather_wt_kernel  same from the transposed copy wqT [K, N] (coalesced)
//   * llm_int8_gather_x_kernel   x_out[m, j] = x[m, idx[j]] * sel[j]
// The select kernel also stores the number of columns it kept (`cnt`, optional).  Given it, the
// gathers write only the first ceil(cnt / 32) 32-column chunks and the int8 tile GEMM's epilogue
// multiplies only those (gemm_tile.hip OutlierArgs::cnt): the outlier work follows the columns
// actually found (none on most rows of most layers) instead of the static cap.
#include "kernels.h"

namespace dli {

// columns of the static [*, max_out] outlier buffers that are live for this product
__device__ __forceinline__ int live_cols(const int* cnt, int max_out) {
  return cnt ? min(max_out, (*cnt + 31) & ~31) : max_out;
}

// One workgroup per 64 columns: 256 threads = 8 column vectors (8 bf16 each) x 32 row lanes.  A
// wave reads 8 rows x 128 contiguous bytes per load; the 32 row-lane maxima are folded in LDS and
// written once, so no pre-zeroing memset and no atomics.  grid = ceil(K / 64) (>= 128 workgroups
// for the Llama K = 8192 / 28672 projections).
constexpr int kColVecs = 8, kRowLanes = 32;

__global__ void __launch_bounds__(256) llm_int8_colmax_kernel(float* __restrict__ colmax,
                                                              const bf16* __restrict__ x,
                                                              int rows, int K) {
  __shared__ float red[kRowLanes][kColVecs * 8 + 1];
  const int cv = threadIdx.x % kColVecs, lane = threadIdx.x / kColVecs;
  const int v = blockIdx.x * kColVecs + cv;   // 8-column vector index
  const bool live = v * 8 < K;
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (live) {
    const bf16* p = x + (size_t)v * 8;
    int r = lane;
    for (; r + 3 * kRowLanes < rows; r += 4 * kRowLanes) {   // four independent loads in flight
      bf16x8 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        a[u] = *reinterpret_cast<const bf16x8*>(p + (size_t)(r + u * kRowLanes) * K);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf((float)a[u][j]));
    }
    for (; r < rows; r += kRowLanes) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(p + (size_t)r * K);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf((float)a[j]));
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[lane][cv * 8 + j] = m[j];
  __syncthreads();
  if (threadIdx.x < kColVecs * 8) {
    const int c = threadIdx.x;
    float r = red[0][c];
#pragma unroll
    for (int l = 1; l < kRowLanes; ++l) r = fmaxf(r, red[l][c]);
    const int col = blockIdx.x * kColVecs * 8 + c;
    if (col < K) colmax[col] = r;
  }
}

// One 1024-thread workgroup; thread t owns the contiguous columns [t * per, t * per + per) in
// registers (K <= 1024 * kSelMaxPer).  Column maxima are non-negative, so their float bits order
// like the values and the cut is found on the bits.
constexpr int kSelThreads = 1024, kSelMaxPer = 32;

__device__ int block_sum(int c, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  int total = 0;
#pragma unroll
  for (int w = 0; w < kSelThreads / 64; ++w) total += red[w];
  return total;
}

// Exclusive block scan: a shuffle scan per wave, then the 16 wave totals through LDS (2 barriers).
__device__ __forceinline__ int block_exclusive_scan(int x, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  __syncthreads();   // wsum may still be read by an earlier block_sum
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < kSelThreads / 64; ++i) {
    const int t = wsum[i];
    before += i < w ? t : 0;
    total += t;
  }
  return before + inc - x;
}

__global__ void __launch_bounds__(kSelThreads) llm_int8_select_kernel(
    const float* __restrict__ colmax, int K, float threshold, int max_out, long* __restrict__ idx,
    float* __restrict__ sel, uint8_t* __restrict__ flags, int* __restrict__ cnt) {
  __shared__ int red[kSelThreads / 64];
  __shared__ int hist[256];
  __shared__ unsigned s_prefix;
  __shared__ int s_rank, s_bincnt;
  const int per = (K + kSelThreads - 1) / kSelThreads;
  const int k0 = threadIdx.x * per, n_mine = max(0, min(per, K - k0));
  unsigned v[kSelMaxPer];   // padding = +0.0, never above a positive cut
  if ((per & 3) == 0 && n_mine == per) {   // 16-byte loads (k0 = t * per is 4-aligned)
    const uint4* src = reinterpret_cast<const uint4*>(colmax + k0);
#pragma unroll
    for (int i = 0; i < kSelMaxPer / 4; ++i) {
      const uint4 q = 4 * i < per ? src[i] : make_uint4(0u, 0u, 0u, 0u);
      v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kSelMaxPer; ++i) v[i] = i < n_mine ? __float_as_uint(colmax[k0 + i]) : 0u;
  }

  // the cut: |x| >= `threshold` (bitsandbytes Linear8bitLt's outlier test), or -- when more than
  // max_out columns pass it -- strictly above the bits t of the (max_out + 1)-th largest column
  // maximum, found by an MSB-first 8-bit radix select.  Tie policy: columns tied AT that radix cut
  // are all dropped (deterministic, <= max_out kept); ops.llm_int8_linear's CPU path applies the
  // same rule.  Column maxima are >= +0.0, so unsigned bit order is float order.
  unsigned t = __float_as_uint(fmaxf(threshold, 0.f));
  bool strict = false;
  int c = 0;
#pragma unroll
  for (int i = 0; i < kSelMaxPer; ++i) c += i < n_mine && v[i] >= t;
  if (block_sum(c, red) > max_out) {
    strict = true;
    unsigned prefix = 0;
    int r = max_out + 1;   // rank (from the top) of the value being located
    for (int shift = 24; shift >= 0; shift -= 8) {
      const unsigned hmask = shift == 24 ? 0u : 0xffffffffu << (shift + 8);
      if (threadIdx.x < 256) hist[threadIdx.x] = 0;
      __syncthreads();
      // run-length aggregated: a thread's contiguous columns mostly share the high digits, so
      // one LDS atomic per run instead of one per column (same-bin atomics serialise)
      int cur = 0, cnt = 0;
#pragma unroll
      for (int i = 0; i < kSelMaxPer; ++i) {
        if (i < n_mine && (v[i] & hmask) == prefix) {
          const int b = (v[i] >> shift) & 255;
          if (b != cur && cnt) { atomicAdd(&hist[cur], cnt); cnt = 0; }
          cur = b;
          ++cnt;
        }
      }
      if (cnt) atomicAdd(&hist[cur], cnt);
      __syncthreads();
      if (threadIdx.x < 64) {   // wave 0: lane l holds bins 255-4l .. 252-4l (descending)
        const int l = threadIdx.x;
        int h[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) h[q] = hist[255 - 4 * l - q];
        const int mine = h[0] + h[1] + h[2] + h[3];
        int inc = mine;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(inc, o);
          if (l >= o) inc += y;
        }
        const int exc = inc - mine;
        if (exc < r && r <= inc) {   // exactly one lane
          int cum = exc, q = 0;
          for (; q < 3 && cum + h[q] < r; ++q) cum += h[q];
          s_prefix = prefix | ((unsigned)(255 - 4 * l - q) << shift);
          s_rank = r - cum;
          s_bincnt = h[q];
        }
      }
      __syncthreads();
      prefix = s_prefix;
      r = s_rank;
      const int bincnt = s_bincnt;
      __syncthreads();
      if (bincnt == 1) {
        // the located value is the only one with this prefix: every value above it has a larger
        // prefix, so cutting at prefix | (unresolved bits all ones) keeps exactly the same set
        // (and there is no tie to drop) -- the remaining passes are skipped
        prefix |= (1u << shift) - 1u;
        break;
      }
    }
    t = prefix;
  }

  // compaction in column order (block-wide exclusive scan of per-thread counts)
  int mine = 0;
#pragma unroll
  for (int i = 0; i < kSelMaxPer; ++i) mine += i < n_mine && (strict ? v[i] > t : v[i] >= t);
  int total;
  int pos = block_exclusive_scan(mine, red, total);
  if (cnt != nullptr && threadIdx.x == 0) *cnt = min(total, max_out);
#pragma unroll
  for (int i = 0; i < kSelMaxPer; ++i) {
    if (i < n_mine) {
      const bool on = strict ? v[i] > t : v[i] >= t;
      flags[k0 + i] = on ? 1 : 0;
      if (on && pos < max_out) {
        idx[pos] = k0 + i;
        sel[pos] = 1.f;
        ++pos;
      }
    }
  }
  for (int j = min(total, max_out) + threadIdx.x; j < max_out; j += kSelThreads) {
    idx[j] = 0;     // padding: column 0 with weight 0 (contributes nothing)
    sel[j] = 0.f;
  }
}

// Row-major gathers: one thread per output element, numbered chunk-major (32-column chunk, then
// row, then column in the chunk) so a wave covers 2 rows x 32 columns (64-byte store runs) and the
// threads of a chunk past the live columns return at once -- the launch stays as wide as the
// one-element-per-thread form (measured faster than looping rows per thread at ~2 workgroups/CU).
__global__ void __launch_bounds__(256) llm_int8_gather_w_kernel(
    bf16* __restrict__ w_out, const int8_t* __restrict__ wq, const float* __restrict__ ws,
    const long* __restrict__ idx, const float* __restrict__ sel, int N, int K, int max_out,
    const int* __restrict__ cnt) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per_chunk = (long)N * 32;
  const int chunk = (int)(e / per_chunk);
  const int n = (int)((e % per_chunk) >> 5), j = chunk * 32 + (int)(e & 31);
  if (chunk * 32 >= live_cols(cnt, max_out) || j >= max_out) return;
  const float v = (float)wq[(size_t)n * K + idx[j]] * ws[n];
  w_out[(size_t)n * max_out + j] = (bf16)(v * sel[j]);
}

__global__ void __launch_bounds__(256) llm_int8_gather_x_kernel(
    bf16* __restrict__ x_out, const bf16* __restrict__ x, const long* __restrict__ idx,
    const float* __restrict__ sel, int M, int K, int max_out, const int* __restrict__ cnt) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per_chunk = (long)M * 32;
  const int chunk = (int)(e / per_chunk);
  const int m = (int)((e % per_chunk) >> 5), j = chunk * 32 + (int)(e & 31);
  if (chunk * 32 >= live_cols(cnt, max_out) || j >= max_out) return;
  x_out[(size_t)m * max_out + j] = (bf16)((float)x[(size_t)m * K + idx[j]] * sel[j]);
}

int launch_llm_int8_colmax(float* colmax, const bf16* x, int rows, int K, hipStream_t stream) {
  if (K % 8 != 0 || rows < 0) return -1;
  if (K == 0) return 0;
  const int grid = (K + kColVecs * 8 - 1) / (kColVecs * 8);
  llm_int8_colmax_kernel<<<grid, kColVecs * kRowLanes, 0, stream>>>(colmax, x, rows, K);
  return 0;
}

int launch_llm_int8_select(const float* colmax, int K, float threshold, int max_out, long* idx,
                           float* sel, uint8_t* flags, hipStream_t stream, int* cnt) {
  if (K <= 0 || K > kSelThreads * kSelMaxPer || max_out <= 0 || max_out > K) return -1;
  llm_int8_select_kernel<<<1, kSelThreads, 0, stream>>>(colmax, K, threshold, max_out, idx, sel,
                                                         flags, cnt);
  return 0;
}

// Same product from the transposed weight copy wqT [K, N]: a workgroup covers 256 n x 16 j.  Each
// wave reads 4 rows idx[j] as 256 contiguous bytes each (4 independent dword loads per lane), the
// tile is transposed through LDS, and lane n writes its 16 outputs as two 16-byte stores.
// Requires N % 4 == 0 (launcher).
__global__ void __launch_bounds__(256) llm_int8_gather_wt_kernel(
    bf16* __restrict__ w_out, const int8_t* __restrict__ wqT, const float* __restrict__ ws,
    const long* __restrict__ idx, const float* __restrict__ sel, int N, int max_out,
    const int* __restrict__ cnt) {
  __shared__ float tile[16][257];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 256, j0 = blockIdx.y * 16;
  if (j0 >= live_cols(cnt, max_out)) return;   // uniform: the whole workgroup leaves
  const int nl = n0 + 4 * lane;
  unsigned q[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = j0 + wv * 4 + u;
    q[u] = (j < max_out && nl < N)
               ? *reinterpret_cast<const unsigned*>(wqT + (size_t)idx[j] * N + nl) : 0u;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      tile[wv * 4 + u][4 * lane + b] = (float)(int8_t)((q[u] >> (8 * b)) & 255u);
  __syncthreads();
  const int n = n0 + threadIdx.x;
  if (n >= N) return;
  const float sn = ws[n];
  bf16* dst = w_out + (size_t)n * max_out + j0;
  if ((max_out & 7) == 0 && j0 + 16 <= max_out) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (bf16)((tile[8 * h + i][threadIdx.x] * sn) * sel[j0 + 8 * h + i]);
      *reinterpret_cast<bf16x8*>(dst + 8 * h) = o;
    }
  } else {
    for (int i = 0; i < 16 && j0 + i < max_out; ++i)
      dst[i] = (bf16)((tile[i][threadIdx.x] * sn) * sel[j0 + i]);
  }
}

int launch_llm_int8_gather_w(bf16* w_out, const int8_t* wq, const float* ws, const long* idx,
                             const float* sel, int N, int K, int max_out, hipStream_t stream,
                             const int* cnt) {
  if (N < 0 || max_out < 0) return -1;
  if ((long)N * max_out == 0) return 0;
  const long total = (long)((max_out + 31) / 32) * N * 32;
  llm_int8_gather_w_kernel<<<(int)((total + 255) / 256), 256, 0, stream>>>(w_out, wq, ws, idx, sel,
                                                                          N, K, max_out, cnt);
  return 0;
}

int launch_llm_int8_gather_wt(bf16* w_out, const int8_t* wqT, const float* ws, const long* idx,
                              const float* sel, int N, int max_out, hipStream_t stream,
                              const int* cnt) {
  if (N % 4 != 0) return -1;
  if ((long)N * max_out == 0) return 0;
  dim3 grid((N + 255) / 256, (max_out + 15) / 16);
  llm_int8_gather_wt_kernel<<<grid, 256, 0, stream>>>(w_out, wqT, ws, idx, sel, N, max_out, cnt);
  return 0;
}

int launch_llm_int8_gather_x(bf16* x_out, const bf16* x, const long* idx, const float* sel, int M,
                             int K, int max_out, hipStream_t stream, const int* cnt) {
  if (M < 0 || max_out < 0) return -1;
  if ((long)M * max_out == 0) return 0;
  const long total = (long)((max_out + 31) / 32) * M * 32;
  llm_int8_gather_x_kernel<<<(int)((total + 255) / 256), 256, 0, stream>>>(x_out, x, idx, sel, M,
                                                                          K, max_out, cnt);
  return 0;
}

}  // namespace dli
