// Skinny GEMM for small decode batches:  y[M, N] = x[M, K] . W[N, K]^T (+ bias),  M <= 4.
//
// At M <= 4 a projection is a pure weight stream (70B bf16: 140 GB per decode step), and the
// tuned hipBLASLt solutions reach only ~4.7 TB/s of it (measured: Llama-3-70B batch 1 decode
// 29.8 ms/token against a 17.6 ms HBM floor).  cdna_hip_programming.md's rule for "GEMV / M <= 16
// decode weights: operand streamed once per block and not shared across waves": no LDS, load
// straight to VGPRs, deep unroll, late vmcnt.  So:
//   * one wave per ROWS = 2 consecutive weight rows; lanes stride K by 8 elements (16-B loads), a
//     wave instruction covers 1 KiB of a row;
//   * UNROLL = 4 k-steps of loads are issued before any FMA (8 x 16 B of weights in flight per
//     lane, ~16 waves per CU -> ~128 KiB per CU in flight, enough to cover HBM latency);
//   * weight loads are non-temporal (streamed exactly once: keep them out of the way of x, which
//     every wave re-reads and stays L1/L2-resident);
//   * v_dot2c_f32_bf16 (two bf16 products into an fp32 accumulator per instruction, no bf16->f32
//     conversions): plain conversions + FMAs made M = 4 VALU-bound; one wave reduction per
//     (m, row) at the end, lane 0 stores.
#include "kernels.h"
#include "gemv_core.h"

namespace dli {

namespace {

constexpr int kUnroll = 4;

// NORM (fused input RMSNorm, 1-2 decode rows): the GEMV's x is rmsnorm(x + res_in) * w, computed
// once per workgroup into LDS by the same arithmetic as norm.hip's rms_norm_kernel (same
// per-thread vector assignment, fma order and block reduction at 256 threads), so the normalised
// row is bit-identical to the separate kernel's; workgroup 0 also writes res_out = x + res_in
// (the residual stream; it must not alias res_in, which every workgroup reads).  Saves one
// launch per norm in the 1-2 row decode step, where every launch costs its dispatch latency.
extern __shared__ __attribute__((aligned(16))) char gemv_lds[];

// rows of K <= 8 * 4 * 256 (every Llama hidden size up to 8192): each thread's 4 vectors of every
// row (and the norm weight) are loaded in one burst and kept in registers through the reduction --
// one L2 round trip instead of the generic loop's one per vector and a second pass for w.  Same
// vector assignment and fma order as the generic loop, so the same bits.
//
// `issue` (the caller's first weight group, which does not depend on x) runs right after the
// prologue's own loads: vmcnt retires loads in order, so a weight group issued BEFORE them would
// have to land before the norm could start (measured: at 8 k-steps per group the fused-norm
// GEMVs ran 30-40 % slower, profiles/r4/gemv_unroll8_ab.txt); issued after, it stays in flight
// through the reduction.
template <int M, typename F>
__device__ __forceinline__ void gemv_norm_prologue_regs(const bf16* __restrict__ x,
                                                        const GemvNorm& nm, int K,
                                                        float* scratch, F&& issue) {
  constexpr int VPT = 4;
  const int nvec = K >> 3;
  bf16x8* xs = reinterpret_cast<bf16x8*>(gemv_lds);
  const bf16x8* w8 = reinterpret_cast<const bf16x8*>(nm.w);
  bf16x8 wv[VPT], a[M][VPT], rv[M][VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) wv[i] = w8[row_vec_idx(i, nvec)];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      a[m][i] = reinterpret_cast<const bf16x8*>(x + (size_t)m * K)[row_vec_idx(i, nvec)];
      if (nm.res_in != nullptr)
        rv[m][i] = reinterpret_cast<const bf16x8*>(nm.res_in + (size_t)m * K)[row_vec_idx(i, nvec)];
    }
  __builtin_amdgcn_sched_barrier(0);
  issue();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    bf16x8* ro = nm.res_out ? reinterpret_cast<bf16x8*>(nm.res_out + (size_t)m * K) : nullptr;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      if (!row_valid(i, nvec)) continue;
      if (nm.res_in != nullptr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[m][i][j] = (bf16)((float)a[m][i][j] + (float)rv[m][i][j]);
        if (ro != nullptr && blockIdx.x == 0) ro[threadIdx.x + i * blockDim.x] = a[m][i];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (float)a[m][i][j];
        ss = __builtin_fmaf(v, v, ss);
      }
    }
    ss = block_reduce_sum(ss, scratch);
    const float rstd = rsqrtf(ss / (float)K + nm.eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      if (!row_valid(i, nvec)) continue;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)a[m][i][j] * rstd * (float)wv[i][j]);
      xs[(size_t)m * nvec + threadIdx.x + i * blockDim.x] = o;
    }
  }
  __syncthreads();
}

template <int M, typename F>
__device__ __forceinline__ void gemv_norm_prologue(const bf16* __restrict__ x, const GemvNorm& nm,
                                                   int K, F&& issue) {
  __shared__ float scratch[8];
  const int nvec = K >> 3;
  if (nvec <= 4 * (int)blockDim.x) {
    gemv_norm_prologue_regs<M>(x, nm, K, scratch, issue);
    return;
  }
  issue();
  bf16* xs = reinterpret_cast<bf16*>(gemv_lds);
  const bf16x8* w8 = reinterpret_cast<const bf16x8*>(nm.w);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)m * K);
    const bf16x8* rr = nm.res_in ? reinterpret_cast<const bf16x8*>(nm.res_in + (size_t)m * K) : nullptr;
    bf16x8* ro = nm.res_out ? reinterpret_cast<bf16x8*>(nm.res_out + (size_t)m * K) : nullptr;
    bf16x8* xo = reinterpret_cast<bf16x8*>(xs + (size_t)m * K);
    float ss = 0.f;
    for (int idx = threadIdx.x; idx < nvec; idx += blockDim.x) {
      bf16x8 a = xr[idx];
      if (rr != nullptr) {
        const bf16x8 r = rr[idx];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (bf16)((float)a[j] + (float)r[j]);
        if (ro != nullptr && blockIdx.x == 0) ro[idx] = a;
      }
      xo[idx] = a;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (float)a[j];
        ss = __builtin_fmaf(v, v, ss);
      }
    }
    ss = block_reduce_sum(ss, scratch);
    const float rstd = rsqrtf(ss / (float)K + nm.eps);
    for (int idx = threadIdx.x; idx < nvec; idx += blockDim.x) {   // own elements only
      const bf16x8 a = xo[idx], ww = w8[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)a[j] * rstd * (float)ww[j]);
      xo[idx] = o;
    }
  }
  __syncthreads();
}

template <int M, int EP = kEpPlain, bool NORM = false>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(const bf16* __restrict__ x_in,
                                                          const bf16* __restrict__ W,
                                                          const bf16* __restrict__ bias,
                                                          bf16* __restrict__ y, int N, int K,
                                                          GemvNorm nm, GemvRope rp) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int n0 = wave * kRows;
  const bf16* wrow[kRows];   // rows clamped: the loads below never leave W, even for idle waves
#pragma unroll
  for (int r = 0; r < kRows; ++r) wrow[r] = W + (size_t)min(gemv_row<EP>(wave, r, rp), N - 1) * K;
  constexpr int kStep = 64 * 8;  // elements per wave instruction
  bf16x8 wv[kUnroll][kRows];
  auto load_w = [&](int u, int k) {
#pragma unroll
    for (int r = 0; r < kRows; ++r)
      wv[u][r] = k < K ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wrow[r] + k))
                       : bf16x8{};
  };

  const int kfirst = lane * 8;
  if constexpr (NORM) {
    // the first k-group of weights does not depend on x: in flight during the norm prologue
    // (only here: with x from global memory the per-step weight / x interleave below is faster)
    // (the unconditional-load form of skinny_gemm_fp8_kernel's load_w_pre measured -0.4 % on
    // the bf16 batch-1 step, profiles/r4/gemv_prologue_ab.txt: not used here)
    gemv_norm_prologue<M>(x_in, nm, K, [&] {   // every thread, before any exit
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) load_w(u, kfirst + u * kStep);
    });
  }
  const bf16* x = NORM ? reinterpret_cast<const bf16*>(gemv_lds) : x_in;
  if ((EP != kEpPlain ? 2 * wave : n0) >= N) return;
  float acc[M][kRows];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kRows; ++r) acc[m][r] = 0.f;

  for (int k0 = kfirst; k0 < K; k0 += kStep * kUnroll) {
    const bool pre = NORM && k0 == kfirst;
    bf16x8 xv[kUnroll][M];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = k0 + u * kStep;
      if (!pre) load_w(u, k);
#pragma unroll
      for (int m = 0; m < M; ++m)
        xv[u][m] = k < K ? *reinterpret_cast<const bf16x8*>(x + (size_t)m * K + k) : bf16x8{};
    }
    // v_dot2c_f32_bf16: two bf16 products accumulated in fp32 per instruction, no conversions
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const bf16x2 xp = {xv[u][m][2 * j], xv[u][m][2 * j + 1]};
#pragma unroll
          for (int r = 0; r < kRows; ++r) {
            const bf16x2 wp = {wv[u][r][2 * j], wv[u][r][2 * j + 1]};
            acc[m][r] = __builtin_amdgcn_fdot2_f32_bf16(xp, wp, acc[m][r], false);
          }
        }
  }
  float v[M][kRows];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int n = min(gemv_row<EP>(wave, r, rp), N - 1);
      v[m][r] = wave_reduce_sum(acc[m][r]) + (bias ? (float)bias[n] : 0.f);
    }
  gemv_store<EP, M>(v, wave, lane, N, y, rp);
}

// fp8 e4m3 weights [N, K] with one fp32 scale per output row: the same weight stream at half
// the bytes.  A lane takes 16 consecutive k (one 16-B load per row), widens them to bf16 with
// v_cvt_scalef32_pk_bf16_fp8 (exact) and accumulates with v_dot2c_f32_bf16 against the
// activations — bf16, or (XF8) the fp8 rows + per-row scales the fused RMSNorm quantiser already
// produced, widened the same way; the scales are applied once to the reduced sum:
// y = wscale[n] * (xscale[m]) * sum_k x[m, k] * w8[n, k].
// WI8: int8 weights instead (LLM.int8 mode's [N, K] int8 + per-row scale).  Each byte is biased
// to unsigned (one v_xor_b32 per 4 bytes: b ^ 0x80 = b + 128), converted by v_cvt_f32_ubyteN
// (exact; an integer below 256 has its bf16 in the top half of its fp32), and two top halves are
// packed into one bf16 pair by v_perm_b32 -- 2.25 VALU per weight byte instead of a per-byte
// sign-extend / convert / round chain.  The bias is removed once from the reduced sum:
// sum x * w = sum x * (w + 128) - 128 * sum x, with sum x accumulated by one extra dot per pair.
template <int M, bool XF8, bool WI8 = false, int EP = kEpPlain, bool NORM = false>
__global__ void __launch_bounds__(256) skinny_gemm_fp8_kernel(const void* __restrict__ x_in,
                                                              const float* __restrict__ xscale,
                                                              const uint8_t* __restrict__ W,
                                                              const float* __restrict__ wscale,
                                                              const bf16* __restrict__ bias,
                                                              bf16* __restrict__ y, int N, int K,
                                                              GemvNorm nm, GemvRope rp) {
  static_assert(!(NORM && XF8), "the fused norm feeds bf16 rows");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int n0 = wave * kRows;
  const uint8_t* wrow[kRows];   // rows clamped: the loads below never leave W, even for idle waves
#pragma unroll
  for (int r = 0; r < kRows; ++r) wrow[r] = W + (size_t)min(gemv_row<EP>(wave, r, rp), N - 1) * K;
  constexpr int kStep = 64 * 16;  // elements per wave instruction
  u32x4n wv[kUnroll][kRows];
  auto load_w = [&](int u, int k) {
#pragma unroll
    for (int r = 0; r < kRows; ++r)
      wv[u][r] = k < K ? __builtin_nontemporal_load(reinterpret_cast<const u32x4n*>(wrow[r] + k))
                       : u32x4n{0u, 0u, 0u, 0u};
  };
  // the weight group issued during the norm prologue: loads past the row end (k >= K, only when
  // K is not a multiple of the group) re-read the row's last 16 bytes instead of branching around
  // the load, so every load is unconditional and hipcc counts the prologue's vmcnt waits (with
  // exec-masked loads it waited for the whole group: measured 30-40 % slower fused-norm GEMVs at
  // 8 k-steps per group).  Their x is zero, so they add exact zeros (finite weights).  The loop's
  // own loads keep the branch: its interleaved schedule measured faster (O 13.2 vs 15.0 us).
  auto load_w_pre = [&](int u, int k) {
    const int kc = k < K ? k : K - 16;
#pragma unroll
    for (int r = 0; r < kRows; ++r)
      wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4n*>(wrow[r] + kc));
  };
  const int kfirst = lane * 16;
  if constexpr (NORM) {
    // the first k-group of weights does not depend on x: in flight during the norm prologue
    // (only here: with x from global memory the per-step weight / x interleave below is faster)
    gemv_norm_prologue<M>(static_cast<const bf16*>(x_in), nm, K, [&] {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) load_w_pre(u, kfirst + u * kStep);
    });
  }
  const void* xv_ = NORM ? static_cast<const void*>(gemv_lds) : x_in;
  if ((EP != kEpPlain ? 2 * wave : n0) >= N) return;
  float acc[M][kRows];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kRows; ++r) acc[m][r] = 0.f;
  float sx[M];   // WI8: sum of this lane's x (the unsigned-bias correction)
#pragma unroll
  for (int m = 0; m < M; ++m) sx[m] = 0.f;

  for (int k0 = kfirst; k0 < K; k0 += kStep * kUnroll) {
    const bool pre = NORM && k0 == kfirst;
    bf16x8 xv[kUnroll][M][2];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = k0 + u * kStep;
      if (!pre) load_w(u, k);
      if (k < K) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          if constexpr (XF8) {
            const uint4 xb = *reinterpret_cast<const uint4*>(
                static_cast<const uint8_t*>(xv_) + (size_t)m * K + k);
            xv[u][m][0] = fp8x8_to_bf16x8(uint2{xb.x, xb.y});
            xv[u][m][1] = fp8x8_to_bf16x8(uint2{xb.z, xb.w});
          } else {
            const bf16* x = static_cast<const bf16*>(xv_);
            xv[u][m][0] = *reinterpret_cast<const bf16x8*>(x + (size_t)m * K + k);
            xv[u][m][1] = *reinterpret_cast<const bf16x8*>(x + (size_t)m * K + k + 8);
          }
        }
      } else {
#pragma unroll
        for (int m = 0; m < M; ++m) xv[u][m][0] = xv[u][m][1] = bf16x8{};
      }
    }
    if constexpr (WI8) {
      // sum x of this lane's k (once per row m, shared by the kRows weight rows)
      const bf16x2 ones = {(bf16)1.f, (bf16)1.f};
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              sx[m] = __builtin_amdgcn_fdot2_f32_bf16(
                  bf16x2{xv[u][m][h][2 * j], xv[u][m][h][2 * j + 1]}, ones, sx[m], false);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int d = 0; d < 4; ++d) {   // dword d = bytes 4d .. 4d+3 = x pairs (2d, 2d+1)
            const unsigned ub = wv[u][r][d] ^ 0x80808080u;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const bf16x2 wp = u8pair_to_bf16x2(ub, j);
              const int e = (d & 1) * 4 + 2 * j;   // element of the 8-wide x half d >> 1
#pragma unroll
              for (int m = 0; m < M; ++m)
                acc[m][r] = __builtin_amdgcn_fdot2_f32_bf16(
                    bf16x2{xv[u][m][d >> 1][e], xv[u][m][d >> 1][e + 1]}, wp, acc[m][r], false);
            }
          }
    } else {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
          const bf16x8 w0 = fp8x8_to_bf16x8(uint2{wv[u][r][0], wv[u][r][1]});
          const bf16x8 w1 = fp8x8_to_bf16x8(uint2{wv[u][r][2], wv[u][r][3]});
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int m = 0; m < M; ++m) {
              const bf16x2 x0 = {xv[u][m][0][2 * j], xv[u][m][0][2 * j + 1]};
              const bf16x2 x1 = {xv[u][m][1][2 * j], xv[u][m][1][2 * j + 1]};
              acc[m][r] = __builtin_amdgcn_fdot2_f32_bf16(x0, bf16x2{w0[2 * j], w0[2 * j + 1]},
                                                          acc[m][r], false);
              acc[m][r] = __builtin_amdgcn_fdot2_f32_bf16(x1, bf16x2{w1[2 * j], w1[2 * j + 1]},
                                                          acc[m][r], false);
            }
        }
    }
  }
  if constexpr (WI8) {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < kRows; ++r) acc[m][r] -= 128.f * sx[m];
  }
  float v[M][kRows];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int n = min(gemv_row<EP>(wave, r, rp), N - 1);
      v[m][r] = wave_reduce_sum(acc[m][r]) * wscale[n] * (XF8 ? xscale[m] : 1.f) +
                (bias ? (float)bias[n] : 0.f);
    }
  gemv_store<EP, M>(v, wave, lane, N, y, rp);
}

}  // namespace

// swiglu: W is a swiglu_interleave'd gate|up weight [N = 2I, K], y is silu(gate) * up [M, I];
// rp (optional): W is the fused QKV weight, the epilogue applies RoPE and writes q / the caches;
// nm (optional): the fused input RMSNorm (x is then the un-normalised row, bf16)
static int gemv_ep(bool swiglu, const GemvRope* rp) {
  return rp != nullptr ? kEpRope : swiglu ? kEpSwiGLU : kEpPlain;
}

template <bool XF8, bool WI8, int M, int EP>
static void launch_fp8_t(bf16* y, const void* x, const float* xscale, const uint8_t* W,
                         const float* wscale, const bf16* bias, int N, int K, const GemvNorm* nm,
                         const GemvRope& rp, int grid, hipStream_t stream) {
  if constexpr (!XF8) {
    if (nm != nullptr) {
      skinny_gemm_fp8_kernel<M, XF8, WI8, EP, true><<<grid, 256, (size_t)M * K * 2, stream>>>(
          x, xscale, W, wscale, bias, y, N, K, *nm, rp);
      return;
    }
  }
  skinny_gemm_fp8_kernel<M, XF8, WI8, EP, false><<<grid, 256, 0, stream>>>(
      x, xscale, W, wscale, bias, y, N, K, GemvNorm{}, rp);
}

template <bool XF8, bool WI8, int M>
static void launch_fp8_ep(bf16* y, const void* x, const float* xscale, const uint8_t* W,
                          const float* wscale, const bf16* bias, int N, int K, int ep,
                          const GemvNorm* nm, const GemvRope* rp, int grid, hipStream_t stream) {
  const GemvRope r = rp ? *rp : GemvRope{};
  if (ep == kEpRope) launch_fp8_t<XF8, WI8, M, kEpRope>(y, x, xscale, W, wscale, bias, N, K, nm, r, grid, stream);
  else if (ep == kEpSwiGLU) launch_fp8_t<XF8, WI8, M, kEpSwiGLU>(y, x, xscale, W, wscale, bias, N, K, nm, r, grid, stream);
  else launch_fp8_t<XF8, WI8, M, kEpPlain>(y, x, xscale, W, wscale, bias, N, K, nm, r, grid, stream);
}

template <bool XF8, bool WI8>
static void launch_fp8_m(bf16* y, const void* x, const float* xscale, const uint8_t* W,
                         const float* wscale, const bf16* bias, int M, int N, int K, bool swiglu,
                         const GemvNorm* nm, const GemvRope* rp, hipStream_t stream) {
  const int ep = gemv_ep(swiglu, rp);
  const int waves = ep != kEpPlain ? N / 2 : (N + kRows - 1) / kRows;
  const int grid = (waves + 3) / 4;
  if (M == 1) launch_fp8_ep<XF8, WI8, 1>(y, x, xscale, W, wscale, bias, N, K, ep, nm, rp, grid, stream);
  else launch_fp8_ep<XF8, WI8, 2>(y, x, xscale, W, wscale, bias, N, K, ep, nm, rp, grid, stream);
}

static bool gemv_norm_ok(const GemvNorm* nm, int M, int K) {
  return nm == nullptr || (nm->w != nullptr && M <= 2 && (size_t)M * K * 2 <= 65536 &&
                           (nm->res_out == nullptr || nm->res_out != nm->res_in));
}

static bool gemv_rope_ok(const GemvRope* rp, bool swiglu, int M, int N) {
  return rp == nullptr ||
         (!swiglu && M <= 2 && rp->D % 2 == 0 && rp->bs % 8 == 0 && rp->q_out != nullptr &&
          N == (rp->nh + 2 * rp->nkv) * rp->D && (rp->cos_sin == nullptr || rp->max_pos > 0));
}

int launch_skinny_gemm_fp8(bf16* y, const void* x, const float* xscale, const uint8_t* W,
                           const float* wscale, const bf16* bias, int M, int N, int K,
                           hipStream_t stream, bool swiglu, const GemvNorm* nm,
                           const GemvRope* rp) {
  if (M < 1 || M > 2 || K % 16 != 0 || N < 1 || (swiglu && N % 32 != 0)) return -1;
  if (!gemv_norm_ok(nm, M, K) || (nm != nullptr && xscale != nullptr)) return -2;
  if (!gemv_rope_ok(rp, swiglu, M, N)) return -3;
  if (xscale != nullptr)
    launch_fp8_m<true, false>(y, x, xscale, W, wscale, bias, M, N, K, swiglu, nullptr, rp, stream);
  else
    launch_fp8_m<false, false>(y, x, xscale, W, wscale, bias, M, N, K, swiglu, nm, rp, stream);
  return 0;
}

int launch_skinny_gemm_int8(bf16* y, const bf16* x, const int8_t* W, const float* wscale,
                            const bf16* bias, int M, int N, int K, hipStream_t stream,
                            bool swiglu, const GemvNorm* nm, const GemvRope* rp) {
  if (M < 1 || M > 2 || K % 16 != 0 || N < 1 || (swiglu && N % 32 != 0)) return -1;
  if (!gemv_norm_ok(nm, M, K)) return -2;
  if (!gemv_rope_ok(rp, swiglu, M, N)) return -3;
  launch_fp8_m<false, true>(y, x, nullptr, reinterpret_cast<const uint8_t*>(W), wscale, bias, M,
                            N, K, swiglu, nm, rp, stream);
  return 0;
}

template <int M, int EP>
static void launch_bf16_t(bf16* y, const bf16* x, const bf16* W, const bf16* bias, int N, int K,
                          const GemvNorm* nm, const GemvRope& rp, int grid, hipStream_t stream) {
  if (nm != nullptr && M <= 2)
    skinny_gemm_kernel<M, EP, true><<<grid, 256, (size_t)M * K * 2, stream>>>(x, W, bias, y, N, K, *nm, rp);
  else
    skinny_gemm_kernel<M, EP, false><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K, GemvNorm{}, rp);
}

template <int M>
static void launch_bf16_ep(bf16* y, const bf16* x, const bf16* W, const bf16* bias, int N, int K,
                           int ep, const GemvNorm* nm, const GemvRope* rp, int grid,
                           hipStream_t stream) {
  const GemvRope r = rp ? *rp : GemvRope{};
  if (ep == kEpRope) launch_bf16_t<M, kEpRope>(y, x, W, bias, N, K, nm, r, grid, stream);
  else if (ep == kEpSwiGLU) launch_bf16_t<M, kEpSwiGLU>(y, x, W, bias, N, K, nm, r, grid, stream);
  else launch_bf16_t<M, kEpPlain>(y, x, W, bias, N, K, nm, r, grid, stream);
}

int launch_skinny_gemm(bf16* y, const bf16* x, const bf16* W, const bf16* bias, int M, int N,
                       int K, hipStream_t stream, bool swiglu, const GemvNorm* nm,
                       const GemvRope* rp) {
  if (M < 1 || M > 4 || K % 8 != 0 || N < 1 || (swiglu && (N % 32 != 0 || M > 2))) return -1;
  if (!gemv_norm_ok(nm, M, K)) return -2;
  if (!gemv_rope_ok(rp, swiglu, M, N)) return -3;
  const int ep = gemv_ep(swiglu, rp);
  const int waves = ep != kEpPlain ? N / 2 : (N + kRows - 1) / kRows;
  const int grid = (waves + 3) / 4;
  switch (M) {
    case 1: launch_bf16_ep<1>(y, x, W, bias, N, K, ep, nm, rp, grid, stream); break;
    case 2: launch_bf16_ep<2>(y, x, W, bias, N, K, ep, nm, rp, grid, stream); break;
    case 3: skinny_gemm_kernel<3><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K, GemvNorm{}, GemvRope{}); break;
    case 4: skinny_gemm_kernel<4><<<grid, 256, 0, stream>>>(x, W, bias, y, N, K, GemvNorm{}, GemvRope{}); break;
  }
  return 0;
}

}  // namespace dli
