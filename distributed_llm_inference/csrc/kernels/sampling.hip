// Token sampling on the last pipeline stage (absent in the reference, which has no LM head —
// SURVEY K13; required to close the generation loop of SURVEY §3.6).
//
// One 1024-thread workgroup per row of logits [B, V] (V = 128256 for Llama-3):
//   * temperature <= 0  -> greedy argmax (ties -> lowest index), one pass.
//   * bf16 rows with V % 8 == 0 and V <= 131072 (sample_row_regs): the row stays in registers and
//     the top-k / top-p thresholds come from a 4-ary search over 16-bit value keys with block
//     reductions — same kept set and Gumbel draw as below, deterministic, 2.2-2.9x faster
//     (profiles/sample_probe.json: top-p over 512 x 128256 1.02 ms -> 0.38 ms, one row 365 ->
//     161 us, identical tokens); the radix path remains for fp32 logits and odd vocabularies.
//   * otherwise x = logits / T, then optional top-k and top-p filtering by *radix select* on the
//     order-preserving uint32 image of x (4 passes of 8 bits, LDS histograms: counts for top-k,
//     probability mass for top-p), and finally Gumbel-max over the kept set:
//     argmax(x_i + g_i), g_i = -log(-log(u_i)) — an exact sample of the renormalised softmax with
//     no sort and no normalisation pass.  u_i comes from a counter-based hash of
//     (seed, ctr[row], i), ctr = the sampled token's position in its sequence: a seeded request
//     draws the same tokens whatever batch, micro-batch, pipeline depth or rank samples it, and a
//     replayed graph gets fresh randomness from the device-side counters.  Without per-row
//     counters (seed, step, row, i) are used.
//   * optional log-probability of the chosen token under softmax(x).
#include "kernels.h"

namespace dli {


__device__ __forceinline__ float load_logit(const SampleParams& p, int row, int i) {
  if (p.logits_is_f32) return reinterpret_cast<const float*>(p.logits)[row * p.row_stride + i];
  return (float)reinterpret_cast<const bf16*>(p.logits)[row * p.row_stride + i];
}

__device__ __forceinline__ unsigned f2key(float f) {
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float uniform01(unsigned long long seed, unsigned long long ctr) {
  const unsigned long long r = splitmix64(seed ^ splitmix64(ctr));
  // 24 random bits -> (0, 1)
  return ((float)(r >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// block argmax of (value, index) pairs; lower index wins ties.
__device__ __forceinline__ void argmax_pair(float& v, int& idx, float ov, int oi) {
  if (ov > v || (ov == v && oi < idx)) {
    v = ov;
    idx = oi;
  }
}

__device__ void block_argmax(float& v, int& idx, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    argmax_pair(v, idx, ov, oi);
  }
  const int nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x >> 6] = v;
    si[threadIdx.x >> 6] = idx;
  }
  __syncthreads();
  v = sv[0];
  idx = si[0];
  for (int i = 1; i < nw; ++i) argmax_pair(v, idx, sv[i], si[i]);
  __syncthreads();
}

// 16-bit order-preserving key of a bf16 value (larger key <=> larger value); for inv_t > 0 the
// order of x = v * inv_t is the order of v, so top-k / top-p thresholds can be searched on it
__device__ __forceinline__ unsigned bkey(unsigned short u) {
  return (u & 0x8000u) ? (~u & 0xFFFFu) : (u | 0x8000u);
}

// block sums of three values with one pair of barriers (deterministic order)
__device__ __forceinline__ void block_reduce_sum3(float& a, float& b, float& c, float* sc) {
  a = wave_reduce_sum(a);
  b = wave_reduce_sum(b);
  c = wave_reduce_sum(c);
  const int nw = blockDim.x >> 6;
  if (lane_id() == 0) {
    sc[wave_id()] = a;
    sc[16 + wave_id()] = b;
    sc[32 + wave_id()] = c;
  }
  __syncthreads();
  a = b = c = 0.f;
  for (int i = 0; i < nw; ++i) {
    a += sc[i];
    b += sc[16 + i];
    c += sc[32 + i];
  }
  __syncthreads();
}

// Temperature sampling with the bf16 row held in registers (NV 16-byte vectors per lane of a
// 1024-thread workgroup; V % 8 == 0): every pass reads registers, not memory, and the top-k /
// top-p thresholds come from a 4-ary search over the 16-bit value keys with block reductions of
// counts / probability mass (three candidate thresholds per pass, 8 passes) instead of radix
// histograms built with LDS atomics (which serialise: most of a row shares a few exponent bins).
// Same kept set as the radix select (the largest threshold whose count reaches k / whose mass
// reaches top_p x the kept mass, ties at it kept), same Gumbel-max draw, deterministic sums.
template <int NV>
__device__ __forceinline__ void sample_row_regs(const SampleParams& p, int row, float temp) {
  __shared__ float sc[48];
  __shared__ float s_f[16];
  __shared__ int s_i[16];
  const int V = p.V, n8 = V >> 3;
  const uint4* r8 = reinterpret_cast<const uint4*>(static_cast<const bf16*>(p.logits) +
                                                   (size_t)row * p.row_stride);
  // the row as packed bf16 pairs: element 2q of vector u in the low half of w[u][q]
  unsigned w[NV][4];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i8 = threadIdx.x + u * blockDim.x;
    const uint4 t = r8[i8 < n8 ? i8 : n8 - 1];
    w[u][0] = t.x; w[u][1] = t.y; w[u][2] = t.z; w[u][3] = t.w;
  }
  // an empty asm use per pass keeps every per-element value from being hoisted out of the
  // search loop (which would hold 2 x NV x 8 extra registers and spill)
  auto pin = [&]() {
#pragma unroll
    for (int u = 0; u < NV; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(w[u][q]));
  };
  auto valid = [&](int u) { return threadIdx.x + u * (int)blockDim.x < n8; };
  // element e (0..7) of vector u: bf16 bits as float / as 16-bit key
  auto fval = [&](int u, int e) {
    const unsigned x = w[u][e >> 1];
    return __uint_as_float((e & 1) ? (x & 0xFFFF0000u) : (x << 16));
  };
  auto key = [&](int u, int e) {
    const unsigned x = w[u][e >> 1];
    return bkey((unsigned short)((e & 1) ? (x >> 16) : (x & 0xFFFFu)));
  };
  const float inv_t = 1.f / temp;
  // row max, and the key range [kmin, kmax] the thresholds can lie in
  float mx = -INFINITY, kmin = 65535.f, kmax = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u)
    if (valid(u))
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mx = fmaxf(mx, fval(u, e) * inv_t);
        const float kf = (float)key(u, e);
        kmin = fminf(kmin, kf);
        kmax = fmaxf(kmax, kf);
      }
  mx = block_reduce_max(mx, s_f);
  kmax = block_reduce_max(kmax, s_f);
  kmin = -block_reduce_max(-kmin, s_f);

  // 4-ary search for the largest t in [lo, hi) with f(t) >= goal, f(t) = count or probability
  // mass of the elements with key >= t (non-increasing; f(lo) >= goal).  `above` = f(hi) is
  // carried, so a pass only visits elements with lo <= key < hi - after the first passes few of
  // them, and a wave skips an element slot none of its lanes has in range.  With z_out the
  // first pass also sums the mass of every key >= lo (top-p's total) and the goal is
  // goal * that total (the thresholds of the first pass do not depend on it).
  auto search = [&](unsigned lo, unsigned hi, float goal, bool mass, float* z_out) {
    float above = 0.f;
    bool first = true;
    while (hi - lo > 1) {
      const unsigned span = hi - lo;
      const unsigned t1 = lo + (span + 3) / 4, t2 = lo + (span + 1) / 2, t3 = lo + (3 * span + 3) / 4;
      float a = 0.f, b = 0.f, c = 0.f, z = 0.f;
      pin();
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        if (!valid(u)) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const unsigned k = key(u, e);
          if (k >= lo && k < hi) {
            const float m = mass ? __expf(fval(u, e) * inv_t - mx) : 1.f;
            z += m;
            a += k >= t1 ? m : 0.f;
            b += k >= t2 ? m : 0.f;
            c += k >= t3 ? m : 0.f;
          }
        }
      }
      if (first && z_out) {
        block_reduce_sum3(a, b, c, sc);
        z = block_reduce_sum(z, s_f);
        *z_out = z;
        goal *= z;
      } else {
        block_reduce_sum3(a, b, c, sc);
      }
      first = false;
      // t1 <= t2 <= t3 (they may coincide on tiny spans): the highest one reaching the goal
      if (above + c >= goal && t3 < hi) {
        lo = t3;
      } else if (above + b >= goal && t2 < hi) {
        if (t3 > t2) { hi = t3; above += c; }
        lo = t2;
      } else if (above + a >= goal && t1 < hi) {
        if (t2 > t1) { hi = t2; above += b; }
        lo = t1;
      } else {
        if (t1 > lo) { hi = t1; above += a; } else { hi = lo + 1; }
      }
    }
    return lo;
  };
  unsigned thr = (unsigned)kmin;   // keep keys >= thr
  const unsigned khi = (unsigned)kmax + 1;
  const int k = p.top_k ? p.top_k[row] : 0;
  if (k > 0 && k < V) thr = search(thr, khi, (float)k, false, nullptr);
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  if (tp < 1.f) {
    float z = 0.f;
    thr = search(thr, khi, tp, true, &z);
  }
  // Gumbel-max over the kept set (the same draw as the radix path)
  const unsigned long long seed = p.seeds ? p.seeds[row] : 0x1234ull;
  const unsigned long long st = p.step ? (unsigned long long)p.step[0] : 0ull;
  const unsigned long long base =
      p.ctr ? (unsigned long long)p.ctr[row] * 0x100000001B3ull
            : (st * 0x100000001B3ull) ^ ((unsigned long long)row << 40);
  float best = -INFINITY;
  int bi = 0x7fffffff;
  pin();
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    if (!valid(u)) continue;
    const int i0 = (threadIdx.x + u * blockDim.x) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (key(u, e) < thr) continue;
      const float uu = uniform01(seed, base + (unsigned long long)(i0 + e));
      argmax_pair(best, bi, fval(u, e) * inv_t - __logf(-__logf(uu)), i0 + e);
    }
  }
  block_argmax(best, bi, s_f, s_i);
  if (bi >= V) bi = 0;
  if (p.out_logprobs) {
    float sm = 0.f;
    pin();
#pragma unroll
    for (int u = 0; u < NV; ++u)
      if (valid(u))
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += __expf(fval(u, e) * inv_t - mx);
    sm = block_reduce_sum(sm, s_f);
    if (threadIdx.x == 0) p.out_logprobs[row] = load_logit(p, row, bi) * inv_t - mx - logf(sm);
  }
  if (threadIdx.x == 0) p.out_tokens[row] = bi;
}

// NV > 0: bf16 rows of at most NV * 8 * 1024 values (V % 8 == 0) take the register path for
// temperature > 0 (sample_row_regs); NV == 0: the radix-histogram path below
template <int NV>
__global__ void __launch_bounds__(1024) sample_kernel(SampleParams p) {
  const int row = blockIdx.x;
  const int V = p.V;
  __shared__ float s_f[16];
  __shared__ int s_i[16];
  __shared__ unsigned h_cnt[256];
  __shared__ float h_mass[256];
  __shared__ unsigned s_prefix;
  __shared__ float s_target;
  __shared__ unsigned s_remaining;

  const float temp = p.temperature ? p.temperature[row] : 0.f;
  // ---------------- greedy ----------------
  if (!(temp > 0.f)) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    if (!p.logits_is_f32 && V % 8 == 0 && p.row_stride % 8 == 0) {
      // bf16 rows: 16-byte loads, 4 in flight per lane (a 128256-wide row is ~16 vectors per
      // lane instead of ~125 dependent 2-byte loads); the argmax is order-independent
      // (lower index wins ties), so the result equals the element-wise loop's
      const bf16x8* r8 = reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(p.logits) +
                                                         (size_t)row * p.row_stride);
      const int n8 = V >> 3;
      for (int base = threadIdx.x; base < n8; base += 4 * blockDim.x) {
        bf16x8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i8 = base + u * blockDim.x;
          v[u] = r8[i8 < n8 ? i8 : n8 - 1];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i8 = base + u * blockDim.x;
          if (i8 < n8)
#pragma unroll
            for (int j = 0; j < 8; ++j) argmax_pair(best, bi, (float)v[u][j], i8 * 8 + j);
        }
      }
    } else {
      for (int i = threadIdx.x; i < V; i += blockDim.x) argmax_pair(best, bi, load_logit(p, row, i), i);
    }
    block_argmax(best, bi, s_f, s_i);
    if (p.out_logprobs) {
      float s = 0.f;
      for (int i = threadIdx.x; i < V; i += blockDim.x) s += __expf(load_logit(p, row, i) - best);
      s = block_reduce_sum(s, s_f);
      if (threadIdx.x == 0) p.out_logprobs[row] = -logf(s);
    }
    if (threadIdx.x == 0) p.out_tokens[row] = bi;
    return;
  }
  if constexpr (NV > 0) {
    sample_row_regs<NV>(p, row, temp);
    return;
  }
  const float inv_t = 1.f / temp;
  // row max of x
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < V; i += blockDim.x) mx = fmaxf(mx, load_logit(p, row, i) * inv_t);
  mx = block_reduce_max(mx, s_f);

  unsigned thr_key = 0;  // keep elements with key >= thr_key
  // ---------------- top-k (radix select on counts) ----------------
  const int k = p.top_k ? p.top_k[row] : 0;
  if (k > 0 && k < V) {
    unsigned prefix = 0, remaining = (unsigned)k;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      const unsigned hi_mask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
      for (int i = threadIdx.x; i < 256; i += blockDim.x) h_cnt[i] = 0;
      __syncthreads();
      for (int i = threadIdx.x; i < V; i += blockDim.x) {
        const unsigned key = f2key(load_logit(p, row, i) * inv_t);
        if ((key & hi_mask) == (prefix & hi_mask)) atomicAdd(&h_cnt[(key >> shift) & 255], 1u);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned acc = 0;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (acc + h_cnt[bin] >= remaining) break;
          acc += h_cnt[bin];
        }
        s_prefix = prefix | ((unsigned)bin << shift);
        s_remaining = remaining - acc;
      }
      __syncthreads();
      prefix = s_prefix;
      remaining = s_remaining;
      __syncthreads();
    }
    thr_key = prefix;
  }
  // ---------------- top-p (radix select on probability mass) ----------------
  const float tp = p.top_p ? p.top_p[row] : 1.f;
  if (tp < 1.f) {
    float z = 0.f;
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float x = load_logit(p, row, i) * inv_t;
      if (f2key(x) >= thr_key) z += __expf(x - mx);
    }
    z = block_reduce_sum(z, s_f);
    unsigned prefix = 0;
    float target = tp * z;  // mass that must be covered, from the top
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      const unsigned hi_mask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
      for (int i = threadIdx.x; i < 256; i += blockDim.x) h_mass[i] = 0.f;
      __syncthreads();
      for (int i = threadIdx.x; i < V; i += blockDim.x) {
        const float x = load_logit(p, row, i) * inv_t;
        const unsigned key = f2key(x);
        if (key >= thr_key && (key & hi_mask) == (prefix & hi_mask))
          atomicAdd(&h_mass[(key >> shift) & 255], __expf(x - mx));
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        float acc = 0.f;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (acc + h_mass[bin] >= target) break;
          acc += h_mass[bin];
        }
        s_prefix = prefix | ((unsigned)bin << shift);
        s_target = target - acc;
      }
      __syncthreads();
      prefix = s_prefix;
      target = s_target;
      __syncthreads();
    }
    thr_key = thr_key > prefix ? thr_key : prefix;
  }
  // ---------------- Gumbel-max over the kept set ----------------
  const unsigned long long seed = p.seeds ? p.seeds[row] : 0x1234ull;
  const unsigned long long st = p.step ? (unsigned long long)p.step[0] : 0ull;
  const unsigned long long base =
      p.ctr ? (unsigned long long)p.ctr[row] * 0x100000001B3ull
            : (st * 0x100000001B3ull) ^ ((unsigned long long)row << 40);
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float x = load_logit(p, row, i) * inv_t;
    if (f2key(x) < thr_key) continue;
    const float u = uniform01(seed, base + (unsigned long long)i);
    const float g = -__logf(-__logf(u));
    argmax_pair(best, bi, x + g, i);
  }
  block_argmax(best, bi, s_f, s_i);
  if (bi >= V) bi = 0;
  if (p.out_logprobs) {
    float s = 0.f;
    for (int i = threadIdx.x; i < V; i += blockDim.x) s += __expf(load_logit(p, row, i) * inv_t - mx);
    s = block_reduce_sum(s, s_f);
    if (threadIdx.x == 0) p.out_logprobs[row] = load_logit(p, row, bi) * inv_t - mx - logf(s);
  }
  if (threadIdx.x == 0) p.out_tokens[row] = bi;
}

int launch_sample(const SampleParams& p, int B, hipStream_t stream) {
  if (B == 0) return 0;
  const int n8 = p.V / 8;
  const bool regs = !p.logits_is_f32 && p.V % 8 == 0 && p.row_stride % 8 == 0;
  if (regs && n8 <= 4 * 1024)
    sample_kernel<4><<<B, 1024, 0, stream>>>(p);
  else if (regs && n8 <= 8 * 1024)
    sample_kernel<8><<<B, 1024, 0, stream>>>(p);
  else if (regs && n8 <= 16 * 1024)
    sample_kernel<16><<<B, 1024, 0, stream>>>(p);
  else
    sample_kernel<0><<<B, 1024, 0, stream>>>(p);
  return 0;
}

}  // namespace dli
