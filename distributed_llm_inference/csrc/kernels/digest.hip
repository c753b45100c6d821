// Payload digest of the pipeline data plane's hop-integrity check (parallel/integrity.py).
//
// The reference ships hidden states between block servers (server/backend.py:42) with nothing
// that would notice a corrupted or mis-routed activation; here, during a run's warmup, every
// stage-pair and head-pair message is digested on the sending rank (on its send stream, before
// the send) and on the receiving rank (on the stream the data landed on), and the two are
// compared through the job's store.  Two order-sensitive 64-bit sums over the payload's 32-bit
// words w_i (mod 2^64):  s1 = sum w_i (2i + 1),  s2 = sum (w_i ^ 0x9E3779B9) ((u32)(i 0x85EBCA6B) + 1)
// - odd weights, so any single changed word changes s1; swapped words change both.  Each
// workgroup writes its two partial sums (no atomics); the host folds the partials.  Integer
// sums: the result is independent of the grid, bit for bit, and equals ops/reference.py digest.
#include "kernels.h"

namespace dli {

__global__ void __launch_bounds__(256) digest_kernel(const uint32_t* __restrict__ w, long n,
                                                     unsigned long long* __restrict__ part) {
  unsigned long long s1 = 0, s2 = 0;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const unsigned long long x = w[i];
    s1 += x * (unsigned long long)(2 * i + 1);
    s2 += (x ^ 0x9E3779B9ull) * ((unsigned long long)((unsigned)i * 0x85EBCA6Bu) + 1ull);
  }
  __shared__ unsigned long long r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
#pragma unroll
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = r1[0];
    part[2 * blockIdx.x + 1] = r2[0];
  }
}

int launch_digest(const void* data, long nwords, int64_t* part, int nblocks, hipStream_t stream) {
  if (nblocks < 1) return -1;
  digest_kernel<<<nblocks, 256, 0, stream>>>(static_cast<const uint32_t*>(data), nwords,
                                             reinterpret_cast<unsigned long long*>(part));
  return 0;
}

}  // namespace dli
