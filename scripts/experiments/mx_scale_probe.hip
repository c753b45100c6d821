// Which lane's e8m0 scale applies to which operand elements in
// v_mfma_scale_f32_16x16x128_f8f6f4, and what opsel does.  All fp8 operand bytes are 1.0 (0x38),
// one of the two scales varies per lane; the host checks D[row][col] against "lane L scales the
// 32 K-values it holds (row/col L&15, K-block L>>4)" with the scale byte chosen by opsel.
//   hipcc --offload-arch=gfx950 -O3 scripts/experiments/mx_scale_probe.hip -o tools_bin/mx_scale_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ int sc(int lane) { return 127 + (lane & 3) - ((lane >> 4) & 3) + ((lane >> 2) & 1); }

template <int WHICH, int OPSEL>
__global__ void probe(float* out) {
  const int lane = threadIdx.x;
  i32x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = 0x38383838; b[j] = 0x38383838; }
  const int s = sc(lane);
  const int packed = (0x7f7f7f7f & ~(0xff << (8 * OPSEL))) | (s << (8 * OPSEL));
  f32x4 c = {0, 0, 0, 0};
  if (WHICH == 0) c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OPSEL, packed, 0, 127);
  else c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, OPSEL, packed);
  // D layout: lane holds rows 4*(lane>>4) + r, column lane & 15
  for (int r = 0; r < 4; ++r) out[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = c[r];
}

static int host_sc(int lane) { return 127 + (lane & 3) - ((lane >> 4) & 3) + ((lane >> 2) & 1); }

template <int WHICH, int OPSEL>
static void run(float* d) {
  probe<WHICH, OPSEL><<<1, 64>>>(d);
  float h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      // WHICH 0 scales operand A (rows i of D), WHICH 1 operand B (columns j)
      const int rc = WHICH == 0 ? i : j;
      double e = 0;
      for (int kb = 0; kb < 4; ++kb) e += 32.0 * std::ldexp(1.0, host_sc(kb * 16 + rc) - 127);
      if (std::fabs(h[i * 16 + j] - e) > 1e-3 * e) ++bad;
    }
  printf("scale on operand %s, opsel %d: %s (%d of 256 mismatch; D[0][0]=%g D[5][9]=%g)\n",
         WHICH ? "B" : "A", OPSEL, bad ? "MISMATCH" : "lane L scales its own 32 K-values", bad, h[0], h[5 * 16 + 9]);
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 4);
  run<0, 0>(d); run<0, 2>(d); run<1, 0>(d); run<1, 1>(d); run<1, 3>(d);
  return 0;
}
