#!/usr/bin/env python3
"""Infinity-Cache (L3) warm-up of batch-1 GEMV weights (ops.l3_prefetch / the attention
launch's warm-up workgroups): Llama-3-70B O-projection weights (8192 x 8192, fp8 or bf16), 80
distinct copies so every replay starts cold, one M = 1 GEMV per copy, captured in hipGraphs:

  cold      80 x gemv(w_i)
  pf        80 x l3_prefetch(w_i, nwg)
  pf+gemv   80 x [l3_prefetch(w_i, nwg), gemv(w_i)]   -> warm gemv = (pf+gemv) - pf

    python3 scripts/l3_prefetch_probe.py [fp8|bf16]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda", 0)
fmt = sys.argv[1] if len(sys.argv) > 1 else "fp8"
N = K = 8192
L = 80
if fmt == "bf16":
    ws = [torch.empty(N, K, device=dev, dtype=torch.bfloat16).normal_(0, 0.02) for _ in range(L)]
else:
    ws = [torch.randint(-100, 100, (N, K), device=dev, dtype=torch.int8).view(torch.uint8)
          .bitwise_and_(0x77).view(torch.float8_e4m3fn) for _ in range(L)]
sc = torch.rand(N, device=dev) * 1e-2 + 1e-3
x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
nbytes = ws[0].numel() * ws[0].element_size()


def gemv(w):
    if fmt == "bf16":
        return ops.skinny_gemm(x, w)
    return ops.skinny_gemm_fp8(x, w, sc)


def timed(fns, reps=10):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for f in fns:
            f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for f in fns:
            f()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6 / L


ref = gemv(ws[0]).clone()
ops.l3_prefetch(ws[0], 224)
torch.cuda.synchronize()
assert torch.equal(gemv(ws[0]), ref), "prefetch changed the GEMV's result"
cold = timed([lambda w=w: gemv(w) for w in ws])
print(f"{fmt} O GEMV {nbytes / 1e6:.0f} MB: cold {cold:.2f} us ({nbytes / cold / 1e6:.2f} TB/s)",
      flush=True)
for nwg in (128, 224, 256, 512):
    pf = timed([lambda w=w: ops.l3_prefetch(w, nwg) for w in ws])
    both = timed([f for w in ws for f in (lambda w=w: ops.l3_prefetch(w, nwg),
                                          lambda w=w: gemv(w))])
    warm = both - pf
    print(f"  nwg {nwg:4d}: prefetch {pf:6.2f} us ({nbytes / pf / 1e6:.2f} TB/s), "
          f"prefetch+gemv {both:6.2f} us -> warm gemv {warm:6.2f} us "
          f"({nbytes / warm / 1e6:.2f} TB/s), saved {cold - warm:5.2f} us", flush=True)
