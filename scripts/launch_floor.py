#!/usr/bin/env python3
"""Per-kernel cost of back-to-back small kernels inside one hipGraph, wall-clocked (no profiler):
the floor every extra launch of the batch-1 decode step pays.  Prints us per kernel for a one-lane
kernel, an M=1 RMSNorm over 8192 columns, and M=1 RoPE + KV write, each replayed N times in a
graph."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda", 0)
C = ops.native()
N = 200
res = {}
x = torch.randn(1, 8192, device=dev, dtype=torch.bfloat16)
r = torch.randn(1, 8192, device=dev, dtype=torch.bfloat16)
w = torch.ones(8192, device=dev, dtype=torch.bfloat16)
o1 = torch.zeros(1, dtype=torch.int32, device=dev)
x2 = torch.randn(1, 2 * 28672, device=dev, dtype=torch.bfloat16)
cases = {
    "touch": lambda: C.touch(o1, torch.cuda.current_stream().cuda_stream),
    "rms_norm_M1": lambda: ops.rms_norm(x, w, 1e-5, residual=r),
    "silu_mul_M1": lambda: ops.swiglu_interleaved(x2),
}
for name, f in cases.items():
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(N):
            f()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 20
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / (reps * N) * 1e6
    res[name] = round(us, 2)
    print(f"{name:14s} {us:6.2f} us per kernel in a {N}-kernel graph", flush=True)
print(json.dumps(res))
