#!/usr/bin/env python3
"""Which hipBLASLt kernels does torch pick for the decode shapes that bypass the tile GEMM, and
are they stream-K (persistent, with cross-workgroup waits)?

Runs each Llama-3-70B projection shape (and the LM head) at small M with torch.matmul (bf16),
a few times each, so a kernel trace (rocprofv3 --kernel-trace --stats) names the library
kernels.  Stream-K Tensile kernels size their grid to the CU count and a workgroup may wait for
another's partial tile: two such kernels in flight on different streams (or processes) can
each hold CUs the other needs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = torch.device("cuda", 0)
H, I, V = 8192, 28672, 128256
SHAPES = [("qkv", 10240, H), ("o", H, H), ("gate_up", 2 * I, H), ("down", H, I), ("head", V, H)]
Ms = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "1,2,8,32,64,127,4096").split(",")]
ws = {n: torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for n, N, K in SHAPES}
for M in Ms:
    for n, N, K in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            y = x @ ws[n].t()
        torch.cuda.synchronize()
        print(f"M={M} {n} [{N}x{K}] done", flush=True)
