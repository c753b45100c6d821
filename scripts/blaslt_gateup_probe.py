#!/usr/bin/env python3
"""Kernel identity of hipBLASLt on the decode gate|up shape (M=512, N=57344, K=8192) and on
8192^3, next to the tile kernel: run under `rocprofv3 --kernel-trace` so the trace names the
Tensile kernel (its name encodes macro tile, MFMA shape, wave layout) and records VGPR / AGPR /
LDS / workgroup size of every kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda", 0)
for (M, N, K) in [(512, 57344, 8192), (8192, 8192, 8192), (512, 8192, 8192), (512, 10240, 8192)]:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    for _ in range(5):
        y = x @ w.t()
    if N % 256 == 0:
        for _ in range(5):
            ops.gemm_tile(x, w, splits=1)
    torch.cuda.synchronize()
    print(f"M={M} N={N} K={K} done", flush=True)
