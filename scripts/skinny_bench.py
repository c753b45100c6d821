"""Skinny GEMM (M <= 4, csrc/kernels/gemv.hip) vs hipBLASLt F.linear on the Llama-3-70B decode
shapes, weights rotated beyond the 256 MiB Infinity Cache (streamed from HBM as in decode)."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
H, I, V = 8192, 28672, 128256
SHAPES = {"qkv": (H, 10240), "o": (H, H), "gate_up": (H, 2 * I), "down": (I, H), "lm_head": (H, V)}


def bench(fn, n):
    for i in range(3):
        fn(i % n)
    torch.cuda.synchronize()
    it = 30
    t = time.perf_counter()
    for i in range(it):
        fn(i % n)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


res = {}
for name, (K, N) in SHAPES.items():
    nrot = max(2, int(1.2e9 // (N * K * 2)) + 1)
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
    for M in (1, 2, 4):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        a = bench(lambda i: F.linear(x, ws[i]), nrot)
        b = bench(lambda i: ops.skinny_gemm(x, ws[i]), nrot)
        gb = N * K * 2 / 1e9
        res[f"{name}_M{M}"] = dict(hipblaslt_us=round(a, 1), skinny_us=round(b, 1),
                                   hipblaslt_TBps=round(gb / a * 1e3, 2),
                                   skinny_TBps=round(gb / b * 1e3, 2))
        print(name, M, res[f"{name}_M{M}"], flush=True)
    del ws
    torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/skinny_bench.json", "w"), indent=1)
