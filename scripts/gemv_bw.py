#!/usr/bin/env python3
"""Batch-1 weight stream of Llama-3-70B on the GEMV kernels (csrc/kernels/gemv.hip), without the
rest of the decode step: 80 layers of (fused QKV, O, gate|up + SwiGLU, down) weights resident in
HBM (bf16, fp8 or int8), one M = 1 GEMV per projection per layer, each projection's 80 launches
captured in one hipGraph and replayed.  Prints us per launch and achieved TB/s per shape, then the
whole 320-launch stream (the floor of a batch-1 decode step for that weight format).

    python3 scripts/gemv_bw.py [bf16|fp8|int8 ...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda", 0)
H, I, L = 8192, 28672, 80
SHAPES = {"qkv": (10240, H, False), "o": (H, H, False), "gate_up": (2 * I, H, True),
          "down": (H, I, False)}


def weights(fmt, N, K):
    if fmt == "bf16":
        return [torch.empty(N, K, device=dev, dtype=torch.bfloat16).normal_(0, 0.02)
                for _ in range(L)]
    w = [torch.randint(-100, 100, (N, K), device=dev, dtype=torch.int8) for _ in range(L)]
    if fmt == "fp8":
        w = [t.view(torch.uint8).bitwise_and_(0x77).view(torch.float8_e4m3fn) for t in w]
    return w


def call(fmt, x, w, s, swiglu):
    if fmt == "bf16":
        return ops.skinny_gemm(x, w, swiglu=swiglu)
    if fmt == "fp8":
        return ops.skinny_gemm_fp8(x, w, s, swiglu=swiglu)
    return ops.skinny_gemm_int8(x, w, s, swiglu=swiglu)


def timed_graph(fns, reps=10):
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
    return (time.perf_counter() - t0) / reps * 1e6


res = {}
for fmt in (sys.argv[1:] or ["bf16", "fp8", "int8"]):
    esz = 2 if fmt == "bf16" else 1
    all_fns, total_bytes, out = [], 0, {}
    for name, (N, K, sw) in SHAPES.items():
        ws = weights(fmt, N, K)
        sc = torch.rand(N, device=dev) * 1e-2 + 1e-3
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        fns = [(lambda w=w, x=x, sc=sc, sw=sw: call(fmt, x, w, sc, sw)) for w in ws]
        us = timed_graph(fns) / L
        b = N * K * esz
        out[name] = {"us": round(us, 2), "TBps": round(b / us / 1e6, 2)}
        print(f"{fmt:5s} {name:8s} N={N:6d} K={K:6d} {us:8.2f} us/launch {b / us / 1e6:6.2f} TB/s",
              flush=True)
        all_fns.append(fns)
        total_bytes += b * L
    # the whole stream in layer order
    seq = [f for layer in zip(*all_fns) for f in layer]
    us = timed_graph(seq, reps=5)
    out["stream"] = {"ms": round(us / 1e3, 3), "TBps": round(total_bytes / us / 1e6, 2),
                     "GB": round(total_bytes / 1e9, 1)}
    print(f"{fmt:5s} whole stream {us / 1e3:.3f} ms ({total_bytes / 1e9:.1f} GB, "
          f"{total_bytes / us / 1e6:.2f} TB/s)", flush=True)
    res[fmt] = out
    del all_fns, seq
    torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/gemv_bw.json", "w"), indent=1)
