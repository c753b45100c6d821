"""GEMM probe for the 70B decode shapes: default hipBLASLt vs TunableOp-tuned, bf16 and fp8.

Weights are sized > Infinity Cache (rotating set of 4 copies) so the numbers are HBM-realistic.
"""
import json
import os
import sys
import time

import torch

dev = torch.device("cuda:0")
H, I, QKV = 8192, 28672, 10240
SHAPES = {"qkv": (H, QKV), "o": (H, H), "gate_up": (H, 2 * I), "down": (I, H), "lm_head": (H, 128256)}


def bench(fn, iters=30):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(iters):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def run(tag, Ms):
    res = {}
    for name, (K, N) in SHAPES.items():
        nrot = max(1, min(4, int(1.2e9 // (N * K * 2)) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
        for M in Ms:
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            t = bench(lambda i: torch.nn.functional.linear(a, ws[i % nrot]))
            res[f"{name}_M{M}"] = dict(us=round(t * 1e6, 1), TBps=round(N * K * 2 / t / 1e12, 2),
                                      TF=round(2 * M * N * K / t / 1e12, 1))
        del ws
    print(tag, json.dumps(res, indent=0), flush=True)
    return res


if __name__ == "__main__":
    out = {}
    Ms = [64, 128, 256]
    out["default"] = run("default", Ms)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(200)
    torch.cuda.tunable.set_filename("gpurun_out/tunableop_results.csv")
    out["tuned"] = run("tuned", Ms)
    torch.cuda.tunable.write_file()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/gemm_probe.json", "w"), indent=1)
