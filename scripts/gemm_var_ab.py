"""In-process interleaved A/B of the bf16 tile GEMM variants (DLI_GEMM_VAR, gemm_tile.hip) on the
70B decode shapes at M = 512: each round times every variant once (graph replay, weights rotated
past the Infinity Cache); reports median and min per variant.

    python scripts/gemm_var_ab.py [--vars 0,1,2] [--rounds 7]   -> gpurun_out/gemm_var_ab.json
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--vars", default="0,1,2")
ap.add_argument("--rounds", type=int, default=7)
a = ap.parse_args()
VARS = [int(v) for v in a.vars.split(",")]
dev = torch.device("cuda:0")
torch.manual_seed(0)
SHAPES = {"gate_up_swiglu": (512, 57344, 8192, 1, True), "down_s4": (512, 8192, 28672, 4, False),
          "qkv_s3": (512, 10240, 8192, 3, False), "o_s4": (512, 8192, 8192, 4, False)}


def make(M, N, K, splits, swiglu):
    sets = max(1, min(6, int(1.2e9 // (N * K * 2)) + 1))
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ws = [(torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16) for _ in range(sets)]
    if swiglu:
        ws = [ops.swiglu_interleave(w) for w in ws]
    out = torch.empty(M, N // 2 if swiglu else N, device=dev, dtype=torch.bfloat16)
    wsp = torch.empty(splits * M * N, device=dev) if splits > 1 else None
    graphs = {}
    for v in VARS:
        os.environ["DLI_GEMM_VAR"] = str(v)
        def f(i):
            ops.gemm_tile(x, ws[i % sets], splits=splits, swiglu=swiglu, out=out, workspace=wsp)
        f(0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(max(sets, 4)):
                f(i)
        graphs[v] = (g, max(sets, 4))
    ref = None
    for v in VARS:   # every variant computes the same product
        os.environ["DLI_GEMM_VAR"] = str(v)
        f(0)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), f"variant {v} differs"
    return graphs, (ws, x, out, wsp)


res = {}
for name, shp in SHAPES.items():
    graphs, keep = make(*shp)
    times = {v: [] for v in VARS}
    for r in range(a.rounds):
        for v in (VARS if r % 2 == 0 else VARS[::-1]):   # alternate the order: no position bias
            g, n = graphs[v]
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / (5 * n) * 1e6)
    res[name] = {str(v): {"median_us": round(statistics.median(t), 1), "min_us": round(min(t), 1)}
                 for v, t in times.items()}
    print(name, res[name], flush=True)
    del graphs, keep
    torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/gemm_var_ab.json", "w"), indent=1)
