"""Greedy / top-p sampler timing on the LM-head shape (rows x 128256 bf16 logits), graph-replayed,
next to torch.argmax on the same logits; checks the greedy tokens against torch.argmax.

    python scripts/sample_probe.py   -> stdout + gpurun_out/sample_probe.json
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda", 0)
V = 128256
res = {}


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(5):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * 5) * 1e6


for rows in (1, 64, 512):
    logits = (torch.randn(rows, V, device=dev) * 3).to(torch.bfloat16)
    temp = torch.zeros(rows, device=dev)
    topk = torch.zeros(rows, dtype=torch.int32, device=dev)
    topp = torch.ones(rows, device=dev)
    seeds = torch.arange(rows, dtype=torch.int64, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.empty(rows, dtype=torch.int32, device=dev)
    f = lambda: ops.sample(logits, temperature=temp, top_k=topk, top_p=topp, seeds=seeds, step=step, out=out)
    us = timed(f)
    f()
    torch.cuda.synchronize()
    ok = torch.equal(out.long(), logits.float().argmax(-1))
    am = timed(lambda: logits.argmax(-1))
    temp2 = torch.full((rows,), 0.8, device=dev)
    topp2 = torch.full((rows,), 0.9, device=dev)
    topk2 = torch.full((rows,), 50, dtype=torch.int32, device=dev)
    r = {}
    toks = {}
    for path in ("1", "0"):   # DLI_SAMPLE_REGS: register path / radix-histogram path
        os.environ["DLI_SAMPLE_REGS"] = path
        r[f"top_p_us_regs{path}"] = round(timed(lambda: ops.sample(
            logits, temperature=temp2, top_k=topk, top_p=topp2, seeds=seeds, step=step, out=out)), 1)
        r[f"top_k_top_p_us_regs{path}"] = round(timed(lambda: ops.sample(
            logits, temperature=temp2, top_k=topk2, top_p=topp2, seeds=seeds, step=step, out=out)), 1)
        ops.sample(logits, temperature=temp2, top_k=topk2, top_p=topp2, seeds=seeds, step=step, out=out)
        torch.cuda.synchronize()
        toks[path] = out.clone()
    os.environ.pop("DLI_SAMPLE_REGS")
    r["same_tokens_frac"] = round((toks["1"] == toks["0"]).float().mean().item(), 4)
    gb = rows * V * 2 / 1e9
    res[rows] = {"greedy_us": round(us, 1), "greedy_TBps": round(gb / us * 1e3, 2), "argmax_equal": ok,
                 "torch_argmax_us": round(am, 1), **r}
    print(rows, res[rows], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/sample_probe.json", "w"), indent=1)

# the decode step's order: LM-head GEMM (hipBLASLt) writes the logits, the sampler reads them next
rows, H = 512, 8192
x = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
w = (torch.randn(V, H, device=dev) * 0.02).to(torch.bfloat16)
logits = torch.empty(rows, V, device=dev, dtype=torch.bfloat16)
temp = torch.zeros(rows, device=dev)
topk = torch.zeros(rows, dtype=torch.int32, device=dev)
topp = torch.ones(rows, device=dev)
seeds = torch.arange(rows, dtype=torch.int64, device=dev)
step = torch.zeros(1, dtype=torch.int64, device=dev)
out = torch.empty(rows, dtype=torch.int32, device=dev)
gemm = lambda: torch.matmul(x, w.t(), out=logits)
both = lambda: (gemm(), ops.sample(logits, temperature=temp, top_k=topk, top_p=topp, seeds=seeds,
                                   step=step, out=out))
t_g, t_b = timed(gemm), timed(both)
res["after_gemm_512"] = {"gemm_us": round(t_g, 1), "gemm_plus_greedy_us": round(t_b, 1),
                         "greedy_after_gemm_us": round(t_b - t_g, 1)}
print("after_gemm_512", res["after_gemm_512"], flush=True)
json.dump(res, open("gpurun_out/sample_probe.json", "w"), indent=1)
