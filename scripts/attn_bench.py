"""Decode-attention microbenchmark (Llama-3-70B head config) on one MI355X.

KV caches are sized far beyond the 256 MiB Infinity Cache and each call reads a different layer's
cache (rotating), so every call streams K/V from HBM as in the real decode step.  Calls are timed
from a captured hipGraph replay (as the engine runs them: no host launch cost in the number).
Prints µs per call and achieved KV bandwidth; writes gpurun_out/attn_bench.json.
``--sweep`` also times other split counts for the small-batch cases.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
nh, nkv, D, bs = 64, 8, 128, 64
CASES = [(512, 600), (256, 2048), (64, 4096), (16, 8192), (16, 32768), (4, 16384), (1, 8192),
         (1, 32768), (1, 600)]


def run(B, L, layers=None, splits=None):
    blocks_per_seq = (L + bs - 1) // bs
    nblk = B * blocks_per_seq
    per_layer = 2 * nblk * nkv * bs * D * 2
    layers = layers or max(2, min(24, int(2.5e9 // per_layer) + 1))
    ks = [torch.randn(nblk, nkv, bs, D, device=dev, dtype=torch.bfloat16) for _ in range(layers)]
    vs = [torch.randn(nblk, nkv, bs // 8, D, 8, device=dev, dtype=torch.bfloat16) for _ in range(layers)]
    bt = torch.randperm(nblk, device=dev).to(torch.int32).view(B, blocks_per_seq)
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    q = torch.randn(B, nh, D, device=dev, dtype=torch.bfloat16)
    splits = splits or ops.decode_splits(B, nkv, nh // nkv, L)
    ws = None
    if splits > 1:
        ws = ops.decode_workspace(B, nh, D, splits, dev)
    out = torch.empty_like(q)

    def call(i):
        ops.attn_decode(q, None, ks[i % layers], vs[i % layers], bt, lens, D ** -0.5,
                        num_splits=splits, workspace=ws, out=out)

    for i in range(layers):
        call(i)
    torch.cuda.synchronize()
    n = max(layers, 8)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            call(i)
    g.replay()
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / (n * reps) * 1e6
    kv_bytes = 2 * B * L * nkv * D * 2
    # numerics spot check against the fp32 reference on a few sequences
    ref = ops.reference.attn_decode(q[:2].cpu(), None, ks[0].cpu(), vs[0].cpu(), bt[:2].cpu(),
                                    lens[:2].cpu(), D ** -0.5)
    ops.attn_decode(q, None, ks[0], vs[0], bt, lens, D ** -0.5, num_splits=splits, workspace=ws,
                    out=out)
    err = (out[:2].float().cpu() - ref.float()).abs().max().item()
    del ks, vs
    torch.cuda.empty_cache()
    return dict(B=B, L=L, splits=splits, us=round(us, 1), TBps=round(kv_bytes / us / 1e6, 2),
                max_err=round(err, 4))


res = []
for a in sys.argv[1:]:
    if a.startswith("--cases="):   # e.g. --cases=1x8192,4x16384
        CASES = [tuple(int(v) for v in c.split("x")) for c in a.split("=", 1)[1].split(",")]
for B, L in CASES:
    r = run(B, L)
    print(r, flush=True)
    res.append(r)
if "--sweep" in sys.argv:
    for B, L in [(1, 8192), (1, 32768), (4, 16384), (16, 8192), (16, 32768), (64, 2048)]:
        for sp in (4, 8, 16, 32, 64, 128, 256):
            if sp * 32 <= L:
                r = run(B, L, splits=sp)
                r["sweep"] = True
                print(r, flush=True)
                res.append(r)
if "--short" in sys.argv:   # batch-1 short contexts: latency-bound, fewer splits skip the merge
    for B, L in [(1, 600), (1, 1100), (1, 2048), (2, 600)]:
        for sp in (1, 2, 4, 8, 16):
            if sp * 32 <= L:
                r = run(B, L, splits=sp)
                r["short"] = True
                print(r, flush=True)
                res.append(r)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/attn_bench.json", "w"), indent=1)
