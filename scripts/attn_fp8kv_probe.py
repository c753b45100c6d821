"""Decode attention with a bf16 vs an fp8 (e4m3fn) KV cache: µs per call and effective KV read
bandwidth (bytes actually stored) at the Llama-3-70B head config, graph replay, rotating layers.
    python scripts/attn_fp8kv_probe.py [--sweep]  -> gpurun_out/attn_fp8kv_probe.json
--sweep also times 2x and 4x the decode_splits() choice (split heuristic check)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
nh, nkv, D, bs = 64, 8, 128, 64
res = []


def timed(B, L, fp8, esz, layers, ks, vs, bt, lens, q, splits, chosen):
    ws = ops.decode_workspace(B, nh, D, splits, dev) if splits > 1 else None
    out = torch.empty_like(q)

    def call(i):
        ops.attn_decode(q, None, ks[i % layers], vs[i % layers], bt, lens, D ** -0.5,
                        num_splits=splits, workspace=ws, out=out, k_scale=0.5, v_scale=0.5)
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
    kv = 2 * B * L * nkv * D * esz
    r = {"B": B, "L": L, "kv": "fp8" if fp8 else "bf16", "splits": splits, "us": round(us, 1),
         "TBps": round(kv / us / 1e6, 2)}
    if not chosen:
        r["sweep"] = True
    print(json.dumps(r), flush=True)
    res.append(r)


CASES = [(512, 600), (64, 4096), (16, 8192), (1, 8192)]
for a in sys.argv[1:]:
    if a.startswith("--cases="):   # e.g. --cases=256x600,512x600
        CASES = [tuple(int(v) for v in c.split("x")) for c in a.split("=", 1)[1].split(",")]
for B, L in CASES:
    for fp8 in (False, True):
        bps = (L + bs - 1) // bs
        nblk = B * bps
        esz = 1 if fp8 else 2
        per_layer = 2 * nblk * nkv * bs * D * esz
        layers = max(2, min(16, int(2.5e9 // per_layer) + 1))
        dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
        ks = [(torch.randn(nblk, nkv, bs, D, device=dev) * 0.5).to(dt) for _ in range(layers)]
        vs = [(torch.randn(nblk, nkv, bs // 8, D, 8, device=dev) * 0.5).to(dt) for _ in range(layers)]
        bt = torch.randperm(nblk, device=dev).to(torch.int32).view(B, bps)
        lens = torch.full((B,), L, dtype=torch.int32, device=dev)
        q = torch.randn(B, nh, D, device=dev, dtype=torch.bfloat16)
        s0 = ops.decode_splits(B, nkv, nh // nkv, L)
        cands = [s0]
        if "--sweep" in sys.argv:
            cands += [c for c in ([2, 4] if s0 == 1 else [2 * s0, 4 * s0]) if c <= min(512, L // 32)]
        for splits in cands:
            timed(B, L, fp8, esz, layers, ks, vs, bt, lens, q, splits, splits == s0)
        del ks, vs
        torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/attn_fp8kv_probe.json", "w"), indent=1)
