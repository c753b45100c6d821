"""Prefill-attention microbenchmark (Llama-3-70B heads: 64 q / 8 kv, D=128) on one MI355X.

Cases are (sequences, new tokens per sequence, tokens already cached).  Prints µs per call and the
achieved causal-attention TFLOP/s (4 * D FLOPs per visible (query, key) pair per head).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
nh, nkv, D, bs = int(os.environ.get("NH", 64)), int(os.environ.get("NKV", 8)), 128, 64
CASES = [(32, 512, 0), (4, 4096, 0), (1, 2048, 6144), (256, 16, 512)]
if os.environ.get("CASES"):   # e.g. CASES="4x4096x0,1x32768x0"
    CASES = [tuple(int(x) for x in c.split("x")) for c in os.environ["CASES"].split(",")]
QB = int(os.environ["QB"]) if os.environ.get("QB") else None   # None: ops.prefill_qb_for
WINDOW = int(os.environ.get("WINDOW", "0"))   # > 0: a sliding-window ring (Mistral), no sinks
KV_FP8 = os.environ.get("KV_FP8", "0") == "1"   # fp8 e4m3 caches (scale 1)
N_SINK = int(os.environ.get("N_SINK", "0"))      # StreamingLLM sink tokens (with WINDOW)


def run(B, q, ctx):
    L = q + ctx
    sink_pad = ((N_SINK + 31) // 32) * 32 if WINDOW else 0
    ring = ((WINDOW - N_SINK + q - 1 + 31) // 32) * 32 if WINDOW else 0
    nbps = ((sink_pad + ring if WINDOW else L) + bs - 1) // bs
    nblk = B * nbps
    kc = torch.randn(nblk, nkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nblk, nkv, bs // 8, D, 8, device=dev, dtype=torch.bfloat16)
    if KV_FP8:
        kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    bt = torch.arange(nblk, device=dev, dtype=torch.int32).view(B, nbps)
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    q_start = torch.arange(0, (B + 1) * q, q, dtype=torch.int32, device=dev)
    Q = torch.randn(B * q, nh, D, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(Q)
    QS = torch.randn_like(Q) if (WINDOW and N_SINK) else None

    tm = ops.prefill_tiles([q] * B, nh, nkv, qb=QB).to(dev) if os.environ.get("DENSE") != "1" else None

    def call():
        ops.attn_prefill(Q, QS, kc, vc, bt, lens, q_start, q, D ** -0.5,
                         N_SINK if WINDOW else 0, sink_pad, ring, WINDOW, tile_map=tm, qb=QB)

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        call()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    pairs = B * sum(min(ctx + i + 1, WINDOW) if WINDOW else ctx + i + 1 for i in range(q))
    tf = 4 * D * nh * pairs / us / 1e6
    return dict(nh=nh, nkv=nkv, window=WINDOW, n_sink=N_SINK, kv_fp8=int(KV_FP8), B=B, q=q, ctx=ctx, qb=QB or ops.prefill_qb_for(q), m32=int(ops.policy().prefill_m32), us=round(us, 1),
                TFLOPs=round(tf, 1))


res = []
for c in CASES:
    r = run(*c)
    print(r, flush=True)
    res.append(r)
os.makedirs("gpurun_out", exist_ok=True)
tag = os.environ.get("TAG", "qb%s_m32%d" % (QB or "auto", int(ops.policy().prefill_m32)))
json.dump(res, open("gpurun_out/attn_prefill_bench_%s.json" % tag, "w"), indent=1)
