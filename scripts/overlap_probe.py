"""Feasibility probe: can memory-bound decode attention overlap the power-bound projection GEMMs?

Stream A replays a graph of gate|up tile GEMMs (Llama-3-70B, M = 512, fused SwiGLU, weights rotated
past the Infinity Cache); stream B replays a graph of decode-attention launches (B sequences,
context L, 64 q / 8 kv heads, D = 128).  Reports each alone, both on two plain streams, and both on
CU-masked streams (hipExtStreamCreateWithCUMask: GEMM on the first 256 - C CUs, attention on the
last C), as wall time for the pair vs the sum of the solo times.

    python scripts/overlap_probe.py   -> gpurun_out/overlap_probe.json
"""
import ctypes
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
BF = torch.bfloat16
out_path = os.path.join("gpurun_out", "overlap_probe.json")
os.makedirs("gpurun_out", exist_ok=True)

# ---- GEMM side: gate|up + SwiGLU at M = 512
M, I, K = 512, 28672, 8192
sets = 2
x = torch.randn(M, K, device=dev, dtype=BF)
ws = [ops.swiglu_interleave((torch.randn(2 * I, K, device=dev) / K ** 0.5).to(BF)) for _ in range(sets)]
h = torch.empty(M, I, device=dev, dtype=BF)

# ---- attention side: B sequences of context L
B, L, nh, nkv, D, bs = 512, 600, 64, 8, 128, 64
mb = (L + bs - 1) // bs
nblocks = B * mb
kc = torch.randn(nblocks, nkv, bs, D, device=dev, dtype=BF)
vc = torch.randn(nblocks, nkv, bs // 8, D, 8, device=dev, dtype=BF)
bt = torch.randperm(nblocks, device=dev).reshape(B, mb).to(torch.int32)
lens = torch.full((B,), L, dtype=torch.int32, device=dev)
q = torch.randn(B, nh, D, device=dev, dtype=BF)
ao = torch.empty_like(q)
scale = 1 / math.sqrt(D)

N_GEMM, N_ATT = 6, 24


def gemm_work():
    for i in range(N_GEMM):
        ops.gemm_tile(x, ws[i % sets], swiglu=True, out=h)


def attn_work():
    for _ in range(N_ATT):
        ops.attn_decode(q, None, kc, vc, bt, lens, scale, out=ao)


hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(lo, hi):
    """A HIP stream restricted to CUs [lo, hi) (hipExtStreamCreateWithCUMask)."""
    words = [0] * 8
    for c in range(lo, hi):
        words[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * 8)(*words)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(8), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return torch.cuda.ExternalStream(s.value, device=dev)


def capture(fn, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            fn()
    torch.cuda.synchronize()
    return g


def timed(pairs, reps=5):
    """pairs: [(graph, stream)] replayed concurrently; median wall ms over reps."""
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for g, s in pairs:
            with torch.cuda.stream(s):
                g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


res = {"gemm": f"gate|up+SwiGLU M={M} x{N_GEMM}", "attn": f"decode B={B} L={L} x{N_ATT}"}
with torch.inference_mode():
    sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    ga, gb = capture(gemm_work, sa), capture(attn_work, sb)
    for _ in range(2):
        timed([(ga, sa)], 2), timed([(gb, sb)], 2)
    t_g = timed([(ga, sa)])
    t_a = timed([(gb, sb)])
    t_both = timed([(ga, sa), (gb, sb)])
    res.update(gemm_ms=t_g, attn_ms=t_a, sum_ms=t_g + t_a, both_plain_ms=t_both)
    print(json.dumps(res), flush=True)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for c_att in (16, 32, 64):
        try:
            s1, s2 = masked_stream(0, cus - c_att), masked_stream(cus - c_att, cus)
        except Exception as e:  # noqa: BLE001
            res["cu_mask_error"] = str(e)
            break
        g1, g2 = capture(gemm_work, s1), capture(attn_work, s2)
        timed([(g1, s1)], 2)
        tg = timed([(g1, s1)])
        ta = timed([(g2, s2)])
        tb = timed([(g1, s1), (g2, s2)])
        res[f"mask_att{c_att}"] = {"gemm_ms": tg, "attn_ms": ta, "both_ms": tb}
        print(json.dumps({f"mask_att{c_att}": res[f"mask_att{c_att}"]}), flush=True)
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res))
