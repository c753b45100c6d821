"""Microbenchmark of the decode step's RoPE + paged-KV write (rope_cache.hip) at the 70B / 512-row
shape: 3 bf16 split-K partials of the QKV GEMM [3, 512, 10240] summed on load, q rotated and
stored [512, 64, 128], k rotated and v written into the paged caches (one slot per sequence, a
distinct block each).  Partials rotate over 8 sets (past the MALL); calls are replayed from a
hipGraph.

    python scripts/rope_bench.py [--rows 512] [--kv-fp8] [--iters 20]
Prints one JSON line (us per call, TB/s of its HBM bytes)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--splits", type=int, default=3)
    ap.add_argument("--kv-fp8", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--no-kv", action="store_true", help="slot -1: no cache writes (diagnostic)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    T, S, NSET = a.rows, a.splits, a.sets
    nh, nkv, D, bs = 64, 8, 128, 64
    N = (nh + 2 * nkv) * D
    g = torch.Generator(device=dev).manual_seed(0)
    parts = [torch.randn(S, T, N, device=dev, generator=g).to(torch.bfloat16) for _ in range(NSET)]
    kdt = torch.float8_e4m3fn if a.kv_fp8 else torch.bfloat16
    nblk = 2 * T + 8
    kc = torch.zeros(nblk, nkv, bs, D, device=dev).to(kdt)
    vc = torch.zeros(nblk, nkv, bs // 8, D, 8, device=dev).to(kdt)
    pos = torch.full((T,), 600, device=dev, dtype=torch.int32)
    slots = torch.arange(T, device=dev, dtype=torch.int64) * (2 * bs) + 37
    if a.no_kv:
        slots.fill_(-1)
    cs = ops.reference.build_cos_sin(D, 4096, 500000.0, None, device=dev)
    qo = [torch.empty(T, nh, D, dtype=torch.bfloat16, device=dev) for _ in range(NSET)]

    def run():
        for i in range(NSET):
            ops.rope_cache(ops.SplitKPartials(parts[i]), pos, slots, cs, nh, nkv, D, kc, vc,
                           q_out=qo[i], k_scale=0.5, v_scale=0.5)

    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(gr):
        run()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters / NSET
    kvb = 1 if a.kv_fp8 else 2
    nbytes = S * T * N * 2 + T * nh * D * 2 + 2 * T * nkv * D * kvb
    print(json.dumps({"kernel": "rope_cache", "rows": T, "splits": S, "kv_fp8": a.kv_fp8, "no_kv": a.no_kv,
                      "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
