"""Microbenchmark of the decode step's row kernels at the 70B / 512-row shape: add + RMSNorm over
4 bf16 split-K partials (norm.hip, bf16 path) and add + RMSNorm + fp8 quantisation (quant.hip,
fp8 path), each reading 4 x 8 MB of partials + an 8 MB residual and writing the residual and its
output.  Buffers rotate over 8 sets (~0.4 GB, past the MALL), calls are replayed from a hipGraph;
a device copy of the same bytes is the bandwidth reference.

    python scripts/norm_bench.py [--rows 512] [--hidden 8192] [--splits 4] [--iters 20]
Prints one JSON line per kernel (us per call, TB/s of its HBM bytes)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llm_inference import ops


def timed(fn, iters):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--splits", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sets", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, H, S, NSET = a.rows, a.hidden, a.splits, a.sets
    g = torch.Generator(device=dev).manual_seed(0)
    parts = [torch.randn(S, M, H, device=dev, generator=g).to(torch.bfloat16) for _ in range(NSET)]
    res = [torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16) for _ in range(NSET)]
    w = (1 + 0.1 * torch.randn(H, device=dev, generator=g)).to(torch.bfloat16)
    outs = [torch.empty(M, H, dtype=torch.bfloat16, device=dev) for _ in range(NSET)]
    rout = [torch.empty(M, H, dtype=torch.bfloat16, device=dev) for _ in range(NSET)]

    def norm():
        for i in range(NSET):
            ops.rms_norm(ops.SplitKPartials(parts[i]), w, 1e-5, res[i], out=outs[i],
                         residual_out=rout[i])

    def quant():
        for i in range(NSET):
            ops.quant_rowwise(ops.SplitKPartials(parts[i]), res[i], w, 1e-5, residual_out=rout[i])

    src = [torch.empty((S + 1) * M * H, dtype=torch.bfloat16, device=dev) for _ in range(NSET)]
    dst = [torch.empty(M * H, dtype=torch.bfloat16, device=dev) for _ in range(NSET)]

    def copy():   # read (S + 1) x 8 MB, write 8 MB: a sum over the partials
        for i in range(NSET):
            torch.sum(src[i].view(S + 1, 2, M * H // 2), 0, out=dst[i].view(2, M * H // 2))

    rd = (S + 1) * M * H * 2
    for name, fn, wr in (("rms_norm_splitk", norm, 2 * M * H * 2),
                         ("quant_rowwise_splitk", quant, M * H * 2 + M * H),
                         ("torch_sum_reference", copy, M * H * 2)):
        us = timed(fn, a.iters) / NSET
        print(json.dumps({"kernel": name, "rows": M, "hidden": H, "splits": S,
                          "us": round(us, 2), "TBps": round((rd + wr) / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
