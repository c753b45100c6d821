#!/usr/bin/env python3
"""Fixed cost of a small decode-attention launch on MI355X (run under rocprofv3 --kernel-trace).

Graph-replays, back to back: a one-lane kernel (the launch floor), B=1 decode attention over
one 32-key step (one split: the kernel's fixed path), and B=1 over 600 keys with 4 and 16 splits
(the LDS-merged split path, plus the combine kernel when splits > 4).  The per-kernel durations
separate the launch floor, the decode kernel's prologue / epilogue and the combine."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda", 0)
C = ops.native()
nh, nkv, D, bs = 64, 8, 128, 64
out1 = torch.zeros(1, dtype=torch.int32, device=dev)


def case(L, splits):
    nblk = (L + bs - 1) // bs
    k = torch.randn(nblk, nkv, bs, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(nblk, nkv, bs // 8, D, 8, device=dev, dtype=torch.bfloat16)
    bt = torch.arange(nblk, device=dev, dtype=torch.int32).view(1, nblk)
    lens = torch.full((1,), L, dtype=torch.int32, device=dev)
    q = torch.randn(1, nh, D, device=dev, dtype=torch.bfloat16)
    ws = ops.decode_workspace(1, nh, D, splits, dev) if splits > 1 else None
    out = torch.empty_like(q)
    return lambda: ops.attn_decode(q, None, k, v, bt, lens, D ** -0.5, num_splits=splits,
                                   workspace=ws, out=out)


calls = [("touch", lambda: C.touch(out1, torch.cuda.current_stream().cuda_stream)),
         ("L32_s1", case(32, 1)), ("L600_s4", case(600, 4)), ("L600_s16", case(600, 16))]
for name, f in calls:
    f()
torch.cuda.synchronize()
for name, f in calls:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(40):
            f()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    print(name, "done", flush=True)
