"""Prefill-chunk gate|up (M = 16384 / 4096, 70B): tile GEMM with fused SwiGLU vs TunableOp-tuned
hipBLASLt + silu_mul (what prefill runs today)."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_llm_inference import ops  # noqa: E402

t = torch.cuda.tunable
t.enable(True)
t.read_file(os.path.join(REPO, "distributed_llm_inference", "tuning", "tunableop_gfx950.csv"))
t.tuning_enable(False)
dev = torch.device("cuda:0")
H, I = 8192, 28672
ws = [(torch.randn(2 * I, H, device=dev) * 0.02).to(torch.bfloat16) for _ in range(2)]


def timed(fn, iters=10):
    for i in range(2):
        fn(i)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


res = {}
for M in (4096, 16384):
    x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    o = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    r = {"hipblaslt+silu_mul_us": round(timed(lambda i: ops.silu_mul(torch.nn.functional.linear(x, ws[i % 2]))), 1),
         "hipblaslt_only_us": round(timed(lambda i: torch.nn.functional.linear(x, ws[i % 2])), 1),
         "tile_swiglu_us": round(timed(lambda i: ops.gemm_tile(x, ws[i % 2], swiglu=True, out=o)), 1)}
    r["TF_tile"] = round(2 * M * 2 * I * H / r["tile_swiglu_us"] / 1e6, 1)
    r["TF_hipblaslt"] = round(2 * M * 2 * I * H / r["hipblaslt_only_us"] / 1e6, 1)
    res[f"M{M}"] = r
    print(M, json.dumps(r), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/prefill_gateup_probe.json", "w"), indent=1)
