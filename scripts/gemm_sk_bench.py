"""Stream-K tail vs a plain second wave for the tile GEMM (csrc/kernels/gemm_tile.hip) on the
Llama-3-70B gate|up shape (fused SwiGLU epilogue) and a plain-store shape with a partial last wave.
Cold weights (rotating set > Infinity Cache).

    python scripts/gemm_sk_bench.py [--out gpurun_out/gemm_sk_bench.json]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_llm_inference import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/gemm_sk_bench.json")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(0)


def timed(fn, nrot, iters=30):
    for i in range(3):
        fn(i % nrot)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(iters):
        fn(i % nrot)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


res = {}
# (name, M, N, K, swiglu)
for name, M, N, K, swiglu in [("gate_up_swiglu", 512, 57344, 8192, True),
                              ("gate_up_store", 512, 57344, 8192, False),
                              ("m384_gate_up_swiglu", 384, 57344, 8192, True)]:
    nrot = max(2, int(1.0e9 // (N * K * 2)) + 1)
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N // 2 if swiglu else N, device=dev, dtype=torch.bfloat16)
    wsp = torch.empty(ops.native().gemm_tile_sk_workspace_floats(), device=dev, dtype=torch.float32)
    r = {"tiles": ((M + 255) // 256) * (N // 256), "stream_k_eligible": ops.tile_gemm_stream_k(M, N, dev)}
    os.environ["DLI_TILE_SK"] = "0"
    r["wave_us"] = round(timed(lambda i: ops.gemm_tile(x, ws[i], swiglu=swiglu, out=out), nrot), 1)
    os.environ["DLI_TILE_SK"] = "1"
    r["stream_k_us"] = round(timed(lambda i: ops.native().gemm_tile(
        out, x, ws[i], 0, 2 if swiglu else 0, wsp), nrot), 1)
    flop = 2 * M * N * K
    r["TF_wave"] = round(flop / r["wave_us"] / 1e6, 1)
    r["TF_stream_k"] = round(flop / r["stream_k_us"] / 1e6, 1)
    r["hipblaslt_us"] = round(timed(lambda i: torch.nn.functional.linear(x, ws[i]), nrot), 1)
    res[name] = r
    print(name, json.dumps(r), flush=True)
    del ws
os.makedirs(os.path.dirname(a.out), exist_ok=True)
json.dump(res, open(a.out, "w"), indent=1)
