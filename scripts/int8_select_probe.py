"""Times the LLM.int8 outlier kernels (colmax, select, gathers) per call on the 70B shapes with
no / few / many outlier columns (hipGraph replay of 20 calls), to see where the select's time goes."""
import json
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
C = ops.native()
res = {}
for K, N in ((8192, 10240), (28672, 8192)):
    for n_out in (0, 20, 500):
        torch.manual_seed(0)
        x = (torch.randn(512, K, device=dev) * 0.5).to(torch.bfloat16)
        if n_out:
            cols = torch.randperm(K, device=dev)[:n_out]
            x[:, cols] *= 40.0
        wq = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        ws = torch.rand(N, device=dev) * 0.01
        colmax = torch.empty(K, device=dev)
        for _ in range(3):
            out = C.llm_int8_outliers(x, wq, ws, 6.0, 64, None, True)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                out = C.llm_int8_outliers(x, wq, ws, 6.0, 64, None, True)
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 100 * 1e3
        res[f"K{K}_out{n_out}"] = {"us_per_call_all_four": round(us, 2), "cnt": int(out[3].item())}
        print(K, n_out, res[f"K{K}_out{n_out}"], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/int8_select_probe.json", "w"), indent=1)
