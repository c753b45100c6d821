"""Hand-written decode GEMM vs tuned hipBLASLt on the Llama-3-70B decode shapes (cold weights)."""
import json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops
dev = torch.device("cuda:0")
H, I = 8192, 28672
SHAPES = {"qkv": (H, 10240), "o": (H, H), "gate_up": (H, 2 * I), "down": (I, H)}
M = int(os.environ.get("M", "256"))
t = torch.cuda.tunable
t.enable(True)
t.read_file(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "distributed_llm_inference", "tuning", "tunableop_gfx950.csv"))
t.tuning_enable(False)

def bench(fn, n):
    for i in range(3): fn(i % n)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(30): fn(i % n)
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / 30 * 1e6

res = {}
for name, (K, N) in SHAPES.items():
    nrot = max(2, int(1.0e9 // (N * K * 2)) + 1)
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    r = {"hipblaslt_us": round(bench(lambda i: torch.nn.functional.linear(x, ws[i]), nrot), 1)}
    ref = torch.nn.functional.linear(x, ws[0]).float()
    for bn in (64, 128):
        for sp in (1, 2, 4, 8):
            if N % bn or (K // 64) % sp:
                continue
            wsp = torch.empty(sp * M * N, dtype=torch.float32, device=dev)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            us = bench(lambda i: ops.gemm_nt(x, ws[i], sp, bn, out, wsp), nrot)
            y = ops.gemm_nt(x, ws[0], sp, bn, out, wsp).float()
            err = ((y - ref).abs().max() / ref.abs().max()).item()
            r[f"dli_bn{bn}_s{sp}_us"] = round(us, 1)
            r[f"dli_bn{bn}_s{sp}_relerr"] = float(f"{err:.2e}")
    best = min((v, k) for k, v in r.items() if k.endswith("_us"))
    r["best"] = best[1]
    r["TF_best"] = round(2 * M * N * K / best[0] / 1e6, 1)
    res[name] = r
    print(name, json.dumps(r), flush=True)
    del ws
json.dump(res, open(f"gpurun_out/gemm_bench_M{M}.json", "w"), indent=1)
