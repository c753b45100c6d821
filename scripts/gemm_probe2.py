"""Decode GEMM variants at M=256 (70B shapes), weights rotated beyond the Infinity Cache:
  A) F.linear(x, W)                      (current)
  B) (W @ x.T).T  operand-swapped        (hipBLASLt sees M=N_w, N=256)
  C) fp8 rowwise _scaled_mm              (config 5)
TunableOp on for all (reads the shipped results)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dev = torch.device("cuda:0")
H, I = 8192, 28672
SHAPES = {"qkv": (H, 10240), "o": (H, H), "gate_up": (H, 2 * I), "down": (I, H)}
M = int(os.environ.get("M", "256"))


def bench(fn, n):
    for i in range(3):
        fn(i % n)
    torch.cuda.synchronize()
    t = time.perf_counter()
    it = 40
    for i in range(it):
        fn(i % n)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


t = torch.cuda.tunable
t.enable(True)
t.read_file(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "distributed_llm_inference", "tuning", "tunableop_gfx950.csv"))
t.set_filename("gpurun_out/tunableop_probe2.csv")
t.tuning_enable(True)
t.set_max_tuning_duration(60)
t.set_rotating_buffer_size(512)
res = {}
for name, (K, N) in SHAPES.items():
    nrot = max(2, int(1.0e9 // (N * K * 2)) + 1)
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    a = bench(lambda i: torch.nn.functional.linear(x, ws[i]), nrot)
    b = bench(lambda i: torch.matmul(ws[i], x.t()).t(), nrot)
    w8 = [w.to(torch.float8_e4m3fn) for w in ws]
    del ws
    x8 = x.to(torch.float8_e4m3fn)
    sa = torch.ones(M, 1, device=dev)
    sb = torch.ones(1, N, device=dev)
    c = bench(lambda i: torch._scaled_mm(x8, w8[i].t(), scale_a=sa, scale_b=sb,
                                         out_dtype=torch.bfloat16), nrot)
    del w8
    res[name] = dict(linear_us=round(a, 1), swapped_us=round(b, 1), fp8_us=round(c, 1),
                     bf16_bytes_MB=N * K * 2 / 1e6)
    print(name, res[name], flush=True)
json.dump(res, open(f"gpurun_out/gemm_probe2_M{M}.json", "w"), indent=1)
