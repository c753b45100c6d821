"""256x256 LDS-DMA MFMA tile GEMM (csrc/kernels/gemm_tile.hip): correctness vs fp32 and timing vs
tuned hipBLASLt on the Llama-3-70B decode shapes (cold weights: rotating set > Infinity Cache).

    python scripts/gemm_tile_bench.py [--m 512] [--check-only]
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
ap.add_argument("--m", type=int, nargs="+", default=[512, 256])
ap.add_argument("--check-only", action="store_true")
ap.add_argument("--out", default="gpurun_out/gemm_tile_bench.json")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(0)

# ---------------------------------------------------------------- correctness
def check(M, N, K, splits, swiglu=False):
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    if swiglu:
        y = ops.gemm_tile(x, ops.swiglu_interleave(w), swiglu=True).float()
        h = (x.float() @ w.float().t()).to(torch.bfloat16).float()
        ref = torch.nn.functional.silu(h[:, :N // 2]) * h[:, N // 2:]
    else:
        y = ops.gemm_tile(x, w, splits=splits).float()
        ref = x.float() @ w.float().t()
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    ok = err < 2e-2
    print(f"check M={M} N={N} K={K} splits={splits} swiglu={swiglu}: rel err {err:.2e} "
          f"{'ok' if ok else 'FAIL'}", flush=True)
    return ok

ok = True
x = torch.eye(256, 128, device=dev, dtype=torch.bfloat16)
w = (torch.arange(256 * 128, device=dev, dtype=torch.float32).reshape(256, 128) % 251).to(torch.bfloat16)
ok &= bool(torch.equal(ops.gemm_tile(x, w).float(), x.float() @ w.float().t()))
print("identity/asymmetric:", ok, flush=True)
for (M, N, K, sp) in [(256, 256, 64, 1), (256, 256, 128, 1), (512, 512, 1024, 1), (100, 768, 512, 1),
                      (512, 1024, 4096, 4), (300, 512, 8192, 3), (1, 256, 256, 1), (512, 256, 192, 2)]:
    ok &= check(M, N, K, sp)
ok &= check(512, 1024, 1024, 1, swiglu=True)
ok &= check(77, 512, 256, 1, swiglu=True)
# fp8 (block-scaled K=128 MFMA) vs the dequantised fp32 product
def check_fp8(M, N, K, splits, swiglu=False):
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    xq, xs = ops.quant_rowwise(x.to(torch.bfloat16))
    wq, ws = ops.quantize_weight_fp8(w.to(torch.bfloat16))
    ref = (xq.float() * xs.reshape(-1, 1)) @ (wq.float() * ws.reshape(-1, 1)).t()
    if swiglu:
        y = ops.gemm_tile_fp8(xq, xs, ops.swiglu_interleave(wq.view(torch.uint8)).view(wq.dtype),
                              ops.swiglu_interleave(ws.reshape(-1, 1)).reshape(-1), swiglu=True).float()
        ref = ops.silu_mul(ref.to(torch.bfloat16)).float()
    else:
        y = ops.gemm_tile_fp8(xq, xs, wq, ws, splits).float()
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    good = err < 2e-2
    print(f"check fp8 M={M} N={N} K={K} splits={splits} swiglu={swiglu}: rel err {err:.2e} "
          f"{'ok' if good else 'FAIL'}", flush=True)
    return good


xi = torch.zeros(256, 128, device=dev)
xi[torch.arange(128), torch.arange(128)] = 1.0
wi = (torch.arange(256 * 128, device=dev, dtype=torch.float32).reshape(256, 128) % 13) - 6
yi = ops.gemm_tile_fp8(xi.to(torch.float8_e4m3fn), torch.ones(256, device=dev),
                       wi.to(torch.float8_e4m3fn), torch.ones(256, device=dev)).float()
ok &= bool(torch.equal(yi, xi @ wi.t()))
print("fp8 identity/asymmetric:", bool(torch.equal(yi, xi @ wi.t())), flush=True)
for (M, N, K, sp) in [(256, 256, 128, 1), (512, 512, 2048, 1), (100, 768, 1024, 3), (512, 1024, 8192, 4)]:
    ok &= check_fp8(M, N, K, sp)
ok &= check_fp8(512, 1024, 1024, 1, swiglu=True)
if not ok:
    raise SystemExit("gemm_tile correctness FAILED")
if a.check_only:
    raise SystemExit(0)

# ---------------------------------------------------------------- timing
t = torch.cuda.tunable
t.enable(True)
t.read_file(os.path.join(REPO, "distributed_llm_inference", "tuning", "tunableop_gfx950.csv"))
t.tuning_enable(False)
H, I = 8192, 28672
SHAPES = {"qkv": (H, 10240), "o": (H, H), "gate_up": (H, 2 * I), "down": (I, H)}


def timed(fn, nrot, iters=20):
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
for M in a.m:
    for name, (K, N) in SHAPES.items():
        nrot = max(2, int(1.0e9 // (N * K * 2)) + 1)
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
        xx = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        flop = 2 * M * N * K
        r = {"hipblaslt_us": round(timed(lambda i: torch.nn.functional.linear(xx, ws[i]), nrot), 1)}
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for sp in (1, 2, 3, 4, 6, 8):
            if sp > 1 and name == "gate_up":
                continue
            wsp = torch.empty(sp * M * N, device=dev, dtype=torch.float32)
            r[f"tile_s{sp}_us"] = round(timed(lambda i: ops.gemm_tile(xx, ws[i], sp, out=out, workspace=wsp), nrot), 1)
        # fp8 weights: hipBLASLt row-wise scaled GEMM vs the fp8 tile kernel
        wq8 = [ops.quantize_weight_fp8(w) for w in ws[:2]]
        xq8, xs8 = ops.quant_rowwise(xx)
        r["fp8_hipblaslt_us"] = round(timed(lambda i: torch._scaled_mm(
            xq8, wq8[i % 2][0].t(), scale_a=xs8, scale_b=wq8[i % 2][1], out_dtype=torch.bfloat16), 2), 1)
        for sp in (1, 2, 3, 4, 6, 8):
            if sp > 1 and name == "gate_up":
                continue
            wsp = torch.empty(sp * M * N, device=dev, dtype=torch.float32)
            r[f"fp8_tile_s{sp}_us"] = round(timed(lambda i: ops.gemm_tile_fp8(
                xq8, xs8, wq8[i % 2][0], wq8[i % 2][1], sp, out=out, workspace=wsp), 2), 1)
        del wq8
        if name == "gate_up":
            o2 = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            r["tile_swiglu_us"] = round(timed(lambda i: ops.gemm_tile(xx, ws[i], swiglu=True, out=o2), nrot), 1)
            h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            r["hipblaslt+silu_mul_us"] = round(timed(lambda i: ops.silu_mul(torch.nn.functional.linear(xx, ws[i])), nrot), 1)
        fbest = min((v, k) for k, v in r.items() if k.startswith("fp8_tile") and k.endswith("_us"))
        r["TF_fp8_hipblaslt"] = round(flop / r["fp8_hipblaslt_us"] / 1e6, 1)
        r["TF_fp8_best_tile"] = round(flop / fbest[0] / 1e6, 1)
        best = min((v, k) for k, v in r.items() if k.startswith("tile") and k.endswith("_us"))
        r["best_tile"] = best[1]
        r["TF_hipblaslt"] = round(flop / r["hipblaslt_us"] / 1e6, 1)
        r["TF_best_tile"] = round(flop / best[0] / 1e6, 1)
        res[f"M{M}_{name}"] = r
        print(f"M={M} {name}", json.dumps(r), flush=True)
        del ws
os.makedirs(os.path.dirname(a.out), exist_ok=True)
json.dump(res, open(a.out, "w"), indent=1)
