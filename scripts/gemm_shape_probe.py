"""Where does the bf16 tile GEMM lose against its template?  Times ``ops.gemm_tile`` (graph replay,
random operands, weights rotated past the Infinity Cache where they are large) on the 70B decode
shapes and on a square 8192^3 reference, next to hipBLASLt on the same operands.

    python scripts/gemm_shape_probe.py            -> gpurun_out/gemm_shape_probe.json
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_llm_inference import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)


def timed(fn, n_inner, reps=10):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n_inner):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * n_inner) * 1e6


def case(name, M, N, K, splits=1, swiglu=False, sets=None, blas=True):
    wbytes = N * K * 2
    sets = sets or max(1, min(6, int(1.2e9 // wbytes) + 1))
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ws = [(torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16) for _ in range(sets)]
    if swiglu:
        ws = [ops.swiglu_interleave(w) for w in ws]
    out = torch.empty(M, N // 2 if swiglu else N, device=dev, dtype=torch.bfloat16)
    wsp = torch.empty(max(splits, 1) * M * N, device=dev) if splits > 1 else None
    if splits == 1 and ops.tile_gemm_stream_k(M, N, dev):
        wsp = None

    def f(i):
        ops.gemm_tile(x, ws[i % sets], splits=splits, swiglu=swiglu, out=out, workspace=wsp)

    us = timed(f, max(sets, 4))
    flop = 2.0 * M * N * K
    r = {"case": name, "M": M, "N": N, "K": K, "splits": splits, "swiglu": swiglu,
         "us": round(us, 1), "TF": round(flop / us / 1e6, 1)}
    if blas:
        o2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def g(i):
            torch.matmul(x, ws[i % sets].t(), out=o2)
        ub = timed(g, max(sets, 4))
        r.update(blas_us=round(ub, 1), blas_TF=round(flop / ub / 1e6, 1))
    print(r, flush=True)
    del ws
    torch.cuda.empty_cache()
    return r


ONLY = [a.split("=", 1)[1].split(",") for a in sys.argv[1:] if a.startswith("--only=")]
NOBLAS = "--no-blas" in sys.argv
_case = case


def case(name, *a, **k):  # noqa: F811 - filtered wrapper
    if ONLY and name not in ONLY[0]:
        return None
    if NOBLAS:
        k["blas"] = False
    return _case(name, *a, **k)


res = []
res.append(case("square8k", 8192, 8192, 8192, sets=2))
res.append(case("square4k", 4096, 4096, 4096, sets=2))
res.append(case("gate_up_M512_swiglu", 512, 57344, 8192, swiglu=True))
res.append(case("gate_up_M512_plain", 512, 57344, 8192))
res.append(case("gate_up_M1024_swiglu", 1024, 57344, 8192, swiglu=True, blas=False))
res.append(case("gate_up_M256_swiglu", 256, 57344, 8192, swiglu=True, blas=False))
res.append(case("gate_up_M512_hotB", 512, 8192, 8192, sets=1, swiglu=True, blas=False))
res.append(case("down_M512_s4", 512, 8192, 28672, splits=4))
res.append(case("qkv_M512_s3", 512, 10240, 8192, splits=3))
res.append(case("o_M512_s4", 512, 8192, 8192, splits=4))
os.makedirs("gpurun_out", exist_ok=True)


def case_fp8(name, M, N, K, splits=1, swiglu=False, sk=False):
    """fp8 e4m3 tile (block-scaled MFMA) vs hipBLASLt's row-scaled fp8 GEMM (torch._scaled_mm)."""
    if ONLY and name not in ONLY[0]:
        return None
    sets = max(1, min(8, int(1.2e9 // (N * K)) + 1))
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    xq, xs = ops.quant_rowwise(x)
    wq, wsc = [], []
    for _ in range(sets):
        q, s_ = ops.quantize_weight_fp8((torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16))
        wq.append(q)
        wsc.append(s_)
    out = torch.empty(M, N // 2 if swiglu else N, device=dev, dtype=torch.bfloat16)
    if sk:
        wsp = torch.empty(ops.native().gemm_tile_sk_workspace_floats(), device=dev)
        sp_ = 0
    else:
        wsp = torch.empty(max(splits, 1) * M * N, device=dev) if splits > 1 else None
        sp_ = splits
    xs1 = xs.reshape(-1).contiguous()
    ws1 = [w.reshape(-1).contiguous() for w in wsc]

    def f(i):
        ops.native().gemm_tile(out, xq, wq[i % sets], int(sp_), 2 if swiglu else 0, wsp, xs1,
                               ws1[i % sets])

    us = timed(f, max(sets, 4))
    flop = 2.0 * M * N * K
    r = {"case": name, "M": M, "N": N, "K": K, "splits": sp_, "swiglu": swiglu, "us": round(us, 1),
         "TF": round(flop / us / 1e6, 1)}
    if not NOBLAS:
        o2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def g(i):
            torch._scaled_mm(xq, wq[i % sets].t(), scale_a=xs, scale_b=wsc[i % sets],
                             out_dtype=torch.bfloat16, out=o2)
        ub = timed(g, max(sets, 4))
        r.update(blas_us=round(ub, 1), blas_TF=round(flop / ub / 1e6, 1))
    print(r, flush=True)
    return r


res.append(case_fp8("fp8_gate_up_swiglu", 512, 57344, 8192, swiglu=True))
res.append(case_fp8("fp8_gate_up_swiglu_sk", 512, 57344, 8192, swiglu=True, sk=True))
res.append(case_fp8("fp8_down_s4", 512, 8192, 28672, splits=4))
res.append(case_fp8("fp8_qkv_s3", 512, 10240, 8192, splits=3))
res.append(case_fp8("fp8_qkv_s2", 512, 10240, 8192, splits=2))
res.append(case_fp8("fp8_o_s4", 512, 8192, 8192, splits=4))
res.append(case_fp8("fp8_o_s2", 512, 8192, 8192, splits=2))
res = [r for r in res if r]
json.dump(res, open("gpurun_out/gemm_shape_probe.json", "w"), indent=1)
