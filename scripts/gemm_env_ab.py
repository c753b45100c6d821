"""In-process interleaved A/B of bf16 tile GEMM variants selected by an environment switch the
launcher reads per launch (--env / --vals; e.g. DLI_GEMM_VAR, csrc/kernels/gemm_tile.hip) on the 70B decode shapes as the decode step calls
them (gate|up with the SwiGLU epilogue, QKV / O / down as bf16 split-K partials), a ragged M and
8192^3: bitwise identity of the variants, an fp32 reference check, then graph-replay timing with
weights rotated past the Infinity Cache (median / min per variant, alternating order).

    python scripts/gemm_ks_ab.py --env DLI_GEMM_VAR --vals 0,1,2,3   -> gpurun_out/gemm_ks_ab.json

(profiles/gemm_ks_ab.json: the k-split main loop, DLI_GEMM_KS, since removed: bit-identical and
11-35 % slower.)
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--shapes", default="")
ap.add_argument("--env", default="DLI_GEMM_KS", help="variant switch read by the launcher")
ap.add_argument("--vals", default="0,1")
ap.add_argument("--out", default="gpurun_out/gemm_ks_ab.json")
a = ap.parse_args()
VARS = a.vals.split(",")
dev = torch.device("cuda:0")
torch.manual_seed(0)
SHAPES = {"gate_up_swiglu": (512, 57344, 8192, 1, True), "down_s4": (512, 8192, 28672, 4, False),
          "qkv_s3": (512, 10240, 8192, 3, False), "o_s4": (512, 8192, 8192, 4, False),
          "gate_up_M300": (300, 57344, 8192, 1, True), "o_M300_s4": (300, 8192, 8192, 4, False),
          "square8k": (8192, 8192, 8192, 1, False), "plain_M512": (512, 57344, 8192, 1, False)}
if a.shapes:
    SHAPES = {k: v for k, v in SHAPES.items() if k in a.shapes.split(",")}


def make(M, N, K, splits, swiglu):
    sets = max(1, min(6, int(1.2e9 // (N * K * 2)) + 1))
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ws = [(torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16) for _ in range(sets)]
    if swiglu:
        ws = [ops.swiglu_interleave(w) for w in ws]
    out = torch.empty(M, N // 2 if swiglu else N, device=dev, dtype=torch.bfloat16)
    hold = {}

    def f(i):
        if splits > 1:
            hold["p"] = ops.gemm_tile(x, ws[i % sets], splits=splits, defer_reduce=True)
        else:
            ops.gemm_tile(x, ws[i % sets], splits=1, swiglu=swiglu, out=out)

    def result():
        if splits > 1:
            p = hold["p"]
            t = getattr(p, "parts", None)
            return (t if t is not None else p).clone()
        return out.clone()

    graphs, outs = {}, {}
    for v in VARS:
        os.environ[a.env] = v
        f(0)
        torch.cuda.synchronize()
        outs[v] = result()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(max(sets, 4)):
                f(i)
        graphs[v] = (g, max(sets, 4))
    same = all(torch.equal(outs[VARS[0]], outs[v]) for v in VARS[1:])
    # fp32 reference of the first weight set (the split parts summed)
    w0 = ops.swiglu_deinterleave(ws[0]) if swiglu else ws[0]
    ref = x.float() @ w0.float().t()
    if swiglu:
        ref = ref.to(torch.bfloat16).float()
        ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
    got = outs[VARS[-1]].float()
    if splits > 1:
        got = got.view(splits, M, N).sum(0)
    err = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
    return graphs, (ws, x, out, hold), same, err


res = {}
for name, shp in SHAPES.items():
    graphs, keep, same, err = make(*shp)
    times = {v: [] for v in VARS}
    for r in range(a.rounds):
        for v in (VARS if r % 2 == 0 else VARS[::-1]):
            g, n = graphs[v]
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / (5 * n) * 1e6)
    M, N, K = shp[:3]
    res[name] = {"shape": shp, "bitwise_equal": same, "rel_err_vs_fp32": round(err, 5)}
    for v, t in times.items():
        med = statistics.median(t)
        res[name][a.env + "=" + v] = {"median_us": round(med, 1), "min_us": round(min(t), 1),
                               "TF": round(2.0 * M * N * K / med / 1e6, 1)}
    print(name, res[name], flush=True)
    assert same, f"{name}: the two main loops differ"
    assert err < 2e-2, f"{name}: error {err} vs the fp32 reference"
    del graphs, keep
    torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open(a.out, "w"), indent=1)
