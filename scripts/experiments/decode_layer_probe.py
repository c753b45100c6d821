#!/usr/bin/env python3
"""Phase timeline of the persistent batch-1 decode-layer kernel (csrc/kernels/decode_layer.hip)
on Llama-3-70B-shaped layers: per-workgroup wall stamps (DLI_DL_STAMPS=1) at every grid barrier
arrival / release, summarised as phase durations (last arrival - previous release) and barrier
latencies (first release - last arrival), next to the whole-layer time of the six-kernel path.

    python3 scripts/decode_layer_probe.py [bf16|fp8|int8] [context]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference.config import PRESETS  # noqa: E402
from distributed_llm_inference.models import CausalLMStage  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "fp8"
ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 600
dev = torch.device("cuda", 0)
L = 4
spec = PRESETS["llama-3-70b"]
stage = CausalLMStage(spec, 0, L, device=dev).init_random(1)
if fmt == "fp8":
    stage.block.quantize_fp8()
elif fmt == "int8":
    stage.block.quantize_int8()
stage.block.set_fused_swiglu(True)
pool = stage.make_pool(64, block_size=64)
pool.manager.append(0, ctx)
meta = pool.build_metadata([0], [ctx])
meta.logits_rows = torch.tensor([ctx - 1], device=dev)
stage(torch.arange(1, ctx + 1, dtype=torch.int32, device=dev) % 1000, meta, pool)
torch.cuda.synchronize()


def step(flag, n=10):
    os.environ["DLI_DECODE_LAYER"] = flag
    ts = []
    for s in range(n):
        pool.manager.append(0, 1)
        m = pool.build_metadata([0], [1])
        tok = torch.tensor([s + 7], dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stage(tok, m, pool)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def graph_step(flag, reps=20):
    """the same decode step replayed from a hipGraph (as the engine runs it)"""
    os.environ["DLI_DECODE_LAYER"] = flag
    pool.manager.append(0, 1)
    m = pool.build_metadata([0], [1])
    tok = torch.tensor([5], dtype=torch.int32, device=dev)
    s_ = torch.cuda.Stream()
    with torch.cuda.stream(s_):
        for _ in range(2):
            stage(tok, m, pool)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s_):
        stage(tok, m, pool)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


g_mk = graph_step("1")
g_six = graph_step("0")
print(f"graph replay, {L} layers: decode-layer kernel {g_mk:.3f} ms, six-kernel path {g_six:.3f} ms")
os.environ["DLI_DL_STAMPS"] = "1"
t_mk = step("1")
t_six = step("0")
step("1", 2)
st = stage.block.layers[1]._dl_stamps.view(-1, 24).cpu().double()
t0 = st[:, 0].min()
rel = (st - t0) / 100.0   # us
names = ["P1 norm+QKV+RoPE", "P2 attention", "P4 merge+O", "P5 norm+gate|up", "P6 down"]
prev_release = 0.0
print(f"{fmt} ctx {ctx}: step with {L} layers (+ head): decode-layer kernel {t_mk:.3f} ms, "
      f"six-kernel path {t_six:.3f} ms")
for k in range(1, 5):
    arr, rls = rel[:, 2 * k - 1], rel[:, 2 * k]
    print(f"  {names[k - 1]:18s} ends {arr.max():7.1f} us (median arrival {arr.median():7.1f}) "
          f"-> {arr.max() - prev_release:6.1f} us;  barrier {k}: release {rls.min():7.1f}..{rls.max():7.1f}"
          f" (latency {rls.min() - arr.max():5.1f} us, L2 write-back med "
          f"{(rel[:, 12 + k] - arr).median():4.1f} max {(rel[:, 12 + k] - arr).max():4.1f} us)")
    prev_release = rls.min().item()
print(f"  (merge + staging of the O input: median {(rel[:, 20] - rel[:, 4]).median():.1f} us, "
      f"max {(rel[:, 20] - rel[:, 4]).max():.1f} us after barrier 2)")
end = rel[:, 9]
print(f"  {names[4]:18s} ends {end.max():7.1f} us -> {end.max() - prev_release:6.1f} us;  "
      f"kernel start skew {rel[:, 0].max():.1f} us")
print("errors", sum(l.decode_layer_errors() for l in stage.block.layers))
