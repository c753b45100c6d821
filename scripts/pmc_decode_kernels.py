"""Workload for PMC passes over the decode-step kernels at the 70B / 512-sequence shapes:
gate|up tile GEMM with the SwiGLU epilogue, the split-K O projection (partials only) — bf16 and
fp8 weights — and the paged decode attention at ~590 keys.  Cold weights (rotating set > Infinity Cache).

    rocprofv3 --pmc <counters> --kernel-trace --output-format csv -d DIR -- python3 scripts/pmc_decode_kernels.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_llm_inference import ops  # noqa: E402
from distributed_llm_inference.ops import reference as ref  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
M, H, I = 512, 8192, 28672
x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
gu = [(torch.randn(2 * I, H, device=dev) * 0.02).to(torch.bfloat16) for _ in range(2)]
wo = [(torch.randn(H, H, device=dev) * 0.02).to(torch.bfloat16) for _ in range(4)]
sp = ops.tile_gemm_splits(M, H, H)
for i in range(6):
    ops.gemm_tile(x, gu[i % 2], swiglu=True)
    ops.gemm_tile(x, wo[i % 4], splits=sp, defer_reduce=True)
# fp8 weights: the same two products on the block-scaled fp8 MFMA (rows / scales interleaved for
# the SwiGLU epilogue as the engine does)
xq, xs = ops.quant_rowwise(x)
gq = [ops.quantize_weight_fp8(ops.swiglu_interleave(g)) for g in gu]
oq = [ops.quantize_weight_fp8(w) for w in wo]
spf = ops.tile_gemm_splits_fp8(M, H, H)
for i in range(6):
    ops.gemm_tile_fp8(xq, xs, gq[i % 2][0], gq[i % 2][1], swiglu=True)
    ops.gemm_tile_fp8(xq, xs, oq[i % 4][0], oq[i % 4][1], splits=spf, defer_reduce=True)
# decode attention: 512 sequences x 590 keys, 64 q heads / 8 kv heads, D = 128
B, L, nh, nkv, D, bs = 512, 590, 64, 8, 128, 64
nb_per = (L + bs - 1) // bs
kc = torch.randn(B * nb_per, nkv, bs, D, device=dev, dtype=torch.bfloat16)
vc = torch.randn(B * nb_per, nkv, bs // 8, D, 8, device=dev, dtype=torch.bfloat16)
bt = torch.arange(B * nb_per, device=dev, dtype=torch.int32).reshape(B, nb_per)
lens = torch.full((B,), L, device=dev, dtype=torch.int32)
q = torch.randn(B, nh, D, device=dev, dtype=torch.bfloat16)
splits = ops.decode_splits(B, nkv, nh // nkv, L)
for i in range(6):
    ops.attn_decode(q, None, kc, vc, bt, lens, D ** -0.5, num_splits=splits)
torch.cuda.synchronize()
print("done")
