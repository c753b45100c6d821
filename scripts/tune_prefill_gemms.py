"""Pre-tune the chunked-prefill GEMM shapes with PyTorch TunableOp (hipBLASLt / rocBLAS solutions).

Chunked prefill runs almost every step at exactly ``max_num_batched_tokens`` rows (16384 by default),
so its projection GEMMs have fixed shapes per model, like the decode shapes tuned at start-up
(``runtime/gemm_tuning.py``).  Those are too slow to tune at serving start, so they are tuned here
once and merged into the shipped ``tuning/tunableop_gfx950.csv``.

    python scripts/tune_prefill_gemms.py --models llama-3-70b llama-3-8b --tokens 16384
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_inference import ops  # noqa: E402
from distributed_llm_inference.config import resolve_model  # noqa: E402


def shapes(spec):
    h, i = spec.hidden_size, spec.intermediate_size
    return {"qkv": (h, spec.qkv_size), "o": (spec.q_size, h), "gate_up": (h, 2 * i), "down": (i, h)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["llama-3-70b", "llama-3-8b"])
    ap.add_argument("--tokens", type=int, nargs="+", default=[16384])
    ap.add_argument("--out", default="gpurun_out/tunableop_prefill.csv")
    ap.add_argument("--fp8", action="store_true", help="also tune the fp8 row-wise scaled GEMMs")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t = torch.cuda.tunable
    t.enable(True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    t.set_filename(a.out, False)
    t.tuning_enable(True)
    t.set_max_tuning_duration(200)
    t.set_max_tuning_iterations(30)
    for m in a.models:
        spec = resolve_model(m)
        for name, (K, N) in shapes(spec).items():
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            for M in a.tokens:
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                t0 = time.perf_counter()
                F.linear(x, w)
                torch.cuda.synchronize()
                # timed with the selected solution
                t1 = time.perf_counter()
                for _ in range(5):
                    F.linear(x, w)
                torch.cuda.synchronize()
                us = (time.perf_counter() - t1) / 5 * 1e6
                tf = 2 * M * K * N / us / 1e6
                print(f"{m} {name} M={M} bf16: tuned in {t1 - t0:.1f}s, {us:.0f} us, {tf:.0f} TFLOP/s",
                      flush=True)
                if a.fp8:
                    wq, ws = ops.quantize_weight_fp8(w)
                    xq, xs = ops.quant_rowwise(x)
                    torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    for _ in range(5):
                        torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
                    torch.cuda.synchronize()
                    us = (time.perf_counter() - t1) / 5 * 1e6
                    print(f"{m} {name} M={M} fp8: {us:.0f} us, {2 * M * K * N / us / 1e6:.0f} TFLOP/s",
                          flush=True)
            del w
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
