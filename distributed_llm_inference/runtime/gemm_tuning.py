"""hipBLASLt solution tuning for the fixed decode GEMM shapes (PyTorch TunableOp).

Decode GEMMs have a handful of fixed shapes per stage (M = graph batch bucket; N, K = the fused
QKV / O / gate-up / down / LM-head weights).  hipBLASLt's default heuristic is far from the best
solution at these skinny M (measured on MI355X, 70B shapes: down-proj M=128 200 -> 138 us, M=256
313 -> 183 us).  At startup each stage benchmarks every hipBLASLt solution for exactly its decode
shapes — with a rotating buffer larger than the 256 MiB Infinity Cache so that weights stream
from HBM as they do in the real step — then disables tuning so prefill's variable shapes keep the
default heuristic (no tuning stalls at serve time).  Results persist in a per-device CSV (shipped
pre-tuned results in ``tuning/`` are read first) so later runs start instantly.
"""
from __future__ import annotations

import logging
import os
from typing import Iterable, List, Optional, Sequence, Set, Tuple

import torch
import torch.nn.functional as F

log = logging.getLogger(__name__)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIPPED = os.path.join(PKG_DIR, "tuning", "tunableop_gfx950.csv")


def _weights(stage) -> List[torch.Tensor]:
    """One representative bf16 weight per distinct GEMM shape."""
    from ..models.common import Linear
    ws, seen = [], set()
    for m in stage.modules():
        if isinstance(m, Linear) and m.weight is not None and m.weight.numel() > 0 and not m.is_fp8:
            key = tuple(m.weight.shape)
            if key not in seen:
                seen.add(key)
                ws.append(m.weight)
    if getattr(stage, "head", None) is not None and stage.head.proj is None and stage.embed is not None:
        ws.append(stage.embed.weight)  # tied LM head
    return ws


def _fp8_linears(stage) -> list:
    """One representative fp8 Linear per distinct weight shape (row-wise scaled GEMMs)."""
    from ..models.common import Linear
    out, seen = [], set()
    for m in stage.modules():
        if isinstance(m, Linear) and m.is_fp8:
            key = tuple(m.weight_fp8.shape)
            if key not in seen:
                seen.add(key)
                out.append(m)
    return out


def tune_decode_gemms(stage, batch_sizes: Iterable[int], results_file: Optional[str] = None,
                      max_duration_ms: int = 60) -> None:
    if not torch.cuda.is_available() or stage.device.type != "cuda":
        return
    if os.environ.get("DLI_TUNING_DIR", "") == "off":
        return   # DLI_TUNING_DIR=off: no TunableOp at all (tests, short runs)
    t = torch.cuda.tunable
    t.enable(True)
    for f in (SHIPPED, results_file):
        if f and os.path.exists(f):
            try:
                t.read_file(f)
            except Exception as e:  # pragma: no cover
                log.warning("could not read tuning file %s: %s", f, e)
    if results_file:
        os.makedirs(os.path.dirname(results_file) or ".", exist_ok=True)
        t.set_filename(results_file, True)
    t.tuning_enable(True)
    t.set_max_tuning_duration(max_duration_ms)
    t.set_max_tuning_iterations(100)
    t.set_rotating_buffer_size(512)  # MiB, > Infinity Cache: tune for HBM-streamed weights
    with torch.inference_mode():
        from .. import ops
        for w in _weights(stage):
            for M in sorted(set(int(b) for b in batch_sizes)):
                if ops.tile_gemm_splits(M, w.shape[0], w.shape[1]):
                    continue  # served by the hand-written tile GEMM, not hipBLASLt
                x = torch.randn(M, w.shape[1], dtype=w.dtype, device=w.device)
                F.linear(x, w)
        for lin in _fp8_linears(stage):
            for M in sorted(set(int(b) for b in batch_sizes)):
                x = torch.randn(M, lin.in_features, dtype=torch.bfloat16, device=stage.device)
                lin(None, x_q=ops.quant_rowwise(x))
    torch.cuda.synchronize()
    t.tuning_enable(False)  # keep using the results; never tune inside serving / capture
    # (torch writes results_file at interpreter exit; multi-rank bench.py ranks skip that, so they
    # re-tune on their next start: the shipped table covers the common shapes)
    log.info("TunableOp: decode GEMMs tuned for batch sizes %s", sorted(set(batch_sizes)))
