"""Building blocks shared by the model families (Llama, GPT-2).

* :class:`Linear` — bf16 weights (hand-written tile GEMM / GEMV for decode, hipBLASLt otherwise),
  fp8-e4m3 weights with per-output-channel scales and per-token dynamic activation scales (the
  MI355X-native 8-bit default), or LLM.int8 weights with the reference's outlier ``threshold``
  (int8 MFMA + bf16 outlier columns) — the replacements of the reference's bitsandbytes
  ``Linear8bitLt`` (utils/model.py:93-113).
* :class:`AttnMetadata` — per-batch device metadata consumed by the attention / cache kernels
  (positions, slot mapping, block tables, sequence lengths, varlen offsets, window policy).  It
  replaces the reference's dense additive causal/padding mask (model.py:78-143): causality,
  padding and windows are all derived in-kernel from these small int tensors.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class Linear(nn.Module):
    """``y = x W^T (+ b)`` with W stored [out, in]; optional fp8 weights."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False,
                 dtype: torch.dtype = torch.bfloat16, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype,
                                               device=device), requires_grad=False)
        self.bias = (nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device),
                                  requires_grad=False) if bias else None)
        self.register_buffer("weight_fp8", None, persistent=False)
        self.register_buffer("weight_scale", None, persistent=False)
        self.register_buffer("weight_int8", None, persistent=False)
        self.register_buffer("weight_int8_t", None, persistent=False)
        self.int8_threshold = 0.0
        # which projection of its layer this is ("qkv" / "o" / "gate_up" / "down", set by the
        # model): KernelPolicy.fp8_gemm4 routes fp8 products per role
        self.role = ""

    @property
    def is_fp8(self) -> bool:
        return self.weight_fp8 is not None

    @property
    def is_int8(self) -> bool:
        return self.weight_int8 is not None

    def quantize_int8(self, threshold: float = 6.0, keep_bf16: bool = False) -> None:
        """LLM.int8 weights (reference utils/model.py:93-113, bitsandbytes ``Linear8bitLt(threshold)``):
        per-channel absmax int8 + bf16 outlier-column decomposition at run time."""
        q, s = ops.quantize_weight_int8(self.weight.data)
        self.weight_int8, self.weight_scale = q, s
        # Optional (KernelPolicy.int8_transposed): a transposed [K, N] copy so the per-product outlier
        # weight-column gather reads contiguous rows (int8_outlier.hip gather_wt): 1.6 vs 2.9
        # ms/step on the 70B --int8 bench (+2.5 % tok/s), but it costs a second byte per weight,
        # i.e. the memory LLM.int8 exists to save (70B PP=1: KV blocks 9413 -> 6323, -33 %
        # concurrent sequences).  Off by default; opt in when KV capacity is not the limit.
        self.weight_int8_t = (q.t().contiguous() if q.is_cuda and ops.policy().int8_transposed
                              else None)
        self.int8_threshold = float(threshold)
        if not keep_bf16:
            self.weight = nn.Parameter(torch.empty(0, dtype=self.weight.dtype,
                                                   device=self.weight.device), requires_grad=False)

    def quantize_fp8(self, keep_bf16: bool = False) -> None:
        """Quantise W to fp8 e4m3 (per output channel).  Frees the bf16 copy unless asked not to."""
        q, s = ops.quantize_weight_fp8(self.weight.data)
        self.weight_fp8, self.weight_scale = q, s
        if not keep_bf16:
            self.weight = nn.Parameter(torch.empty(0, dtype=self.weight.dtype,
                                                   device=self.weight.device), requires_grad=False)

    def stream_weights(self):
        """(weight, per-row scale or None, bias or None) in the format the weight-streaming
        kernels read: bf16 [N, K], fp8 e4m3 [N, K] or int8 [N, K] with fp32 scales [N]."""
        if self.weight_fp8 is not None:
            return self.weight_fp8, self.weight_scale.reshape(-1), self.bias
        if self.weight_int8 is not None:
            return self.weight_int8, self.weight_scale.reshape(-1), self.bias
        return self.weight, None, self.bias

    def tile_splits(self, x: torch.Tensor) -> int:
        """Split-K factor if ``gemm_tile`` takes this product on the GPU, else 0."""
        if (self.bias is not None or not x.is_cuda or x.dim() != 2 or x.dtype != torch.bfloat16
                or not x.is_contiguous() or self.weight_fp8 is not None
                or self.weight_int8 is not None):
            return 0
        return ops.tile_gemm_splits(x.shape[0], self.out_features, self.in_features)

    def gemv_ok(self, rows: int, swiglu: bool = False, bf16_rows: bool = True) -> bool:
        """Whether :meth:`gemv` takes a product of ``rows`` GPU rows (bf16 rows, or with
        ``bf16_rows=False`` the fused quantiser's fp8 rows for fp8 weights)."""
        if not 1 <= rows <= ops.SKINNY_DISPATCH_M:
            return False
        if swiglu and (self.bias is not None or self.out_features % 32):
            return False
        if self.weight_int8 is not None:
            return bf16_rows and self.in_features % 16 == 0 and ops.policy().gemv
        if self.weight_fp8 is not None:
            return self.in_features % 16 == 0 and ops.policy().gemv
        return bf16_rows and self.in_features % 8 == 0 and ops.policy().gemv

    def gemv(self, x: Optional[torch.Tensor], x_q: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
             swiglu: bool = False, norm: Optional["ops.RowNorm"] = None) -> Optional[torch.Tensor]:
        """The weight-streaming GEMV (1-2 decode rows on the GPU) of this Linear, with its
        optional fused epilogue (``swiglu``: this is a swiglu_interleave'd gate|up projection,
        silu(gate) * up is returned) and fused prologue (``norm``: x is the un-normalised row and
        the GEMV applies the input RMSNorm itself).  None when the GEMV does not take the
        product (more rows, CPU, shapes it does not cover) -- the caller falls back."""
        src = x if x is not None else (x_q[0] if x_q is not None else None)
        if (src is None or not src.is_cuda or src.dim() != 2 or isinstance(x_q, ops.MxFp8)
                or not self.gemv_ok(src.shape[0], swiglu, bf16_rows=x is not None)):
            return None
        if x is not None and (x.dtype != torch.bfloat16 or not x.is_contiguous()):
            return None
        if norm is not None and x is None:
            return None
        if self.weight_int8 is not None:
            return ops.skinny_gemm_int8(x, self.weight_int8, self.weight_scale, self.bias,
                                        swiglu=swiglu, norm=norm)
        if self.weight_fp8 is not None:
            if norm is not None or (x_q is None and x is not None):
                return ops.skinny_gemm_fp8(x, self.weight_fp8, self.weight_scale, None, self.bias,
                                           swiglu=swiglu, norm=norm)
            xq, xs = x_q if x_q is not None else ops.quant_rowwise(x)
            return ops.skinny_gemm_fp8(xq, self.weight_fp8, self.weight_scale, xs, self.bias,
                                       swiglu=swiglu)
        return ops.skinny_gemm(x, self.weight, self.bias, swiglu=swiglu, norm=norm)

    def gemv_qkv_rope(self, x: torch.Tensor, meta: "AttnMetadata", k_cache: torch.Tensor,
                      v_cache: torch.Tensor, cos_sin: torch.Tensor, nh: int, nkv: int,
                      head_dim: int, norm: Optional["ops.RowNorm"] = None
                      ) -> Optional[torch.Tensor]:
        """This Linear as the fused QKV projection of 1-2 decode rows with RoPE and the paged
        KV write in the GEMV's epilogue (see :func:`ops.skinny_gemm_qkv_rope`): returns q
        [M, nh, D], or None when that path does not apply (window mode's sink query, more rows,
        CPU) -- the caller then runs the GEMV and rope_cache separately."""
        if (x is None or not x.is_cuda or x.dim() != 2 or x.dtype != torch.bfloat16
                or not self.gemv_ok(x.shape[0]) or meta.want_sink or meta.custom_mask is not None
                or self.out_features != (nh + 2 * nkv) * head_dim):
            return None
        if self.weight_int8 is not None:
            w, ws = self.weight_int8, self.weight_scale
        elif self.weight_fp8 is not None:
            w, ws = self.weight_fp8, self.weight_scale
        else:
            w, ws = self.weight, None
        return ops.skinny_gemm_qkv_rope(x, w, ws, self.bias, meta.positions, meta.slot_mapping,
                                        cos_sin, nh, nkv, head_dim, k_cache, v_cache,
                                        meta.k_scale, meta.v_scale, norm=norm)

    def gemv_swiglu(self, x: Optional[torch.Tensor],
                    x_q: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
                    ) -> Optional[torch.Tensor]:
        """silu(gate) * up straight from the GEMV's epilogue (see :meth:`gemv`)."""
        return self.gemv(x, x_q, swiglu=True)

    def forward(self, x: Optional[torch.Tensor],
                x_q: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                defer_reduce: bool = False):
        """``x_q`` = (fp8 rows, scales) already quantised by a fused producer kernel; then ``x`` may
        be None (fp8 weights only).  ``defer_reduce``: a split-K tile GEMM returns its fp32
        partials (``ops.SplitKPartials``) for an RMSNorm consumer to reduce."""
        if self.weight_int8 is not None:
            if (x.is_cuda and x.dim() == 2 and 1 <= x.shape[0] <= ops.SKINNY_DISPATCH_M
                    and x.dtype == torch.bfloat16 and self.in_features % 16 == 0
                    and ops.policy().gemv):
                # 1-2 row decode: int8 weight-streaming GEMV on the bf16 rows (the weights are
                # the whole cost; bf16 activations need no outlier decomposition)
                return ops.skinny_gemm_int8(x, self.weight_int8, self.weight_scale, self.bias)
            y = ops.llm_int8_linear(x.reshape(-1, self.in_features), self.weight_int8,
                                    self.weight_scale, self.int8_threshold,
                                    wq_t=self.weight_int8_t,
                                    defer_reduce=defer_reduce and self.bias is None)
            if isinstance(y, ops.SplitKPartials):   # the consumer reduces (rms_norm / rope_cache)
                return y
            y = y.reshape(*x.shape[:-1], self.out_features)
            return y + self.bias if self.bias is not None else y
        if self.weight_fp8 is None:
            if (x.is_cuda and x.dim() == 2 and 1 <= x.shape[0] <= ops.SKINNY_DISPATCH_M
                    and x.dtype == torch.bfloat16 and x.is_contiguous()
                    and self.in_features % 8 == 0 and ops.policy().gemv):
                # 1-2 row decode batches: weight-streaming HIP kernel (csrc/kernels/gemv.hip)
                return ops.skinny_gemm(x, self.weight, self.bias)
            sp = self.tile_splits(x)
            if sp:  # decode micro-batches: 256x256 MFMA tile kernel (csrc/kernels/gemm_tile.hip)
                return ops.gemm_tile(x, self.weight, splits=sp, defer_reduce=defer_reduce)
            return F.linear(x, self.weight, self.bias)
        if isinstance(x_q, ops.MxFp8):
            # MX activations from the fp8 SwiGLU epilogue: their e8m0 block scales go to the
            # block-scaled MFMA (gemm_tile.hip kFp8Mx); the MLP only hands these over when the
            # product is tileable (LlamaMLP.forward)
            sp = ops.tile_gemm_splits_fp8(x_q.q.shape[0], self.out_features, self.in_features)
            y = ops.gemm_tile_fp8_mx(x_q, self.weight_fp8, self.weight_scale, sp or 1,
                                     defer_reduce=defer_reduce and self.bias is None,
                                     gemm4=ops.policy().fp8_on_gemm4(self.role))
            if self.bias is not None:
                y = y + self.bias
            return y
        if (x_q is None and x is not None and x.is_cuda and x.dim() == 2
                and 1 <= x.shape[0] <= ops.SKINNY_DISPATCH_M and x.dtype == torch.bfloat16
                and self.in_features % 16 == 0 and ops.policy().gemv):
            # 1-2 row decode: fp8 weight-streaming GEMV on the bf16 rows (no quantisation pass;
            # KernelPolicy.gemv=False quantises the rows as a batch of >= 3 would --
            # docs/parity.md C11)
            return ops.skinny_gemm_fp8(x, self.weight_fp8, self.weight_scale, None, self.bias)
        if x_q is None:
            x_q = ops.quant_rowwise(x)
        xq, xs = x_q
        if (xq.is_cuda and xq.dim() == 2 and 1 <= xq.shape[0] <= ops.SKINNY_DISPATCH_M
                and self.in_features % 16 == 0 and ops.policy().gemv):
            # 1-2 row decode on the fused quantiser's fp8 rows: half the weight bytes of bf16
            # streamed by the GEMV kernel (hipBLASLt's fp8 GEMM at M = 1 streamed them slower
            # than the bf16 GEMV: Llama-3.1-70B batch-1 decode ran at the bf16 speed)
            return ops.skinny_gemm_fp8(xq, self.weight_fp8, self.weight_scale, xs, self.bias)
        if xq.is_cuda and self.bias is None and xq.dim() == 2:
            sp = ops.tile_gemm_splits_fp8(xq.shape[0], self.out_features, self.in_features)
            if sp:  # long-K fp8 products: block-scaled MFMA tile kernel (csrc/kernels/gemm_tile.hip)
                return ops.gemm_tile_fp8(xq, xs, self.weight_fp8, self.weight_scale, sp,
                                         defer_reduce=defer_reduce,
                                         gemm4=ops.policy().fp8_on_gemm4(self.role))
        if xq.is_cuda:
            y = torch._scaled_mm(xq, self.weight_fp8.t(), scale_a=xs, scale_b=self.weight_scale,
                                 out_dtype=torch.bfloat16)
        else:  # CPU: dequantised reference
            y = ((xq.float() * xs) @ (self.weight_fp8.float() * self.weight_scale.t()).t()
                 ).to(torch.bfloat16)
        if self.bias is not None:
            y = y + self.bias
        return y

    def extra_repr(self) -> str:
        return (f"in={self.in_features}, out={self.out_features}, bias={self.bias is not None}, "
                f"fp8={self.is_fp8}, int8={self.is_int8}")


@dataclass
class AttnMetadata:
    """Device metadata of one forward batch (varlen: T tokens from B sequences)."""

    num_tokens: int
    num_seqs: int
    is_decode: bool                  # every sequence contributes exactly one new token
    positions: torch.Tensor          # [T] int32 rope positions
    slot_mapping: torch.Tensor       # [T] int64 physical cache slot (-1: don't write)
    block_tables: torch.Tensor       # [B, max_blocks] int32
    seq_lens: torch.Tensor           # [B] int32 (absolute length incl. new tokens)
    q_start: torch.Tensor            # [B+1] int32 token offsets
    max_q: int
    num_splits: int = 1
    workspace: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    # attention-sink window policy (all zero for a full cache)
    n_sink: int = 0
    sink_pad: int = 0
    ring: int = 0
    window: int = 0
    # fp8 KV cache scales (stored = x / scale); 1.0 for bf16 caches
    k_scale: float = 1.0
    v_scale: float = 1.0
    # prefill work list [n_tiles, 2] (sequence, token tile) for the attention kernel, or None
    tile_map: Optional[torch.Tensor] = None
    # rows (token index) whose hidden state feeds the LM head, or None = all rows
    logits_rows: Optional[torch.Tensor] = None
    # caller-supplied pre-inverted additive 4-D mask [B, 1|nh, T, >= L] (LlamaBlock.forward's
    # reference-compatible path): replaces the in-kernel causal mask
    custom_mask: Optional[torch.Tensor] = None

    @property
    def windowed(self) -> bool:
        return self.ring > 0

    @property
    def want_sink(self) -> bool:
        return self.ring > 0 and self.n_sink > 0


def seeded_normal_(t: torch.Tensor, seed: int, std: float) -> torch.Tensor:
    """Deterministic N(0, std) init independent of device placement order (so a PP=8 split and a
    PP=1 model built from the same seed hold identical weights)."""
    g = torch.Generator(device=t.device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    with torch.no_grad():
        if t.dtype in (torch.float32, torch.float64):
            t.normal_(0.0, std, generator=g)
        else:
            # generate in chunks to bound the fp32 temporary
            flat = t.view(-1)
            step = 1 << 26
            for i in range(0, flat.numel(), step):
                chunk = flat[i:i + step]
                tmp = torch.empty(chunk.shape, dtype=torch.float32, device=t.device)
                tmp.normal_(0.0, std, generator=g)
                chunk.copy_(tmp)
    return t


def param_seed(base: int, layer_idx: int, name: str) -> int:
    h = 1469598103934665603
    for ch in f"{layer_idx}:{name}".encode():
        h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return (h ^ (base * 0x9E3779B97F4A7C15)) & 0x7FFFFFFFFFFFFFFF
