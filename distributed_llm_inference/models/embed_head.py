"""Token embedding (first stage) and final norm + LM head (last stage).

Absent from the reference, whose ``LlamaBlock`` has no embedding, final norm or LM head
 — the generation loop is closed here: stage 0 embeds, the last stage produces
logits for the rows that sample and hands them to the sampling kernel (csrc/kernels/sampling.hip).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..config import ModelSpec
from .common import Linear, param_seed, seeded_normal_


class Embedding(nn.Module):
    def __init__(self, spec: ModelSpec, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.spec = spec
        self.weight = nn.Parameter(torch.empty(spec.vocab_size, spec.hidden_size, dtype=dtype,
                                               device=device), requires_grad=False)
        self.position = None
        if spec.arch == "gpt2":
            self.position = nn.Parameter(torch.empty(spec.max_position_embeddings, spec.hidden_size,
                                                     dtype=dtype, device=device),
                                         requires_grad=False)

    def init_random(self, seed: int, std: float = 0.02):
        seeded_normal_(self.weight.data, param_seed(seed, -1, "embed_tokens"), std)
        if self.position is not None:
            seeded_normal_(self.position.data, param_seed(seed, -1, "wpe"), 0.01)
        return self

    def forward(self, input_ids: torch.Tensor, positions: Optional[torch.Tensor] = None):
        h = F.embedding(input_ids.long(), self.weight)
        if self.position is not None:
            if positions is None:
                raise ValueError("GPT-2 embedding needs positions")
            h = ops.add(h.contiguous(), F.embedding(positions.long(), self.position).contiguous())
        return h


class LMHead(nn.Module):
    """Final norm (RMSNorm for Llama, LayerNorm for GPT-2) + vocabulary projection."""

    def __init__(self, spec: ModelSpec, device=None, dtype=torch.bfloat16,
                 tied: Optional[Embedding] = None):
        super().__init__()
        self.spec = spec
        h = spec.hidden_size
        self.norm_weight = nn.Parameter(torch.ones(h, dtype=dtype, device=device), requires_grad=False)
        self.norm_bias = (nn.Parameter(torch.zeros(h, dtype=dtype, device=device), requires_grad=False)
                          if spec.arch == "gpt2" else None)
        self._tied = tied
        self.proj = None if tied is not None else Linear(h, spec.vocab_size, dtype=dtype, device=device)

    def init_random(self, seed: int, std: float = 0.02):
        self.norm_weight.data.fill_(1.0)
        if self.norm_bias is not None:
            self.norm_bias.data.zero_()
        if self.proj is not None:
            seeded_normal_(self.proj.weight.data, param_seed(seed, -2, "lm_head"), std)
        return self

    def forward(self, hidden: torch.Tensor, residual: Optional[torch.Tensor] = None,
                rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``hidden``/``residual`` are the last layer's (out, residual) pair (residual may be None
        when ``hidden`` already is the full hidden state).  Only ``rows`` produce logits."""
        return self.project(self.norm(hidden, residual, rows))

    def norm(self, hidden: torch.Tensor, residual: Optional[torch.Tensor] = None,
             rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The final norm alone (what the last pipeline stage sends when another rank runs the
        vocabulary projection: runtime/head.py)."""
        if rows is not None:
            hidden = hidden.index_select(0, rows)
            if residual is not None:
                residual = residual.index_select(0, rows)
        elif residual is not None:
            residual = residual.clone()  # do not clobber the caller's residual stream
        if self.norm_bias is None:
            normed, _ = ops.rms_norm(hidden, self.norm_weight, self.spec.rms_norm_eps, residual)
        else:
            normed, _ = ops.layer_norm(hidden, self.norm_weight, self.norm_bias,
                                       self.spec.rms_norm_eps, residual)
        return normed

    def project(self, normed: torch.Tensor, tile: bool = False) -> torch.Tensor:
        """Vocabulary projection of final-normed hidden states -> logits.  ``tile``: on the GPU
        take the hand-written tile GEMM even where hipBLASLt is faster (the rotating head's side
        stream: a library stream-K kernel there may be in flight next to another one on the
        compute stream, and persistent kernels that wait for each other's workgroups can
        deadlock - ops.library_gemms)."""
        w = self._tied.weight if self.proj is None else self.proj.weight
        if (tile and normed.is_cuda and normed.dim() == 2 and normed.dtype == torch.bfloat16
                and w.dtype == torch.bfloat16 and w.numel() and w.shape[0] % 256 == 0
                and (self.proj is None or self.proj.bias is None)
                and (w.shape[1] * 2) % 128 == 0):
            return ops.gemm_tile(normed.contiguous(), w, splits=1)
        if self.proj is None:
            return F.linear(normed, self._tied.weight)
        return self.proj(normed)
