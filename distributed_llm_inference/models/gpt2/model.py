"""GPT-2 stage family (BASELINE config 1: "GPT-2-small single-process CPU forward via
distributed_llm_inference/models").

The reference has no GPT-2 (SURVEY §6 note); this family exercises the same stage / cache /
pipeline plumbing with a different block: LayerNorm, fused ``c_attn`` with bias (HF Conv1D
weights are stored transposed and are transposed at load time), learned absolute position
embeddings (in the stage-0 embedding; no RoPE — the cache kernel is called without a cos/sin
table) and a tanh-GELU MLP whose bias is fused into the activation kernel.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ... import ops
from ...config import ModelSpec, resolve_model
from ..common import AttnMetadata, Linear, param_seed, seeded_normal_


class LayerNorm(nn.Module):
    def __init__(self, h, eps, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(h, dtype=dtype, device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(h, dtype=dtype, device=device), requires_grad=False)
        self.eps = eps

    def forward(self, x, residual=None, residual_out=None):
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual,
                              residual_out=residual_out)


class GPT2Layer(nn.Module):
    def __init__(self, spec: ModelSpec, layer_idx: int, device=None, dtype=torch.bfloat16):
        super().__init__()
        h = spec.hidden_size
        self.layer_idx = layer_idx
        self.num_heads, self.head_dim = spec.num_heads, spec.head_dim
        self.scale = spec.head_dim ** -0.5
        self.ln_1 = LayerNorm(h, spec.rms_norm_eps, device, dtype)
        self.c_attn = Linear(h, 3 * h, bias=True, dtype=dtype, device=device)
        self.attn_proj = Linear(h, h, bias=True, dtype=dtype, device=device)
        self.ln_2 = LayerNorm(h, spec.rms_norm_eps, device, dtype)
        self.c_fc = Linear(h, spec.intermediate_size, bias=False, dtype=dtype, device=device)
        self.c_fc_bias = nn.Parameter(torch.zeros(spec.intermediate_size, dtype=dtype, device=device),
                                      requires_grad=False)
        self.mlp_proj = Linear(spec.intermediate_size, h, bias=True, dtype=dtype, device=device)

    def forward(self, hidden, residual, meta: AttnMetadata, k_cache, v_cache, cos_sin=None):
        T = hidden.shape[0]
        first = residual is None
        if first:
            residual = hidden  # never modified in place (see LlamaDecoderLayer.forward)
            normed, _ = self.ln_1(hidden)
        else:
            normed, residual = self.ln_1(hidden, residual)
        qkv = self.c_attn(normed)
        q, q_sink = ops.rope_cache(qkv, meta.positions, meta.slot_mapping, None, self.num_heads,
                                   self.num_heads, self.head_dim, k_cache, v_cache,
                                   window=meta.window, want_sink=meta.want_sink,
                                   k_scale=meta.k_scale, v_scale=meta.v_scale)
        if meta.is_decode:
            o = ops.attn_decode(q, q_sink, k_cache, v_cache, meta.block_tables, meta.seq_lens,
                                self.scale, meta.n_sink, meta.sink_pad, meta.ring, meta.window,
                                num_splits=meta.num_splits, workspace=meta.workspace,
                                k_scale=meta.k_scale, v_scale=meta.v_scale)
        else:
            o = ops.attn_prefill(q, q_sink, k_cache, v_cache, meta.block_tables, meta.seq_lens,
                                 meta.q_start, meta.max_q, self.scale, meta.n_sink, meta.sink_pad,
                                 meta.ring, meta.window, k_scale=meta.k_scale,
                                 v_scale=meta.v_scale, tile_map=meta.tile_map)
        attn = self.attn_proj(o.view(T, -1))
        normed, residual = self.ln_2(attn, residual,
                                     residual_out=torch.empty_like(residual) if first else None)
        act = ops.gelu_bias(self.c_fc(normed), self.c_fc_bias)
        return self.mlp_proj(act), residual

    def load_hf_state_dict(self, sd: dict) -> None:
        """HF GPT-2 layer keys (relative to ``h.{i}.``); Conv1D weights are [in, out]."""
        dt = self.ln_1.weight.dtype
        with torch.no_grad():
            self.ln_1.weight.copy_(sd["ln_1.weight"].to(dt))
            self.ln_1.bias.copy_(sd["ln_1.bias"].to(dt))
            self.c_attn.weight.copy_(sd["attn.c_attn.weight"].t().to(dt))
            self.c_attn.bias.copy_(sd["attn.c_attn.bias"].to(dt))
            self.attn_proj.weight.copy_(sd["attn.c_proj.weight"].t().to(dt))
            self.attn_proj.bias.copy_(sd["attn.c_proj.bias"].to(dt))
            self.ln_2.weight.copy_(sd["ln_2.weight"].to(dt))
            self.ln_2.bias.copy_(sd["ln_2.bias"].to(dt))
            self.c_fc.weight.copy_(sd["mlp.c_fc.weight"].t().to(dt))
            self.c_fc_bias.copy_(sd["mlp.c_fc.bias"].to(dt))
            self.mlp_proj.weight.copy_(sd["mlp.c_proj.weight"].t().to(dt))
            self.mlp_proj.bias.copy_(sd["mlp.c_proj.bias"].to(dt))

    def hf_state_dict(self) -> dict:
        return {
            "ln_1.weight": self.ln_1.weight, "ln_1.bias": self.ln_1.bias,
            "attn.c_attn.weight": self.c_attn.weight.t(), "attn.c_attn.bias": self.c_attn.bias,
            "attn.c_proj.weight": self.attn_proj.weight.t(), "attn.c_proj.bias": self.attn_proj.bias,
            "ln_2.weight": self.ln_2.weight, "ln_2.bias": self.ln_2.bias,
            "mlp.c_fc.weight": self.c_fc.weight.t(), "mlp.c_fc.bias": self.c_fc_bias,
            "mlp.c_proj.weight": self.mlp_proj.weight.t(), "mlp.c_proj.bias": self.mlp_proj.bias,
        }


class GPT2Block(nn.Module):
    """Layer-range stage of GPT-2 (same role as :class:`LlamaBlock`)."""

    def __init__(self, config, layer_ids: Sequence[int], device=None, dtype=torch.bfloat16):
        super().__init__()
        spec = resolve_model(config) if not isinstance(config, ModelSpec) else config
        if spec.arch != "gpt2":
            raise ValueError("GPT2Block needs a gpt2 spec")
        self.config = spec
        self.layer_ids: List[int] = list(layer_ids)
        self.layers = nn.ModuleList(GPT2Layer(spec, i, device, dtype) for i in self.layer_ids)
        self.register_buffer("_dev", torch.empty(0, device=device), persistent=False)
        self.cos_sin = None

    @property
    def device(self):
        return self._dev.device

    def init_random(self, seed: int = 0, std: float = 0.02) -> "GPT2Block":
        for layer in self.layers:
            for name, p in layer.named_parameters():
                if name.startswith("ln_") and name.endswith("weight"):
                    p.data.fill_(1.0)
                elif "bias" in name:
                    p.data.zero_()
                else:
                    seeded_normal_(p.data, param_seed(seed, layer.layer_idx, name), std)
        return self

    def quantize_int8(self, threshold: float = 6.0) -> "GPT2Block":
        for layer in self.layers:
            for lin in (layer.c_attn, layer.attn_proj, layer.c_fc, layer.mlp_proj):
                lin.quantize_int8(threshold)
        return self

    def quantize_fp8(self) -> "GPT2Block":
        for layer in self.layers:
            for lin in (layer.c_attn, layer.attn_proj, layer.c_fc, layer.mlp_proj):
                lin.quantize_fp8()
        return self

    def forward_tokens(self, hidden, meta, pool, residual=None, layer_offset: int = 0,
                       collect: Optional[list] = None):
        for i, layer in enumerate(self.layers):
            if collect is not None:
                collect.append(hidden if residual is None else ops.add(hidden, residual))
            k, v = pool.layer(layer_offset + i)
            hidden, residual = layer(hidden, residual, meta, k, v)
        return hidden, residual
