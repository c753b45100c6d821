"""``LlamaBlock`` — one pipeline stage: an arbitrary set of decoder layers.

Reference: /root/reference/distributed_llm_inference/models/llama/model.py:16-76 (``LlamaBlock(config,
layer_ids)``, ``forward(generation_id, hidden_states, attention_mask=None, position_ids=None,
past_key_value=None, output_hidden_states=None, cache_position=None)``).  The public signature and
return convention (a tuple ``(hidden_states[, all_hidden_states])``) are kept; the intended
semantics replace the reference's bugs:
  * B1/B2 — RoPE cos/sin are fp32 tables (llama3 scaling included), applied per token;
  * B4/B5 — positions default to ``past_len + arange(T)`` per session row;
  * B6    — attention is always causal (in-kernel, from sequence lengths);
  * B7-B9 — standard residual stream and ``config.rms_norm_eps``.

Two entry points:
  * :meth:`LlamaBlock.forward` — the reference-compatible, session-keyed API ([B, T, H] tensors,
    ``PartialLlamaSinkCache``), used directly by library users and by the server backend;
  * :meth:`LlamaBlock.forward_tokens` — the runtime's fast path on packed varlen tokens [T, H]
    with precomputed :class:`AttnMetadata`; this is what the pipeline executor graph-captures.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ... import ops
from ...config import ModelSpec, resolve_model
from ...ops.reference import build_cos_sin
from ..common import AttnMetadata, param_seed, seeded_normal_
from .cache import KVPool, PartialLlamaSinkCache
from .modules import LlamaDecoderLayer


class LlamaBlock(nn.Module):
    def __init__(self, config, layer_ids: Sequence[int], device=None, dtype=torch.bfloat16,
                 max_position: Optional[int] = None):
        super().__init__()
        spec = resolve_model(config) if not isinstance(config, ModelSpec) else config
        self.config = spec
        self.layer_ids: List[int] = [int(i) for i in layer_ids]
        if any(i < 0 or i >= spec.num_layers for i in self.layer_ids):
            raise ValueError(f"layer ids {self.layer_ids} out of range for {spec.num_layers} layers")
        self.padding_idx = spec.pad_token_id
        self.vocab_size = spec.vocab_size
        self.layers = nn.ModuleList(LlamaDecoderLayer(spec, i, device, dtype) for i in self.layer_ids)
        maxp = int(max_position or max(spec.max_position_embeddings, 8192))
        self.register_buffer("cos_sin", build_cos_sin(spec.head_dim, maxp, spec.rope_theta,
                                                      spec.rope_scaling_dict, device=device,
                                                      max_position_embeddings=spec.max_position_embeddings),
                             persistent=False)

    # ------------------------------------------------------------------ construction helpers
    @property
    def device(self) -> torch.device:
        return self.cos_sin.device

    def init_random(self, seed: int = 0, std: float = 0.02) -> "LlamaBlock":
        """Deterministic random init (per global layer index, so any stage split of the same seed
        holds the same weights as the unsplit model)."""
        for layer in self.layers:
            for name, p in layer.named_parameters():
                if name.endswith("layernorm.weight"):
                    p.data.fill_(1.0)
                elif name.endswith("bias"):
                    p.data.zero_()
                else:
                    seeded_normal_(p.data, param_seed(seed, layer.layer_idx, name), std)
        return self

    def set_fused_swiglu(self, on: bool = True) -> "LlamaBlock":
        """Reorder every gate|up weight for the tile GEMM's fused SwiGLU epilogue (GPU decode)."""
        for layer in self.layers:
            layer.mlp.set_fused_swiglu(on)
        return self

    def quantize_int8(self, threshold: float = 6.0) -> "LlamaBlock":
        """LLM.int8 weights for every projection (reference convert_to_optimized_block)."""
        self.set_fused_swiglu(False)
        for layer in self.layers:
            for lin in (layer.self_attn.qkv_proj, layer.self_attn.o_proj, layer.mlp.gate_up_proj,
                        layer.mlp.down_proj):
                lin.quantize_int8(threshold)
        return self

    def quantize_fp8(self) -> "LlamaBlock":
        self.set_fused_swiglu(False)
        for layer in self.layers:
            for lin in (layer.self_attn.qkv_proj, layer.self_attn.o_proj, layer.mlp.gate_up_proj,
                        layer.mlp.down_proj):
                lin.quantize_fp8()
        return self

    def new_cache(self, window_length: int = 0, num_sink_tokens: int = 0, num_blocks: int = 256,
                  block_size: int = 64) -> PartialLlamaSinkCache:
        c = PartialLlamaSinkCache(window_length, num_sink_tokens, num_blocks, block_size)
        return c.bind(self.config, self.layer_ids, self.device, torch.bfloat16)

    # ------------------------------------------------------------------ fast path
    def forward_tokens(self, hidden: torch.Tensor, meta: AttnMetadata, pool: KVPool,
                       residual: Optional[torch.Tensor] = None, layer_offset: int = 0,
                       collect: Optional[list] = None,
                       cos_sin: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Run the local layers on packed tokens ``hidden [T, H]``.  Returns ``(out, residual)``;
        the stage output hidden state is ``out + residual``.  ``cos_sin``: this call's RoPE table
        (dynamic NTK scaling) instead of the block's."""
        cos_sin = self.cos_sin if cos_sin is None else cos_sin
        last = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            if collect is not None:
                collect.append(hidden if residual is None else ops.add(hidden, residual))
            k, v = pool.layer(layer_offset + i)
            # between layers the down projection's split-K partials go straight into the next
            # input RMSNorm; the block's output is always materialised
            hidden, residual = layer(hidden, residual, meta, k, v, cos_sin,
                                     defer_out=collect is None and i < last)
        return hidden, residual

    def _dynamic_table(self, meta: AttnMetadata) -> Optional[torch.Tensor]:
        """The RoPE table of one forward under dynamic NTK scaling: rebuilt with the rescaled
        base when the call's longest position + 1 exceeds max_position_embeddings (HF
        recomputes inv_freq from max(position_ids) + 1 the same way); None otherwise."""
        spec = self.config
        if spec.rope_type != "dynamic" or meta.positions.numel() == 0:
            return None
        seq_len = int(meta.positions.max()) + 1
        if seq_len <= spec.max_position_embeddings:
            return None
        return build_cos_sin(spec.head_dim, max(seq_len, self.cos_sin.shape[0]), spec.rope_theta,
                             spec.rope_scaling_dict, device=self.cos_sin.device,
                             max_position_embeddings=spec.max_position_embeddings,
                             seq_len=seq_len)

    # ------------------------------------------------------------------ reference API
    def forward(self, generation_id: str, hidden_states: torch.Tensor,
                attention_mask: Optional[torch.Tensor] = None,
                position_ids: Optional[torch.LongTensor] = None,
                past_key_value: Optional[PartialLlamaSinkCache] = None,
                output_hidden_states: Optional[bool] = None,
                cache_position: Optional[torch.LongTensor] = None):
        """Run this block for session ``generation_id`` on ``hidden_states [B, T, H]``.

        ``attention_mask`` (optional, ``[B, T]`` or ``[B, past+T]``, 1 = real token) drops padded
        positions (their output rows are zero).  ``position_ids``/``cache_position`` override the
        default RoPE positions ``past_len + arange``.  Without ``past_key_value`` the call is
        stateless (causal attention within the chunk only).  ``output_hidden_states=None`` takes
        the config's ``output_hidden_states`` (reference model.py:35-37); the states are the L
        layer inputs and the output (L+1 tensors), zeros for padded rows - all zeros when every
        row is padding.  With ``rope_type: dynamic`` a call whose longest position exceeds
        ``max_position_embeddings`` rotates with the NTK-rescaled base for that length (HF
        ``dynamic_rope_update``).
        """
        if output_hidden_states is None:
            output_hidden_states = bool(getattr(self.config, "output_hidden_states", False))
        if hidden_states.dim() != 3:
            raise ValueError("hidden_states must be [batch, seq, hidden]")
        B, T, H = hidden_states.shape
        dev = hidden_states.device
        cache = past_key_value
        if cache is None:
            cache = PartialLlamaSinkCache(0, 0, num_blocks=max(1, B * ((T + 63) // 64)),
                                          block_size=64)
        cache.bind(self.config, self.layer_ids, dev, torch.bfloat16)
        if cache.layer_ids != self.layer_ids:
            raise ValueError("cache is bound to a different layer set")

        # which new tokens are real (padding support)
        custom = None
        if attention_mask is not None and attention_mask.dim() == 4:
            # reference model.py:115-119: a 4-D mask comes pre-inverted (additive, max == 0) and
            # is used as-is, sliced to the key length (modules.py:92-94); every new token is real
            if attention_mask.shape[0] != B or attention_mask.shape[2] != T or \
                    attention_mask.shape[1] not in (1, self.config.num_heads):
                raise ValueError(f"4-D attention_mask must be [batch={B}, 1 or num_heads, "
                                 f"seq={T}, key_len], got {tuple(attention_mask.shape)}")
            if attention_mask.max() != 0:
                raise ValueError("Custom 4D attention mask should be passed in inverted form "
                                 "with max==0")
            if cache.window_length:
                raise ValueError("4-D attention masks need a full (non-windowed) cache")
            custom = attention_mask
            am = torch.ones(B, T, dtype=torch.bool, device=dev)
        elif attention_mask is not None:
            if attention_mask.dim() != 2:
                raise ValueError("attention_mask must be [batch, seq] (1 = token) or a pre-inverted "
                                 f"4-D mask, got {attention_mask.dim()} dims")
            am = attention_mask[:, -T:].to(torch.bool)
        else:
            am = torch.ones(B, T, dtype=torch.bool, device=dev)
        q_lens = [int(q) for q in am.sum(-1).tolist()]
        # explicit positions override the default past_len + arange
        pos_src = position_ids if position_ids is not None else (
            cache_position.unsqueeze(0).expand(B, -1) if cache_position is not None else None)
        if pos_src is not None and (pos_src.dim() != 2 or pos_src.shape[0] not in (1, B)
                                    or pos_src.shape[1] < T):
            raise ValueError(f"position_ids must be [batch={B} or 1, >= {T}], "
                             f"got {tuple(pos_src.shape)}")
        m = cache.pool.manager
        # Everything that can be checked is checked before the session grows: a rejected call
        # leaves the cache exactly as it was.
        prev = cache._sessions.get(generation_id)
        if prev is not None and len(prev) != B:
            raise ValueError(f"session {generation_id!r} has batch {len(prev)}, got {B}")
        if custom is not None:
            past = [m.length(r) if m.has_sequence(r) else 0 for r in prev] if prev else [0] * B
            L_max = max([p + q for p, q in zip(past, q_lens) if q > 0] + [0])
            if custom.shape[-1] < L_max:
                raise ValueError(f"4-D attention_mask key length {custom.shape[-1]} < {L_max} "
                                 "cached + new tokens")
        rows = cache.session_rows(generation_id, B)
        cache.reserve_rows(generation_id, rows, q_lens, T)   # all or nothing, MemoryError
        try:
            keep = [b for b in range(B) if q_lens[b] > 0]
            out_full = torch.zeros_like(hidden_states)
            if not keep:   # all padding: nothing cached; L + 1 zero states like a real call
                if not output_hidden_states:
                    return (out_full,)
                return out_full, tuple(torch.zeros_like(hidden_states)
                                       for _ in range(len(self.layers) + 1))
            sids = [rows[b] for b in keep]
            qls = [q_lens[b] for b in keep]
            meta = cache.pool.build_metadata(sids, qls)
            if custom is not None:
                meta.custom_mask = (custom if len(keep) == B else custom[keep]).to(dev)
            if pos_src is not None:
                # rows with no real token contribute nothing to am, so the packing order matches
                meta.positions = pos_src.to(dev).expand(B, -1)[:, -T:][am].to(
                    torch.int32).contiguous()
            x = hidden_states[am].to(torch.bfloat16).contiguous()  # [T_total, H] packed
            collect = [] if output_hidden_states else None
            out, res = self.forward_tokens(x, meta, cache.pool, collect=collect,
                                           cos_sin=self._dynamic_table(meta))
            y = ops.add(out, res)
        except BaseException:
            cache.unreserve_rows(generation_id, rows, q_lens, T)
            raise
        out_full[am] = y.to(out_full.dtype)
        if output_hidden_states:
            all_hs = []
            for h in collect + [y]:
                full = torch.zeros_like(hidden_states)
                full[am] = h.to(full.dtype)
                all_hs.append(full)
            return out_full, tuple(all_hs)
        return (out_full,)
