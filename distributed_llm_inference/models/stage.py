"""A complete pipeline stage: [embedding] + layer range + [final norm, LM head].

This is the per-GPU model shard the runtime executes: stage 0 owns the
embedding, the last stage owns the final norm and the LM head, and every stage owns a contiguous
``[start, end)`` layer range (the reference worker's ``block_index_start/end``, server/worker.py:13-14).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..config import ModelSpec, resolve_model
from .common import AttnMetadata
from .embed_head import Embedding, LMHead
from .gpt2.model import GPT2Block
from .llama.cache import KVPool
from .llama.model import LlamaBlock


def apply_quantization(block, mode, threshold: float = 6.0):
    """Quantise a Llama / GPT-2 block in place: ``mode`` False / None / "none" (bf16), True /
    "fp8" (e4m3 weights, per-channel scales) or "int8" (LLM.int8, outlier ``threshold``)."""
    if mode in (False, None, "none", "bf16"):
        return block
    if mode is True or mode == "fp8":
        return block.quantize_fp8()
    if mode == "int8":
        return block.quantize_int8(threshold)
    raise ValueError(f"unknown quantisation mode {mode!r} (expected fp8 / int8)")


def make_block(spec: ModelSpec, layer_ids, device=None, dtype=torch.bfloat16):
    if spec.arch == "llama":
        return LlamaBlock(spec, layer_ids, device=device, dtype=dtype)
    if spec.arch == "gpt2":
        return GPT2Block(spec, layer_ids, device=device, dtype=dtype)
    raise ValueError(f"unsupported arch {spec.arch}")


class CausalLMStage(nn.Module):
    def __init__(self, config, start: int, end: int, device=None, dtype=torch.bfloat16,
                 has_embed: Optional[bool] = None, has_head: Optional[bool] = None):
        super().__init__()
        spec = resolve_model(config)
        self.spec = spec
        self.start, self.end = int(start), int(end)
        if not (0 <= self.start < self.end <= spec.num_layers):
            raise ValueError(f"bad layer range [{start}, {end}) for {spec.num_layers} layers")
        self.has_embed = (self.start == 0) if has_embed is None else has_embed
        self.has_head = (self.end == spec.num_layers) if has_head is None else has_head
        self.block = make_block(spec, range(self.start, self.end), device, dtype)
        self.embed = Embedding(spec, device, dtype) if (self.has_embed or (
            self.has_head and spec.tie_word_embeddings)) else None
        self.head = (LMHead(spec, device, dtype, tied=self.embed if spec.tie_word_embeddings else None)
                     if self.has_head else None)

    @property
    def device(self) -> torch.device:
        return self.block.device

    @property
    def num_layers(self) -> int:
        return self.end - self.start

    def init_random(self, seed: int = 0) -> "CausalLMStage":
        self.block.init_random(seed)
        if self.embed is not None:
            self.embed.init_random(seed)
        if self.head is not None:
            self.head.init_random(seed)
        return self

    def quantize_fp8(self) -> "CausalLMStage":
        self.block.quantize_fp8()
        return self

    def quantize_int8(self, threshold: float = 6.0) -> "CausalLMStage":
        self.block.quantize_int8(threshold)
        return self

    def quantize(self, mode, threshold: float = 6.0) -> "CausalLMStage":
        """``mode``: False / None / "none"; True / "fp8" (e4m3, the MI355X default); "int8"
        (LLM.int8 with outlier ``threshold``)."""
        apply_quantization(self.block, mode, threshold)
        return self

    def make_pool(self, num_blocks: int, block_size: int = 64, window_length: int = 0,
                  num_sink_tokens: int = 0, max_chunk: int = 512,
                  kv_dtype: torch.dtype = torch.bfloat16, k_scale: float = 1.0,
                  v_scale: float = 1.0) -> KVPool:
        return KVPool(self.spec, self.num_layers, num_blocks, block_size, self.device,
                      kv_dtype, window_length, num_sink_tokens, max_chunk, k_scale, v_scale)

    def forward(self, inputs: torch.Tensor, meta: AttnMetadata, pool: KVPool,
                project: bool = True) -> torch.Tensor:
        """``inputs``: token ids [T] (stage 0) or hidden states [T, H].  Returns hidden [T, H]
        (non-last stage) or logits [R, V] for the rows in ``meta.logits_rows`` (last stage);
        ``project=False`` on the last stage stops after the final norm (normed hidden [R, H]) for a
        vocabulary projection that runs on another rank (runtime/head.py)."""
        if self.has_embed:
            hidden = self.embed(inputs, meta.positions)
        else:
            hidden = inputs
        out, res = self.block.forward_tokens(hidden, meta, pool)
        if self.has_head:
            if not project:
                return self.head.norm(out, res, meta.logits_rows)
            return self.head(out, res, meta.logits_rows)
        return ops.add(out, res)
