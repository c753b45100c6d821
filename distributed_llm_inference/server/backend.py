"""Inference-only module backend with tensor schemas and a batching pool.

Reference: ``InferenceBackend(ModuleBackend)`` (/root/reference/distributed_llm_inference/server/
backend.py:11-51): schemas, output-schema inference by a dummy forward, one TaskPool named
``{name}_inference``, backward disabled.  Fixes: ``get_pools()`` returns a tuple;
session metadata (``generation_id``) travels out-of-band next to the tensors instead of being
forced through a tensor schema (B13).

For a layer-range module (:class:`LlamaBlock` / :class:`GPT2Block`) the pool does real
continuous batching across sessions: the pending tasks of many generation_ids — each
``hidden [b_i, t_i, H]`` with its own cache state — are packed into ONE varlen token batch and
run through the block's fast path (paged attention kernels) in a single forward.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import nn

from ..models.llama.cache import PartialLlamaSinkCache
from .task_pool import Task, TaskPool

log = logging.getLogger(__name__)

DUMMY_BATCH_SIZE = 3


@dataclass(frozen=True)
class BatchTensorDescriptor:
    """Shape (without the batch dim) + dtype of one tensor argument."""

    shape: Tuple[int, ...]
    dtype: torch.dtype = torch.bfloat16

    def make_zeros(self, batch_size: int, device=None) -> torch.Tensor:
        return torch.zeros((batch_size,) + tuple(self.shape), dtype=self.dtype, device=device)

    @classmethod
    def from_tensor(cls, t: torch.Tensor) -> "BatchTensorDescriptor":
        return cls(tuple(t.shape[1:]), t.dtype)


def _nested_map(fn, x):
    if isinstance(x, (tuple, list)):
        return type(x)(_nested_map(fn, y) for y in x)
    if isinstance(x, dict):
        return {k: _nested_map(fn, v) for k, v in x.items()}
    return fn(x)


class InferenceBackend:
    def __init__(self, name: str, module: nn.Module, *,
                 args_schema: Optional[Tuple[BatchTensorDescriptor, ...]] = None,
                 kwargs_schema: Optional[Dict[str, BatchTensorDescriptor]] = None,
                 outputs_schema=None, max_batch_size: int = 256, cache: Optional[PartialLlamaSinkCache] = None,
                 pool_timeout: float = 0.002, **kwargs):
        self.name, self.module, self.optimizer, self.scheduler = name, module, None, None
        self.args_schema = args_schema = tuple(args_schema or ())
        self.kwargs_schema = kwargs_schema = dict(kwargs_schema or {})
        if not (args_schema or kwargs_schema):
            raise ValueError("Module must take at least one positional or keyword input. "
                             "Did you forget to provide args_schema/kwargs_schema?")
        self.is_block = hasattr(module, "forward_tokens") and hasattr(module, "layer_ids")
        self.cache = cache
        if self.is_block and self.cache is None:
            self.cache = PartialLlamaSinkCache(0, 0, num_blocks=kwargs.pop("num_blocks", 512))
        dev = self._device()
        if outputs_schema is None:
            dummy_args = tuple(s.make_zeros(DUMMY_BATCH_SIZE, dev) for s in args_schema)
            dummy_kwargs = {k: s.make_zeros(DUMMY_BATCH_SIZE, dev) for k, s in kwargs_schema.items()}
            with torch.inference_mode():
                if self.is_block:
                    out = module("__schema__", *dummy_args, past_key_value=self.cache,
                                 **dummy_kwargs)
                    self.cache.close_session("__schema__")
                else:
                    out = module(*dummy_args, **dummy_kwargs)
            outputs_schema = _nested_map(BatchTensorDescriptor.from_tensor, out)
        self.forward_schema = (self.args_schema, self.kwargs_schema)
        self.outputs_schema = outputs_schema
        self.backward_schema = (self.forward_schema, self.outputs_schema)
        self.grad_inputs_schema = self.forward_schema
        self.inference_pool = TaskPool(self._process_tasks if self.is_block else self.forward,
                                       max_batch_size=max_batch_size, name=f"{name}_inference",
                                       timeout=pool_timeout, collate=not self.is_block)

    def _device(self):
        for p in self.module.parameters():
            return p.device
        return torch.device("cpu")

    # ------------------------------------------------------------------ compute
    @torch.inference_mode()
    def forward(self, *inputs: torch.Tensor, generation_id: Optional[str] = None, **kw):
        if self.is_block:
            if generation_id is None:
                raise ValueError("block backends need a generation_id")
            return self.module(generation_id, *inputs, past_key_value=self.cache, **kw)
        return self.module(*inputs, **kw)

    @torch.inference_mode()
    def _process_tasks(self, tasks: List[Task]) -> List[Any]:
        """Pack every pending session step into one varlen forward through the block."""
        blk = self.module
        cache = self.cache
        dev = self._device()
        cache.bind(blk.config, blk.layer_ids, dev, torch.bfloat16)
        m = cache.pool.manager
        sids, qlens, xs, spans = [], [], [], []
        for t in tasks:
            (h,) = t.args[:1]
            gid = t.meta["generation_id"]
            B, T, H = h.shape
            rows = cache.session_rows(gid, B)
            for r in rows:
                m.append(r, T)
            cache._seen_tokens[gid] += T
            spans.append((len(sids), B, T))
            sids += rows
            qlens += [T] * B
            xs.append(h.reshape(B * T, H).to(dev, torch.bfloat16))
        meta = cache.pool.build_metadata(sids, qlens)
        out, res = blk.forward_tokens(torch.cat(xs, 0), meta, cache.pool)
        y = out + res
        results, off = [], 0
        for (_, B, T) in spans:
            results.append((y[off: off + B * T].view(B, T, -1),))
            off += B * T
        return results

    def submit(self, *inputs, generation_id: Optional[str] = None):
        return self.inference_pool.submit_task(*inputs, generation_id=generation_id)

    def close_session(self, generation_id: str) -> None:
        if self.cache is not None:
            self.cache.close_session(generation_id)

    # ------------------------------------------------------------------ training API (disabled)
    def backward(self, *inputs: torch.Tensor):
        raise NotImplementedError("InferenceBackend does not support backward pass")

    def on_backward(self, batch_size: int) -> None:
        raise NotImplementedError("InferenceBackend does not support backward pass")

    def get_pools(self) -> Tuple[TaskPool, ...]:
        return (self.inference_pool,)

    def shutdown(self) -> None:
        self.inference_pool.shutdown()
