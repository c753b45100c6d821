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
            dev = self._device()
            inputs = tuple(x.to(dev, torch.bfloat16) if torch.is_tensor(x) else x for x in inputs)
            kw = {k: v.to(dev) if torch.is_tensor(v) else v for k, v in kw.items()}
            return self.module(generation_id, *inputs, past_key_value=self.cache, **kw)
        return self.module(*inputs, **kw)

    @torch.inference_mode()
    def _process_tasks(self, tasks: List[Task]) -> List[Any]:
        """Pack every pending session step into one varlen forward through the block.

        Several steps of one session in the same batch run in submission order: the k-th step of
        every session goes into the k-th packed forward ("wave").  A step that carries the
        reference stage API's extra arguments (``attention_mask``, ``position_ids``,
        ``output_hidden_states``: task meta ``kwargs``) runs alone through ``LlamaBlock.forward``
        at its place in submission order; the plain steps around it are packed as usual."""
        results: List[Any] = [None] * len(tasks)
        seg: List[int] = []
        for i, t in enumerate(tasks + [None]):
            if t is not None and not t.meta.get("kwargs"):
                seg.append(i)
                continue
            if seg:
                for j, r in zip(seg, self._process_packed([tasks[j] for j in seg])):
                    results[j] = r
                seg = []
            if t is not None:
                try:
                    results[i] = self.forward(*t.args, generation_id=t.meta.get("generation_id"),
                                              **t.meta["kwargs"])
                except Exception as e:  # noqa: BLE001 - this task's waiter only
                    results[i] = e
        return results

    def _process_packed(self, tasks: List[Task]) -> List[Any]:
        blk = self.module
        self.cache.bind(blk.config, blk.layer_ids, self._device(), torch.bfloat16)
        results: List[Any] = [None] * len(tasks)
        waves: List[List[int]] = []
        count: Dict[Any, int] = {}
        for i, t in enumerate(tasks):
            k = count.get(t.meta.get("generation_id"), 0)
            count[t.meta.get("generation_id")] = k + 1
            if k == len(waves):
                waves.append([])
            waves[k].append(i)
        for k, wave in enumerate(waves):
            # a later step of a session whose earlier step failed in this batch fails too
            failed = {tasks[i].meta.get("generation_id") for w in waves[:k] for i in w
                      if isinstance(results[i], BaseException)}
            for i in wave:
                if tasks[i].meta.get("generation_id") in failed:
                    results[i] = RuntimeError("an earlier step of this session failed")
            wave = [i for i in wave if results[i] is None]
            try:
                self._run_wave(tasks, wave, results)
            except Exception as e:  # noqa: BLE001 - the whole wave failed (reservations undone)
                for i in wave:
                    if results[i] is None:
                        results[i] = e
        return results

    def _run_wave(self, tasks: List[Task], wave: List[int], results: List[Any]) -> None:
        blk, cache, dev = self.module, self.cache, self._device()
        # Each task reserves its rows all-or-nothing: a task that does not fit (or is malformed)
        # fails alone and leaves its session untouched; the tasks that fit still run.  If the
        # packed forward itself raises, every reservation of the wave is rolled back.
        sids, qlens, xs, spans, done = [], [], [], [], []
        for i in wave:
            t = tasks[i]
            try:
                (h,) = t.args[:1]
                gid = t.meta["generation_id"]
                if gid is None:
                    raise ValueError("block backends need a generation_id")
                if h.dim() != 3:
                    raise ValueError("hidden_states must be [batch, seq, hidden]")
                B, T, H = h.shape
                # to the device BEFORE reserving: a failed copy (OOM, bad shape) leaves nothing
                # reserved
                x = h.reshape(B * T, H).to(dev, torch.bfloat16)
                rows = cache.session_rows(gid, B)
                cache.reserve_rows(gid, rows, [T] * B, T)
            except Exception as e:  # noqa: BLE001 - delivered to this task's waiter only
                results[i] = e
                continue
            done.append((gid, rows, T))
            spans.append((i, B, T))
            sids += rows
            qlens += [T] * B
            xs.append(x)
        if not spans:
            return
        try:
            meta = cache.pool.build_metadata(sids, qlens)
            out, res = blk.forward_tokens(torch.cat(xs, 0), meta, cache.pool)
            y = out + res
        except BaseException:
            for gid, rows, T in reversed(done):
                cache.unreserve_rows(gid, rows, [T] * len(rows), T)
            raise
        off = 0
        for (i, B, T) in spans:
            results[i] = (y[off: off + B * T].view(B, T, -1),)
            off += B * T

    def submit(self, *inputs, generation_id: Optional[str] = None, **kwargs):
        """Queue one step; ``kwargs``: the reference stage API's ``attention_mask`` /
        ``position_ids`` / ``output_hidden_states`` (run unpacked, in order)."""
        kwargs = {k: v for k, v in kwargs.items() if v is not None and v is not False}
        return self.inference_pool.submit_task(*inputs, generation_id=generation_id,
                                               kwargs=kwargs or None)

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
