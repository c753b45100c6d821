"""Worker holding a contiguous block range.

Reference: ``Block`` TypedDict and ``InferenceWorker(model, block_index_start, block_index_end,
block_)`` (/root/reference/distributed_llm_inference/server/worker.py:4-23), a stub meant to build
``Dict[block_id, TransformerBackend]`` via ``load_block()``.  Implemented: the worker loads (or
random-initialises) the layers ``[start, end)`` on its device, groups them into blocks of
``layers_per_block`` layers (default: the whole range — one MI355X-sized block), wraps each in an
:class:`InferenceBackend` with its own session cache and batching pool, and routes
``forward(block_id, generation_id, hidden)`` / ``forward_range(generation_id, hidden)`` calls.
"""
from __future__ import annotations

import logging
import threading
from typing import Dict, List, Optional, Tuple, TypedDict

import torch

from ..config import resolve_model
from ..models.llama.cache import PartialLlamaSinkCache
from ..utils.model import convert_to_optimized_block, load_block
from .backend import BatchTensorDescriptor, InferenceBackend

log = logging.getLogger(__name__)


class Block(TypedDict):
    block_index: int
    block_id: str


class InferenceWorker:
    def __init__(self, model: str, block_index_start: int, block_index_end: int,
                 layers_per_block: Optional[int] = None, device=None, random_init: bool = True,
                 checkpoint: Optional[str] = None, quantize: bool = False,
                 max_batch_size: int = 64, window_length: int = 0, num_sink_tokens: int = 0,
                 num_blocks: int = 512, seed: int = 0):
        self.model = model
        self.spec = resolve_model(checkpoint or model)
        if not (0 <= block_index_start < block_index_end <= self.spec.num_layers):
            raise ValueError("bad block range")
        self.start, self.end = block_index_start, block_index_end
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
            else torch.device("cpu"))
        self._load_kw = dict(layers_per_block=layers_per_block, checkpoint=checkpoint,
                             random_init=random_init, quantize=quantize,
                             max_batch_size=max_batch_size, window_length=window_length,
                             num_sink_tokens=num_sink_tokens, num_blocks=num_blocks, seed=seed)
        # forward's block lookup + submit and move_to's swap hold this lock: a task is never
        # submitted to a backend whose pool has been told to stop
        self._swap = threading.Lock()
        self.block_ids, self.blocks = self._load_range(block_index_start, block_index_end)
        self._running = False

    def _load_range(self, start: int, end: int) -> Tuple[List[Block], Dict[str, InferenceBackend]]:
        kw = self._load_kw
        n = kw["layers_per_block"] or (end - start)
        block_ids: List[Block] = []
        blocks: Dict[str, InferenceBackend] = {}
        for s in range(start, end, n):
            e = min(end, s + n)
            bid = f"{self.spec.name}.{s}-{e}"
            blk = load_block(kw["checkpoint"] or self.model, list(range(s, e)),
                             use_quantized=False, device=self.device,
                             random_init=kw["checkpoint"] is None and kw["random_init"],
                             seed=kw["seed"])
            if kw["quantize"]:
                blk = convert_to_optimized_block(blk, quantize=True, device=self.device)
            cache = PartialLlamaSinkCache(kw["window_length"], kw["num_sink_tokens"],
                                          num_blocks=kw["num_blocks"])
            be = InferenceBackend(bid, blk,
                                  args_schema=(BatchTensorDescriptor((1, self.spec.hidden_size)),),
                                  max_batch_size=kw["max_batch_size"], cache=cache)
            blocks[bid] = be
            block_ids.append(Block(block_index=s, block_id=bid))
        return block_ids, blocks

    def move_to(self, start: int, end: int) -> None:
        """Serve layers ``[start, end)`` instead (swarm rebalancing, server/registry.py
        ``rebalance_target``): the new blocks are loaded while the old ones keep serving, then
        swapped in; the old pools finish what was submitted to them and stop.  Sessions open on
        the old range lose their KV - the block server moves only when it holds none, and a
        client whose chain still points here gets 409 and fails over (server/block_server.py)."""
        if not (0 <= start < end <= self.spec.num_layers):
            raise ValueError(f"bad block range [{start}, {end})")
        block_ids, blocks = self._load_range(start, end)
        if self._running:
            for be in blocks.values():
                be.inference_pool.start()
        with self._swap:
            old = self.blocks
            self.block_ids, self.blocks = block_ids, blocks
            self.start, self.end = start, end
        for be in old.values():
            be.shutdown()
        log.info("worker now serves layers [%d, %d)", start, end)

    def run(self) -> None:
        for be in self.blocks.values():
            be.inference_pool.start()
        self._running = True

    def shutdown(self) -> None:
        for be in self.blocks.values():
            be.shutdown()
        self._running = False

    def is_healthy(self) -> bool:
        return self._running and all(be.inference_pool.is_alive for be in self.blocks.values())

    def forward(self, block_id: str, generation_id: str, hidden: torch.Tensor, **kw):
        """One block.  ``kw``: the reference stage API's ``attention_mask`` / ``position_ids`` /
        ``output_hidden_states`` (reference models/llama/model.py:25-33).  Returns the hidden
        states, or ``(hidden, all_hidden_states)`` with ``output_hidden_states``."""
        with self._swap:
            fut = self.blocks[block_id].submit(hidden, generation_id=generation_id, **kw)
        res = fut.result()
        if kw.get("output_hidden_states"):
            return res[0], tuple(res[1])
        return res[0]

    def forward_range(self, generation_id: str, hidden: torch.Tensor, **kw):
        """Run every block of this worker in order (the whole stage); with
        ``output_hidden_states`` the per-layer inputs of every block and the final output."""
        want = bool(kw.get("output_hidden_states"))
        hs: list = []
        for b in list(self.block_ids):
            out = self.forward(b["block_id"], generation_id, hidden, **kw)
            if want:
                out, blk_hs = out
                hs = hs[:-1] + list(blk_hs)   # a block's first entry is the previous output
            hidden = out
        return (hidden, tuple(hs)) if want else hidden

    def sessions(self) -> List[str]:
        """The generation ids holding KV on any block of this worker."""
        ids = set()
        for be in self.blocks.values():
            if be.cache is not None:
                ids.update(k for k in be.cache._sessions if k != "__schema__")
        return sorted(ids)

    def close_session(self, generation_id: str) -> None:
        for be in self.blocks.values():
            be.close_session(generation_id)
