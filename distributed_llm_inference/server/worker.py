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


class WorkerMoving(RuntimeError):
    """The worker is loading another layer range (swarm rebalancing): no new sessions now."""


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
        # set for the whole of a move (load + swap): forwards that would open a session are
        # refused (WorkerMoving -> HTTP 409), so nothing opened meanwhile is dropped by the swap
        self.moving = False
        self._inflight = 0   # submitted tasks not yet finished (a move also waits for these)

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

    def move_to(self, start: int, end: int, require_idle: bool = False) -> bool:
        """Serve layers ``[start, end)`` instead (swarm rebalancing, server/registry.py
        ``rebalance_target``): the new blocks are loaded while the old ones keep serving, then
        swapped in; the old pools finish what was submitted to them and stop.  Sessions open on
        the old range lose their KV - so while the move runs no new session is admitted
        (:class:`WorkerMoving`), and with ``require_idle`` the move is abandoned (False) if a
        session still holds KV when the swap would happen (checked under the swap lock, so no
        forward can slip in between).  A client whose chain still points here gets 409 and
        fails over (server/block_server.py)."""
        if not (0 <= start < end <= self.spec.num_layers):
            raise ValueError(f"bad block range [{start}, {end})")
        with self._swap:
            if require_idle and not self._idle():
                return False
            self.moving = True
        try:
            block_ids, blocks = self._load_range(start, end)
            if self._running:
                for be in blocks.values():
                    be.inference_pool.start()
            with self._swap:
                if require_idle and not self._idle():
                    abandon, old = blocks, None
                else:
                    abandon, old = None, self.blocks
                    self.block_ids, self.blocks = block_ids, blocks
                    self.start, self.end = start, end
        finally:
            self.moving = False
        if abandon is not None:
            for be in abandon.values():
                be.shutdown()
            log.info("move to [%d, %d) abandoned: sessions opened meanwhile", start, end)
            return False
        for be in old.values():
            be.shutdown()
        log.info("worker now serves layers [%d, %d)", start, end)
        return True

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

    def _submit(self, blocks: Dict[str, InferenceBackend], block_id: str, generation_id: str,
                hidden: torch.Tensor, kw: dict):
        with self._swap:
            if self.moving and not any(generation_id in be.cache._sessions
                                       for be in blocks.values() if be.cache is not None):
                raise WorkerMoving(f"moving from layers [{self.start}, {self.end}): no new "
                                   "sessions")
            fut = blocks[block_id].submit(hidden, generation_id=generation_id, **kw)
            self._inflight += 1
        fut.add_done_callback(self._task_done)
        return fut

    def _task_done(self, _fut) -> None:
        with self._swap:
            self._inflight -= 1

    def _idle(self) -> bool:
        """No session holds KV and no task is queued or running (call under ``_swap``)."""
        return self._inflight == 0 and not self._sessions_of(self.blocks)

    def forward(self, block_id: str, generation_id: str, hidden: torch.Tensor, **kw):
        """One block.  ``kw``: the reference stage API's ``attention_mask`` / ``position_ids`` /
        ``output_hidden_states`` (reference models/llama/model.py:25-33).  Returns the hidden
        states, or ``(hidden, all_hidden_states)`` with ``output_hidden_states``."""
        res = self._submit(self.blocks, block_id, generation_id, hidden, kw).result()
        if kw.get("output_hidden_states"):
            return res[0], tuple(res[1])
        return res[0]

    def forward_range(self, generation_id: str, hidden: torch.Tensor, **kw):
        """Run every block of this worker in order (the whole stage); with
        ``output_hidden_states`` the per-layer inputs of every block and the final output.  The
        walk uses ONE snapshot of the blocks: a move that swaps them meanwhile cannot hand it a
        same-named block of the new range (which holds no KV for the session)."""
        want = bool(kw.get("output_hidden_states"))
        with self._swap:
            block_ids, blocks = list(self.block_ids), self.blocks
        hs: list = []
        for b in block_ids:
            res = self._submit(blocks, b["block_id"], generation_id, hidden, kw).result()
            out = (res[0], tuple(res[1])) if want else res[0]
            if want:
                out, blk_hs = out
                hs = hs[:-1] + list(blk_hs)   # a block's first entry is the previous output
            hidden = out
        return (hidden, tuple(hs)) if want else hidden

    @staticmethod
    def _sessions_of(blocks: Dict[str, InferenceBackend]) -> List[str]:
        ids = set()
        for be in blocks.values():
            if be.cache is not None:
                ids.update(k for k in be.cache._sessions if k != "__schema__")
        return sorted(ids)

    def sessions(self) -> List[str]:
        """The generation ids holding KV on any block of this worker."""
        return self._sessions_of(self.blocks)

    def close_session(self, generation_id: str) -> None:
        for be in self.blocks.values():
            be.close_session(generation_id)
