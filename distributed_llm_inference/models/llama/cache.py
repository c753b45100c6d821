"""Paged KV cache: one preallocated pool per stage + session-keyed views.

Reference: ``PartialLlamaSinkCache`` (/root/reference/distributed_llm_inference/models/llama/
cache.py:7-135) — a multi-session StreamingLLM cache keyed by ``generation_id`` whose state is
Python dicts of per-layer tensors grown with ``torch.cat`` every token (O(S) copy per token per
layer) and re-rotated on eviction.

MI355X design:
* :class:`KVPool` allocates ONE K tensor ``[L, blocks, nkv, bs, D]`` and ONE transposed V tensor
  ``[L, blocks, nkv, bs/8, D, 8]`` per stage, sized from free HBM (288 GB per MI355X: for Llama-3-70B
  PP=8 that is millions of cached tokens per stage).  Blocks are handed out by the native
  :class:`BlockManager` (csrc/runtime/block_manager.cpp).
* :class:`PartialLlamaSinkCache` keeps the reference's public surface — construction from
  ``(window_length, num_sink_tokens)``, ``get_seq_length(layer_idx, generation_id)``,
  ``update(key, value, layer_idx, cache_kwargs)`` — on top of the pool.  A session
  (``generation_id``) holds B rows, each an independent sequence in the pool.  Eviction is free
  (ring slots are overwritten in place) and no cached key is ever re-rotated: the attention
  kernel scores sink keys with a query rotated at the in-window position instead (see
  csrc/kernels/attention.hip), which yields exactly the relative positions the reference's
  re-rotation produces.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from ...config import ModelSpec
from ..common import AttnMetadata


def _runtime():
    from ... import _runtime  # built by conftest / _build.build_runtime()
    return _runtime


class KVPool:
    """Per-stage paged KV storage for ``num_layers`` local layers."""

    def __init__(self, spec: ModelSpec, num_layers: int, num_blocks: int, block_size: int = 64,
                 device=None, dtype=torch.bfloat16, window_length: int = 0,
                 num_sink_tokens: int = 0, max_chunk: int = 512, k_scale: float = 1.0,
                 v_scale: float = 1.0):
        """``dtype`` bf16, or ``torch.float8_e4m3fn`` for an fp8 cache that stores k / k_scale
        and v / v_scale (half the bytes the decode attention streams, twice the tokens)."""
        if block_size % 32:
            raise ValueError("block_size must be a multiple of 32")
        if dtype not in (torch.bfloat16, torch.float8_e4m3fn):
            raise ValueError(f"unsupported KV cache dtype {dtype}")
        self.dtype = dtype
        self.k_scale, self.v_scale = float(k_scale), float(v_scale)
        self.spec = spec
        self.num_layers = num_layers
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        nkv, D = spec.num_kv_heads, spec.head_dim
        self.k = torch.zeros(num_layers, num_blocks, nkv, block_size, D, dtype=dtype, device=self.device)
        self.v = torch.zeros(num_layers, num_blocks, nkv, block_size // 8, D, 8, dtype=dtype,
                             device=self.device)
        self.manager = _runtime().BlockManager(num_blocks, block_size, window_length,
                                               num_sink_tokens, max_chunk)

    @staticmethod
    def bytes_per_block(spec: ModelSpec, num_layers: int, block_size: int, dtype_bytes: int = 2) -> int:
        return 2 * num_layers * spec.num_kv_heads * spec.head_dim * block_size * dtype_bytes

    @classmethod
    def size_from_memory(cls, spec: ModelSpec, num_layers: int, block_size: int,
                         free_bytes: int, utilization: float, reserve_bytes: int = 0,
                         dtype_bytes: int = 2) -> int:
        per = cls.bytes_per_block(spec, num_layers, block_size, dtype_bytes)
        return max(1, int((free_bytes * utilization - reserve_bytes) // per))

    def layer(self, i: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.k[i], self.v[i]

    def attn_params(self) -> Dict[str, float]:
        """Everything the attention kernels need besides the batch: window policy + KV scales."""
        d = dict(self.window_params())
        d.update(k_scale=self.k_scale, v_scale=self.v_scale)
        return d

    # window policy exposed to AttnMetadata
    def window_params(self) -> Dict[str, int]:
        m = self.manager
        if m.window_length <= 0:
            return dict(n_sink=0, sink_pad=0, ring=0, window=0)
        return dict(n_sink=m.num_sink_tokens, sink_pad=m.sink_pad, ring=m.ring,
                    window=m.window_length)

    def build_metadata(self, seq_ids: Sequence[int], q_lens: Sequence[int],
                       pos_offsets: Optional[Sequence[int]] = None,
                       num_splits: Optional[int] = None,
                       logits_rows: Optional[torch.Tensor] = None) -> AttnMetadata:
        """Eager (non-graph) metadata for sequences whose new tokens were already reserved."""
        from ... import ops
        B = len(seq_ids)
        T = int(sum(q_lens))
        m = self.manager
        max_blocks = max([len(m.block_table(s)) for s in seq_ids] + [1])
        pin = self.device.type == "cuda"
        slot = torch.empty(T, dtype=torch.int64, pin_memory=pin)
        pos = torch.empty(T, dtype=torch.int32, pin_memory=pin)
        bt = torch.empty(B, max_blocks, dtype=torch.int32, pin_memory=pin)
        sl = torch.empty(B, dtype=torch.int32, pin_memory=pin)
        qs = torch.empty(B + 1, dtype=torch.int32, pin_memory=pin)
        m.prepare(list(seq_ids), list(q_lens), slot.data_ptr(), pos.data_ptr(), bt.data_ptr(),
                  max_blocks, sl.data_ptr(), qs.data_ptr(), 0,
                  list(pos_offsets) if pos_offsets is not None else [])
        dev = self.device
        is_decode = all(q == 1 for q in q_lens)
        wp = self.attn_params()
        if num_splits is None:
            max_len = int(sl.max()) if B else 1
            num_splits = ops.decode_splits(B, self.spec.num_kv_heads, self.spec.group_size,
                                           max_len, kv_fp8=self.dtype != torch.bfloat16
                                           ) if (is_decode and dev.type == "cuda") else 1
        tile_map = None
        if not is_decode and dev.type == "cuda" and B:
            tile_map = ops.prefill_tiles(q_lens, self.spec.num_heads,
                                         self.spec.num_kv_heads).to(dev, non_blocking=True)
        return AttnMetadata(
            num_tokens=T, num_seqs=B, is_decode=is_decode, tile_map=tile_map,
            positions=pos.to(dev, non_blocking=True), slot_mapping=slot.to(dev, non_blocking=True),
            block_tables=bt.to(dev, non_blocking=True), seq_lens=sl.to(dev, non_blocking=True),
            q_start=qs.to(dev, non_blocking=True), max_q=int(max(q_lens)) if B else 0,
            num_splits=num_splits, logits_rows=logits_rows, **wp)


class PartialLlamaSinkCache:
    """Multi-session (``generation_id``-keyed) KV cache with optional attention-sink window.

    API-compatible with the reference class (cache.py:7-135).  ``window_length=0`` gives a full
    cache.  The pool is created lazily by the first :class:`LlamaBlock` that uses the cache (it
    needs the model dimensions and the block's layer ids), or explicitly via :meth:`bind`.
    """

    def __init__(self, window_length: int = 0, num_sink_tokens: int = 0, num_blocks: int = 1024,
                 block_size: int = 64, max_chunk: int = 512):
        self.window_length = int(window_length)
        self.num_sink_tokens = int(num_sink_tokens)
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.max_chunk = max_chunk
        self.pool: Optional[KVPool] = None
        self.layer_ids: List[int] = []
        self._layer_slot: Dict[int, int] = {}
        self._sessions: Dict[str, List[int]] = {}
        self._next_sid = 0
        self._seen_tokens: Dict[str, int] = {}

    # ------------------------------------------------------------------ setup
    def bind(self, spec: ModelSpec, layer_ids: Sequence[int], device=None,
             dtype=torch.bfloat16) -> "PartialLlamaSinkCache":
        if self.pool is None:
            self.layer_ids = list(layer_ids)
            self._layer_slot = {l: i for i, l in enumerate(self.layer_ids)}
            self.pool = KVPool(spec, len(self.layer_ids), self.num_blocks, self.block_size, device,
                               dtype, self.window_length, self.num_sink_tokens, self.max_chunk)
        return self

    # ------------------------------------------------------------------ sessions
    def session_rows(self, generation_id: str, batch: int) -> List[int]:
        rows = self._sessions.get(generation_id)
        if rows is None:
            rows = list(range(self._next_sid, self._next_sid + batch))
            self._next_sid += batch
            self._sessions[generation_id] = rows
            self._seen_tokens[generation_id] = 0
        if len(rows) != batch:
            raise ValueError(f"session {generation_id!r} has batch {len(rows)}, got {batch}")
        return rows

    def has_session(self, generation_id: str) -> bool:
        return generation_id in self._sessions

    def close_session(self, generation_id: str) -> None:
        """Free the KV blocks of a session (the reference has no such API)."""
        for sid in self._sessions.pop(generation_id, []):
            if self.pool is not None:
                self.pool.manager.free_sequence(sid)
        self._seen_tokens.pop(generation_id, None)

    def sessions(self) -> List[str]:
        return list(self._sessions)

    # ------------------------------------------------------------------ reference API
    def get_seq_length(self, layer_idx: Optional[int] = 0, generation_id: Optional[str] = None) -> int:
        """Number of cached tokens (in-window for a sink cache) for the session."""
        if not generation_id:
            raise ValueError("generation_id not provided")
        rows = self._sessions.get(generation_id)
        if not rows or self.pool is None:
            return 0
        m = self.pool.manager
        if not m.has_sequence(rows[0]):
            return 0
        L = m.length(rows[0])
        if self.window_length > 0:
            return min(L, self.window_length)
        return L

    def get_seen_tokens(self, generation_id: str) -> int:
        return self._seen_tokens.get(generation_id, 0)

    def reserve(self, generation_id: str, batch: int, n_new: int) -> List[int]:
        rows = self.session_rows(generation_id, batch)
        self.reserve_rows(generation_id, rows, [n_new] * len(rows), n_new)
        return rows

    def reserve_rows(self, generation_id: str, rows: Sequence[int], q_lens: Sequence[int],
                     seen: int) -> None:
        """All-or-nothing reservation of ``q_lens[i]`` new tokens on each of the session's rows
        (and ``seen`` more tokens on its seen-token counter).  On pool exhaustion nothing changes
        -- a session created for this call is dropped again -- and ``MemoryError`` is raised."""
        m = self.pool.manager
        if not m.append_batch(list(rows), [int(q) for q in q_lens]):
            if self._seen_tokens.get(generation_id, 0) == 0 and not any(
                    m.has_sequence(r) for r in rows):
                self._sessions.pop(generation_id, None)
                self._seen_tokens.pop(generation_id, None)
            raise MemoryError("KV pool exhausted: close sessions or enlarge num_blocks")
        self._seen_tokens[generation_id] += int(seen)

    def unreserve_rows(self, generation_id: str, rows: Sequence[int], q_lens: Sequence[int],
                       seen: int) -> None:
        """Undo :meth:`reserve_rows` after a failed forward: the session is as long as before the
        call (a session the call created disappears)."""
        m = self.pool.manager
        m.rollback_batch(list(rows), [int(q) for q in q_lens])
        left = self._seen_tokens.get(generation_id, 0) - int(seen)
        if left <= 0 and not any(m.has_sequence(r) for r in rows):
            self._sessions.pop(generation_id, None)
            self._seen_tokens.pop(generation_id, None)
        else:
            self._seen_tokens[generation_id] = left

    def update(self, key_states: torch.Tensor, value_states: torch.Tensor, layer_idx: int,
               cache_kwargs: Optional[Dict[str, Any]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """HF ``Cache.update`` protocol: store already-rotated ``key_states``/``value_states``
        ``[B, nkv, T, D]`` for ``cache_kwargs['generation_id']`` and return the session's cached
        keys/values ``[B, nkv, S, D]`` in slot order (sinks first, then the rolling window).

        The first layer of this cache reserves the slots for the new tokens.
        """
        if cache_kwargs is None or "generation_id" not in cache_kwargs:
            raise ValueError("generation_id not found in cache_kwargs")
        gid = cache_kwargs["generation_id"]
        if self.pool is None:
            raise RuntimeError("cache is not bound to a model; call bind(spec, layer_ids)")
        B, nkv, T, D = key_states.shape
        li = self._layer_slot[layer_idx]
        if li == 0:
            self.reserve(gid, B, T)
        rows = self._sessions[gid]
        m = self.pool.manager
        kc, vc = self.pool.layer(li)
        bs = self.pool.block_size
        outs_k, outs_v = [], []
        for b, sid in enumerate(rows):
            L = m.length(sid)
            slots = torch.tensor([m.slot_of(sid, a) for a in range(L - T, L)], dtype=torch.long)
            blk, off = (slots // bs).to(kc.device), (slots % bs).to(kc.device)
            kc[blk, :, off, :] = key_states[b].transpose(0, 1).to(kc.dtype)
            vc[blk, :, off // 8, :, off % 8] = value_states[b].transpose(0, 1).to(vc.dtype)
            nslots = m.slots_for(L)
            bt = torch.tensor(m.block_table(sid), dtype=torch.long, device=kc.device)
            nb = (nslots + bs - 1) // bs
            K = kc[bt[:nb]].permute(1, 0, 2, 3).reshape(nkv, nb * bs, D)[:, :nslots]
            V = vc[bt[:nb]].permute(1, 0, 2, 4, 3).reshape(nkv, nb * bs, D)[:, :nslots]
            if self.window_length > 0 and L > self.num_sink_tokens:
                keep = list(range(min(L, self.num_sink_tokens)))
                sink_pad = m.sink_pad
                ring = m.ring
                lo = max(self.num_sink_tokens, L - (self.window_length - self.num_sink_tokens))
                keep += [sink_pad + (a - self.num_sink_tokens) % ring for a in range(lo, L)]
                idx = torch.tensor(keep, device=kc.device)
                K, V = K[:, idx], V[:, idx]
            outs_k.append(K)
            outs_v.append(V)
        return torch.stack(outs_k), torch.stack(outs_v)

    # ------------------------------------------------------------------ fast path
    def metadata(self, generation_id: str, q_len: int, batch: int,
                 position_offsets: Optional[Sequence[int]] = None) -> AttnMetadata:
        rows = self.session_rows(generation_id, batch)
        return self.pool.build_metadata(rows, [q_len] * batch, pos_offsets=position_offsets)

    def layer_cache(self, layer_idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        return self.pool.layer(self._layer_slot[layer_idx])
