"""Per-GPU stage executor.

Owns one :class:`CausalLMStage` (layer range [+ embedding] [+ LM head]), its paged KV pool and the
per-step host->device metadata path.  One ``execute(plan, inputs)`` call runs one micro-batch step:

  1. free finished sequences / reserve KV blocks for the new tokens (native BlockManager);
  2. write slot_mapping, positions, block tables, seq_lens, q_start (and sampling parameters on
     the last stage) straight into a pinned staging buffer (C++, no Python loops) and issue one
     small async H2D copy per section into persistent device buffers;
  3. decode steps (every sequence feeds one token) replay a hipGraph captured per batch-size
     bucket — the whole stage (all local layers [+ head + sampling]) is ONE graph launch, padded
     rows carry seq_len 0 / slot -1 so one graph serves every batch up to its bucket; prefill /
     mixed steps run eagerly on the same kernels (varlen, chunked).

This replaces the reference's per-op graph capture of RoPE / RMSNorm pieces
(modules.py:28-34, 130-144 via utils/cuda.py) with whole-step capture.
"""
from __future__ import annotations

import bisect
import logging
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from ..models.common import AttnMetadata
from ..models.llama.cache import KVPool
from ..models.stage import CausalLMStage
from ..utils.cuda import capture_guard, prime_graph_rng
from .hostclock import HOST
from .watchdog import TRACKER, wait_event

log = logging.getLogger(__name__)

import os as _os  # noqa: E402

# DLI_DEBUG (comma list): "trace" = roctx range per stage step (rocprofv3 --marker-trace / torch
# profiler); "sync" = synchronise after every stage step and check outputs (NaN/Inf, token range)
_DEBUG_FLAGS = {f.strip() for f in _os.environ.get("DLI_DEBUG", "").split(",")}
_TRACE = "trace" in _DEBUG_FLAGS
_DEBUG = "sync" in _DEBUG_FLAGS


@dataclass
class StepPlan:
    """One micro-batch step, identical on every stage (broadcast by the driver)."""

    step: int
    mb: int
    seq_ids: List[int]
    q_lens: List[int]
    free_ids: List[int] = field(default_factory=list)
    sample_rows: List[int] = field(default_factory=list)   # indices into seq_ids
    temperature: List[float] = field(default_factory=list)  # one per sample row
    top_k: List[int] = field(default_factory=list)
    top_p: List[float] = field(default_factory=list)
    seeds: List[int] = field(default_factory=list)
    sample_pos: List[int] = field(default_factory=list)     # sampled token's position (RNG key)
    kind: str = "run"                                       # run | barrier | stop
    tokens: Optional[List[int]] = None                      # stage-0 input (not broadcast)

    def __post_init__(self):
        # computed once: both are read several times per step on every stage
        self._num_tokens = int(sum(self.q_lens))
        self._decode = bool(self.seq_ids) and self._num_tokens == len(self.q_lens)

    @property
    def is_decode(self) -> bool:
        return self._decode

    @property
    def num_tokens(self) -> int:
        return self._num_tokens

    def to_wire(self) -> dict:
        d = dict(step=self.step, mb=self.mb, seq_ids=self.seq_ids, q_lens=self.q_lens,
                 free_ids=self.free_ids, sample_rows=self.sample_rows,
                 temperature=self.temperature, top_k=self.top_k, top_p=self.top_p,
                 seeds=self.seeds, sample_pos=self.sample_pos, kind=self.kind)
        return d

    @classmethod
    def from_wire(cls, d: dict) -> "StepPlan":
        return cls(**d)


def _fill_pos(dst: torch.Tensor, plan: StepPlan, n: int) -> None:
    """Per-sample-row RNG counters (the sampled token's position); plans without them (built by
    hand) fall back to the step number, which keeps them distinct across steps."""
    if len(plan.sample_pos) == n:
        dst[:n] = torch.as_tensor(plan.sample_pos, dtype=torch.int64)
    else:
        dst[:n] = plan.step


class _Staging:
    """Pinned host staging + persistent device buffers with typed section views."""

    def __init__(self, max_tokens: int, max_seqs: int, max_blocks: int, device: torch.device):
        self.max_tokens, self.max_seqs, self.max_blocks = max_tokens, max_seqs, max_blocks
        specs = [("slot_mapping", torch.int64, (max_tokens,)),
                 ("seeds", torch.int64, (max_seqs,)),
                 ("sample_pos", torch.int64, (max_seqs,)),
                 ("logits_rows", torch.int64, (max_seqs,)),
                 ("step", torch.int64, (1,)),
                 ("positions", torch.int32, (max_tokens,)),
                 ("tokens", torch.int32, (max_tokens,)),
                 ("tile_map", torch.int32, (max_tokens + max_seqs, 2)),
                 ("block_tables", torch.int32, (max_seqs, max_blocks)),
                 ("seq_lens", torch.int32, (max_seqs,)),
                 ("q_start", torch.int32, (max_seqs + 1,)),
                 ("top_k", torch.int32, (max_seqs,)),
                 ("temperature", torch.float32, (max_seqs,)),
                 ("top_p", torch.float32, (max_seqs,))]
        self.offsets: Dict[str, Tuple[int, torch.dtype, tuple]] = {}
        off = 0
        for name, dt, shape in specs:
            n = 1
            for s in shape:
                n *= s
            nbytes = n * torch.empty((), dtype=dt).element_size()
            self.offsets[name] = (off, dt, shape)
            off += (nbytes + 255) // 256 * 256
        gpu = device.type == "cuda"
        # a RING of host slots: the uploads of step k may still be pending on the stream when the
        # host already stages step k+1 (the host runs ahead of the GPU), so a slot is reused only
        # after the event recorded behind its uploads has completed.  On the GPU the slots are
        # coherent, device-mapped host memory and ONE copy kernel per step moves the written
        # sections on the caller's stream (csrc/comm/streams.hip copy_segments): a host -> device
        # memcpy would go through a copy queue shared by every stream of the process, where the
        # rotating head's uploads (ordered behind a spinning receive) hold up the step's uploads
        self.nslots = 4 if gpu else 1
        self._hbufs = []
        if gpu:
            from .. import ops
            self._C = ops.native()
            self._hbufs = [self._C.HostBuffer(off) for _ in range(self.nslots)]
            self.hosts = [b.tensor() for b in self._hbufs]
        else:
            self.hosts = [torch.zeros(off, dtype=torch.uint8) for _ in range(self.nslots)]
        self.hviews = [{k: self._view(h, k) for k in self.offsets} for h in self.hosts]
        self.events: List[Optional[torch.cuda.Event]] = [None] * self.nslots
        self._pending: List[Tuple[int, int]] = []
        self.slot = 0
        self.waited_ms = 0.0   # host time blocked in acquire() (the device behind the ring)
        self.host = self.hosts[0]
        self.h = self.hviews[0]
        self.dev = torch.zeros(off, dtype=torch.uint8, device=device)
        self.d = {k: self._view(self.dev, k) for k in self.offsets}
        self.device = device

    def acquire(self) -> None:
        """Switch to the next host slot, waiting until its previous uploads have executed."""
        self.slot = (self.slot + 1) % self.nslots
        ev = self.events[self.slot]
        if ev is not None and not ev.query():
            t0 = time.perf_counter()
            wait_event(ev, "staging slot (uploads of an earlier step)")
            ms = (time.perf_counter() - t0) * 1e3
            self.waited_ms += ms
            HOST.add("staging_wait", ms)
        self.host = self.hosts[self.slot]
        self.h = self.hviews[self.slot]

    def release(self) -> None:
        """Enqueue the current slot's uploads (one copy kernel on the current stream) and mark
        the slot reusable once the event behind them completes."""
        if self.device.type == "cuda":
            s = torch.cuda.current_stream().cuda_stream
            for i in range(0, len(self._pending), 24):   # the kernel takes <= 24 segments
                self._C.copy_segments(self.dev.data_ptr(), self._hbufs[self.slot].dev_ptr,
                                      self._pending[i:i + 24], s)
            self._pending = []
            ev = self.events[self.slot] or torch.cuda.Event()
            ev.record()
            self.events[self.slot] = ev

    def _view(self, buf, name):
        off, dt, shape = self.offsets[name]
        n = 1
        for s in shape:
            n *= s
        es = torch.empty((), dtype=dt).element_size()
        return buf[off: off + n * es].view(dt).view(shape)

    def upload(self, name: str, count: int) -> None:
        """Copy the first ``count`` elements (rows for 2-D) of section ``name`` to the device
        (GPU: at :meth:`release`, in one kernel with the slot's other sections)."""
        if count <= 0:
            return
        off, dt, shape = self.offsets[name]
        row = 1
        for s in shape[1:]:
            row *= s
        es = torch.empty((), dtype=dt).element_size()
        nb = count * row * es
        if self.device.type == "cuda":
            self._pending.append((off, nb))   # moved by release()'s copy kernel
        else:
            self.dev[off: off + nb].copy_(self.host[off: off + nb])


class StageExecutor:
    def __init__(self, stage: CausalLMStage, pool: KVPool, max_num_seqs: int = 256,
                 max_num_batched_tokens: int = 8192, max_seq_len: int = 8192,
                 use_graphs: bool = True, graph_batch_sizes: Optional[Sequence[int]] = None):
        self.stage = stage
        self.pool = pool
        self.spec = stage.spec
        self.device = stage.device
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max(max_num_batched_tokens, max_num_seqs)
        self.max_seq_len = max_seq_len
        self.max_blocks = pool.manager.max_blocks_per_seq(max_seq_len)
        self.staging = _Staging(self.max_tokens, max_num_seqs, self.max_blocks, self.device)
        self.use_graphs = use_graphs and self.device.type == "cuda"
        gbs = sorted(set(graph_batch_sizes or [1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 224, 256]))
        self.graph_sizes = [b for b in gbs if b <= max_num_seqs]
        if self.use_graphs and (not self.graph_sizes or self.graph_sizes[-1] < max_num_seqs):
            self.graph_sizes.append(max_num_seqs)
        self._graphs: Dict[int, "_GraphEntry"] = {}
        self._graph_pool = None
        H = self.spec.hidden_size
        self._hidden_in = torch.empty(max_num_seqs, H, dtype=torch.bfloat16, device=self.device) \
            if not stage.has_embed else None
        self._sample_out = torch.empty(max_num_seqs, dtype=torch.int32, device=self.device)
        self._wp = pool.attn_params()
        self._step_counter = 0
        # warm-up / capture stream (a pipeline rank passes its dedicated one: runtime/streams.py)
        self.capture_stream: Optional[torch.cuda.Stream] = None
        self.warm_prefill_gemms()

    def warm_prefill_gemms(self) -> None:
        """Run each distinct prefill-sized projection of this stage once at start-up.  Above
        ``KernelPolicy.tile_gemm_max_m`` rows the projections go to hipBLASLt, which loads a
        kernel's code object the first time a shape selects it: without this the first long
        prompt paid ~1 s of loads (Llama-3.1-70B 32k-token TTFT, profiles/r6/pgemm/).  The
        vocabulary-wide LM head is skipped (prefill projects a few rows through it)."""
        pol = ops.policy()
        M = self.max_tokens
        if (self.device.type != "cuda" or not pol.warm_library_gemms or not ops.library_gemms()
                or pol.tile_gemm_max_m <= 0 or M <= pol.tile_gemm_max_m):
            return
        from ..models.common import Linear
        seen = set()
        with torch.no_grad():
            for mod in self.stage.modules():
                if not isinstance(mod, Linear) or mod.out_features >= ops.TILE_GEMM_WIDE_N:
                    continue
                key = (mod.in_features, mod.out_features, mod.is_fp8, mod.is_int8,
                       mod.bias is not None)
                if key in seen:
                    continue
                seen.add(key)
                mod(torch.zeros(M, mod.in_features, dtype=torch.bfloat16, device=self.device))
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ capacity / bookkeeping
    def apply_frees(self, ids: Sequence[int]) -> None:
        for s in ids:
            self.pool.manager.free_sequence(int(s))

    def reserve(self, seq_ids: Sequence[int], q_lens: Sequence[int]) -> None:
        m = self.pool.manager
        if not m.append_batch(seq_ids, q_lens):
            raise MemoryError(f"KV pool exhausted on stage [{self.stage.start},{self.stage.end}) "
                              f"({m.num_free_blocks} free blocks)")

    # ------------------------------------------------------------------ metadata
    def _stage_metadata(self, plan: StepPlan, rows: int) -> Tuple[int, int]:
        """Fill the staging buffers for ``plan`` padded to ``rows`` sequences; returns (T, nb)."""
        st = self.staging
        B = len(plan.seq_ids)
        if rows > self.max_num_seqs or plan.num_tokens > self.max_tokens:
            raise ValueError("step exceeds executor limits (max_num_seqs / max_num_batched_tokens)")
        st.acquire()
        h = st.h
        nb = self.max_blocks
        T = self.pool.manager.prepare(
            plan.seq_ids, plan.q_lens, h["slot_mapping"].data_ptr(), h["positions"].data_ptr(),
            h["block_tables"].data_ptr(), nb, h["seq_lens"].data_ptr(), h["q_start"].data_ptr(),
            rows, [])
        Tp = max(T, rows) if plan.is_decode else T
        if Tp > T:  # padded decode rows: no cache write, position 0
            h["slot_mapping"][T:Tp] = -1
            h["positions"][T:Tp] = 0
        st.upload("slot_mapping", Tp)
        st.upload("positions", Tp)
        st.upload("block_tables", rows)
        st.upload("seq_lens", rows)
        st.upload("q_start", rows + 1)
        self._n_tiles = 0
        if not plan.is_decode and self.device.type == "cuda":
            tm = ops.prefill_tiles(plan.q_lens, self.spec.num_heads, self.spec.num_kv_heads,
                                   out=h["tile_map"])
            self._n_tiles = tm.shape[0]
            st.upload("tile_map", self._n_tiles)
        if plan.tokens is not None:
            tok = h["tokens"]
            tok[:T] = torch.as_tensor(plan.tokens, dtype=torch.int32)
            if Tp > T:
                tok[T:Tp] = 0
            st.upload("tokens", Tp)
        if self.stage.has_head:
            ns = len(plan.sample_rows)
            if plan.is_decode and ns == B:
                # every row samples (graph path): parameters per row, padded greedy
                h["temperature"][:B] = torch.as_tensor(plan.temperature, dtype=torch.float32)
                h["top_k"][:B] = torch.as_tensor(plan.top_k, dtype=torch.int32)
                h["top_p"][:B] = torch.as_tensor(plan.top_p, dtype=torch.float32)
                h["seeds"][:B] = torch.as_tensor(plan.seeds, dtype=torch.int64)
                _fill_pos(h["sample_pos"], plan, B)
                if rows > B:
                    h["temperature"][B:rows] = 0.0
                    h["top_k"][B:rows] = 0
                    h["top_p"][B:rows] = 1.0
                    h["seeds"][B:rows] = 0
                    h["sample_pos"][B:rows] = 0
                n = rows
            else:
                qs = h["q_start"]
                h["logits_rows"][:ns] = torch.as_tensor([int(qs[r + 1]) - 1 for r in plan.sample_rows],
                                                        dtype=torch.int64)
                h["temperature"][:ns] = torch.as_tensor(plan.temperature, dtype=torch.float32)
                h["top_k"][:ns] = torch.as_tensor(plan.top_k, dtype=torch.int32)
                h["top_p"][:ns] = torch.as_tensor(plan.top_p, dtype=torch.float32)
                h["seeds"][:ns] = torch.as_tensor(plan.seeds, dtype=torch.int64)
                _fill_pos(h["sample_pos"], plan, ns)
                st.upload("logits_rows", ns)
                n = ns
            st.upload("temperature", n)
            st.upload("top_k", n)
            st.upload("top_p", n)
            st.upload("seeds", n)
            st.upload("sample_pos", n)
            h["step"][0] = plan.step
            st.upload("step", 1)
        st.release()
        return T, nb

    def _metadata(self, plan: StepPlan, rows: int, num_splits: int,
                  decode: bool) -> AttnMetadata:
        d = self.staging.d
        T = rows if decode else plan.num_tokens
        logits_rows = None
        if self.stage.has_head and not (decode and len(plan.sample_rows) == len(plan.seq_ids)):
            logits_rows = d["logits_rows"][: len(plan.sample_rows)]
        return AttnMetadata(
            num_tokens=T, num_seqs=rows, is_decode=decode, positions=d["positions"][:T],
            slot_mapping=d["slot_mapping"][:T], block_tables=d["block_tables"][:rows],
            seq_lens=d["seq_lens"][:rows], q_start=d["q_start"][: rows + 1],
            max_q=max(plan.q_lens) if plan.q_lens else 0, num_splits=num_splits,
            workspace=self._workspace(rows, num_splits) if decode else None,
            tile_map=(d["tile_map"][: self._n_tiles] if (not decode and self._n_tiles) else None),
            logits_rows=logits_rows, **self._wp)

    def _workspace(self, rows: int, splits: int):
        if splits <= 1:
            return None
        key = (rows, splits)
        ws = getattr(self, "_ws", {})
        self._ws = ws
        if key not in ws:
            ws[key] = ops.decode_workspace(rows, self.spec.num_heads, self.spec.head_dim, splits,
                                           self.device)
        return ws[key]

    def _splits(self, rows: int) -> int:
        if self.device.type != "cuda":
            return 1
        return ops.decode_splits(rows, self.spec.num_kv_heads, self.spec.group_size,
                                 self.max_seq_len, kv_fp8=self.pool.dtype != torch.bfloat16)

    # ------------------------------------------------------------------ forward
    def _forward(self, meta: AttnMetadata, inputs: torch.Tensor, n_sample: int,
                 project: bool = True) -> torch.Tensor:
        out = self.stage(inputs, meta, self.pool, project=project)
        if not self.stage.has_head or not project:
            return out
        d = self.staging.d
        tokens = self._sample_out[:n_sample]
        ops.sample(out, temperature=d["temperature"][:n_sample], top_k=d["top_k"][:n_sample],
                   top_p=d["top_p"][:n_sample], seeds=d["seeds"][:n_sample], step=d["step"],
                   out=tokens, counters=d["sample_pos"][:n_sample])
        return tokens

    def input_buffer(self, plan: StepPlan) -> Optional[torch.Tensor]:
        """Where the previous stage's hidden states for ``plan`` should be received (non-first
        stages): the graph's static input for decode steps, a fresh tensor otherwise."""
        if self.stage.has_embed:
            return None
        if plan.is_decode and self._graph_rows(len(plan.seq_ids)) is not None:
            return self._hidden_in[: len(plan.seq_ids)]
        return torch.empty(plan.num_tokens, self.spec.hidden_size, dtype=torch.bfloat16,
                           device=self.device)

    def _graph_rows(self, B: int) -> Optional[int]:
        if not self.use_graphs or B > self.graph_sizes[-1]:
            return None
        return self.graph_sizes[bisect.bisect_left(self.graph_sizes, B)]

    @torch.inference_mode()
    def execute(self, plan: StepPlan, inputs: Optional[torch.Tensor] = None,
                token_src: Optional[torch.Tensor] = None, project: bool = True) -> torch.Tensor:
        """Run one step.  ``inputs``: hidden states [T, H] for non-first stages (ignored on stage 0,
        which embeds ``plan.tokens``).  Returns hidden [T, H] or sampled tokens [n_sample] int32
        (device tensors; the caller decides when to synchronise).  ``project=False`` (last stage,
        decode steps whose vocabulary projection + sampling run on another rank): returns the
        final-normed hidden states [B, H] instead of tokens."""
        if not (_TRACE or _DEBUG):
            return self._execute(plan, inputs, token_src, project)
        tag = f"stage[{self.stage.start},{self.stage.end}) step={plan.step} mb={plan.mb} " \
              f"{'decode' if plan.is_decode else 'prefill'} B={len(plan.seq_ids)} T={plan.num_tokens}"
        if _TRACE and self.device.type == "cuda":
            torch.cuda.nvtx.range_push(tag)  # roctx range on ROCm (rocprofv3 --marker-trace)
        try:
            out = self._execute(plan, inputs, token_src, project)
        finally:
            if _TRACE and self.device.type == "cuda":
                torch.cuda.nvtx.range_pop()
        if _DEBUG and out.numel():
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            if out.is_floating_point() and not torch.isfinite(out.float()).all():
                raise FloatingPointError(f"non-finite output in {tag}")
            if not out.is_floating_point() and (out.min() < 0 or out.max() >= self.spec.vocab_size):
                raise ValueError(f"sampled token out of range in {tag}")
        return out

    def _execute(self, plan: StepPlan, inputs: Optional[torch.Tensor],
                 token_src: Optional[torch.Tensor] = None, project: bool = True) -> torch.Tensor:
        # host phases (runtime/hostclock.py): "stage" = frees, KV reservation, metadata staging;
        # "staging_wait" (charged by _Staging.acquire) = blocked behind the device; "launch" =
        # graph replay / eager kernel launches
        t0, w0 = time.perf_counter(), self.staging.waited_ms
        self.apply_frees(plan.free_ids)
        if not plan.seq_ids:
            return torch.empty(0, device=self.device)
        self.reserve(plan.seq_ids, plan.q_lens)
        B = len(plan.seq_ids)
        decode = plan.is_decode
        grows = self._graph_rows(B) if decode else None
        rows = grows if grows is not None else B
        self._stage_metadata(plan, rows)
        if TRACKER._words is not None:
            TRACKER.note_plan(plan.step, B=B, T=plan.num_tokens, rows=rows,
                              max_len=int(self.staging.h["seq_lens"][:B].max()))
        if self.stage.has_embed and plan.tokens is None:
            # lookahead step: this step's input tokens are the previous step's sampler output,
            # still on the device (stream order makes the copy wait for that sampler)
            if token_src is None or not decode:
                raise ValueError("a plan without tokens needs token_src (decode steps only)")
            self.staging.d["tokens"][:B].copy_(token_src[:B], non_blocking=True)
        n_sample = len(plan.sample_rows)
        all_sample = decode and n_sample == B
        project = project or not self.stage.has_head
        if not project and not all_sample:
            raise ValueError("project=False needs a decode step in which every row samples")
        if grows is not None and (not self.stage.has_head or all_sample):
            if not self.stage.has_embed:
                src = inputs[:B]
                if src.data_ptr() != self._hidden_in.data_ptr():
                    self._hidden_in[:B].copy_(src)
            key = grows if project else (grows, "norm")
            g = self._graphs.get(key)
            if g is None:
                g = self._capture(grows, project)
            TRACKER.device_mark("compute_in", plan.step, torch.cuda.current_stream())
            t1 = time.perf_counter()
            HOST.add("stage", (t1 - t0) * 1e3 - (self.staging.waited_ms - w0))
            g.graph.replay()
            if self.stage.has_head and project:
                HOST.since("launch", t1)
                return g.out[:n_sample]
            out = g.out[:B].clone()
            HOST.since("launch", t1)
            return out
        splits = self._splits(rows) if decode else 1
        meta = self._metadata(plan, rows, splits, decode)
        if self.stage.has_embed:
            x = self.staging.d["tokens"][: meta.num_tokens]
        else:
            x = inputs
        t1 = time.perf_counter()
        HOST.add("stage", (t1 - t0) * 1e3 - (self.staging.waited_ms - w0))
        out = self._forward(meta, x, n_sample if self.stage.has_head else 0, project)
        HOST.since("launch", t1)
        return out if project else out[:B]

    # ------------------------------------------------------------------ graphs
    def _capture(self, rows: int, project: bool = True) -> "_GraphEntry":
        """Capture the decode step for ``rows`` sequences (buffers already staged by the caller);
        ``project=False``: the last stage's variant that ends at the final norm."""
        splits = self._splits(rows)
        plan_like = StepPlan(0, 0, list(range(rows)), [1] * rows,
                             sample_rows=list(range(rows)))
        meta = self._metadata(plan_like, rows, splits, True)
        x = self.staging.d["tokens"][:rows] if self.stage.has_embed else self._hidden_in[:rows]
        n_sample = rows if self.stage.has_head else 0
        # warm up on a side stream (hipBLASLt heuristics, allocator) then capture
        s = self.capture_stream or torch.cuda.Stream()
        cur = torch.cuda.current_stream()
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(2):
                self._forward(meta, x, n_sample, project)
        cur.wait_stream(s)
        prime_graph_rng(self.device)
        graph = torch.cuda.CUDAGraph()
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        # thread_local: another thread (token publisher) may synchronise events meanwhile
        with capture_guard(), torch.cuda.graph(graph, pool=self._graph_pool, stream=s,
                                               capture_error_mode="thread_local"):
            out = self._forward(meta, x, n_sample, project)
        cur.wait_stream(s)
        entry = _GraphEntry(graph, out)
        self._graphs[rows if project else (rows, "norm")] = entry
        log.info("captured decode graph rows=%d splits=%d stage=[%d,%d)%s", rows, splits,
                 self.stage.start, self.stage.end, "" if project else " (ends at the final norm)")
        # (the captured run did not execute; the caller replays the graph for the real step)
        return entry

    def warmup_graphs(self, sizes: Optional[Sequence[int]] = None,
                      variants: Sequence[bool] = (True,)) -> None:
        """Pre-capture decode graphs with dummy (empty, seq_len 0) batches.  ``variants``: the
        ``project`` flags to capture (False = the last stage's graph that ends at the final norm,
        used when the LM head rotates)."""
        if not self.use_graphs:
            return
        todo = [(r, p) for r in (sizes or self.graph_sizes) for p in variants
                if (r if p else (r, "norm")) not in self._graphs]
        for r, project in todo:
            self.staging.acquire()
            h = self.staging.h
            h["seq_lens"][:r] = 0
            h["slot_mapping"][:r] = -1
            h["positions"][:r] = 0
            h["block_tables"][:r] = 0
            h["q_start"][: r + 1] = 0
            h["tokens"][:r] = 0
            h["temperature"][:r] = 0
            h["top_k"][:r] = 0
            h["top_p"][:r] = 1
            h["seeds"][:r] = 0
            h["sample_pos"][:r] = 0
            for k, n in (("seq_lens", r), ("slot_mapping", r), ("positions", r), ("block_tables", r),
                         ("q_start", r + 1), ("tokens", r), ("temperature", r), ("top_k", r),
                         ("top_p", r), ("seeds", r), ("sample_pos", r)):
                self.staging.upload(k, n)
            self.staging.release()
            if self._hidden_in is not None:
                self._hidden_in[:r].zero_()
            self._capture(r, project)
        torch.cuda.synchronize()


@dataclass
class _GraphEntry:
    graph: "torch.cuda.CUDAGraph"
    out: torch.Tensor
