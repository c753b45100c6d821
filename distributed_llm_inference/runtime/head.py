"""Rotating LM head: the vocabulary projection + sampling of decode steps spread over every
pipeline rank.

With the head on the last stage only, that stage carries its layers PLUS the widest GEMM of the
model (Llama-3-70B: 8192 x 128256, 0.75 ms at 512 rows on MI355X against ~0.98 ms per layer) and
the sampler, and sets the pipeline's pace: at PP=8 (10 layers per stage) it runs ~7 % longer than
every other stage, and whole layers cannot be moved to even that out.  Here the last stage stops at
the final RMSNorm for decode steps and ships the normed hidden states (B x H bf16, 8 MB at
B = 512) over a dedicated xGMI pair communicator to the rank whose turn it is
(``plan.step % N``); that rank projects + samples on a side HIP stream of its own (concurrent
with its layer work) and returns the tokens to the driver on its shm token channel.  Every rank
then does its layers + 1/N of the heads, and the last stage no longer pays for the head.

The reference has no head at all (reference models/llama/model.py:16-23: a block server returns
hidden states); this is the new framework's own cost, kept off the critical path.

Prefill / mixed steps (and steps whose rows do not all sample) keep the head on the last stage.
Sampling is bit-identical wherever it runs: the same kernels on the same bf16 inputs, and the
sampler's RNG is keyed by (seed, step), not by device.
"""
from __future__ import annotations

import bisect
import collections
import logging
from typing import Deque, List, Optional, Sequence

import torch

from .. import ops
from ..models.embed_head import LMHead
from ..utils.cuda import capture_guard, prime_graph_rng
from .executor import StepPlan, _Staging, _fill_pos
from .streams import token_ring
from .watchdog import TRACKER

log = logging.getLogger(__name__)


class HeadPolicy:
    """Which rank projects + samples a step (identical on every rank)."""

    def __init__(self, world: int, enabled: bool, max_rows: int):
        self.world = world
        self.enabled = bool(enabled) and world > 1
        self.max_rows = max_rows

    def rank_for(self, plan: StepPlan) -> int:
        last = self.world - 1
        if not self.enabled or not plan.seq_ids:
            return last
        B = len(plan.seq_ids)
        if plan.is_decode and len(plan.sample_rows) == B and B <= self.max_rows:
            return plan.step % self.world
        return last

    def offloaded(self, plan: StepPlan) -> bool:
        return self.rank_for(plan) != self.world - 1


class HeadRunner:
    """Vocabulary projection + sampling of final-normed hidden states [B, H] of a decode step
    (every row samples).  Decode buckets replay a hipGraph (projection + sampler), like the stage
    executor's; the sampling parameters are staged the same way (pinned ring -> device)."""

    def __init__(self, head: LMHead, device: torch.device, max_rows: int, use_graphs: bool = True,
                 graph_sizes: Optional[Sequence[int]] = None,
                 capture_stream: Optional["torch.cuda.Stream"] = None):
        self.head = head
        self.capture_stream = capture_stream
        self.device = device
        self.max_rows = max_rows
        self.use_graphs = use_graphs and device.type == "cuda"
        gs = sorted(set(b for b in (graph_sizes or [max_rows]) if b <= max_rows))
        if not gs or gs[-1] < max_rows:
            gs.append(max_rows)
        self.graph_sizes = gs
        H = head.spec.hidden_size
        self.x = torch.empty(max_rows, H, dtype=torch.bfloat16, device=device)
        self.out = torch.empty(max_rows, dtype=torch.int32, device=device)
        self.staging = _Staging(max_rows, max_rows, 1, device)
        self._graphs = {}
        self._pool = None

    def _rows(self, B: int) -> int:
        if not self.use_graphs:
            return B
        return self.graph_sizes[bisect.bisect_left(self.graph_sizes, B)]

    def _stage(self, plan: StepPlan, rows: int) -> None:
        st = self.staging
        st.acquire()
        h = st.h
        B = len(plan.seq_ids)
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
        h["step"][0] = plan.step
        for k in ("temperature", "top_k", "top_p", "seeds", "sample_pos"):
            st.upload(k, rows)
        st.upload("step", 1)
        st.release()

    def _forward(self, rows: int) -> torch.Tensor:
        d = self.staging.d
        logits = self.head.project(self.x[:rows], tile=True)
        return ops.sample(logits, temperature=d["temperature"][:rows], top_k=d["top_k"][:rows],
                          top_p=d["top_p"][:rows], seeds=d["seeds"][:rows], step=d["step"],
                          out=self.out[:rows], counters=d["sample_pos"][:rows])

    @torch.inference_mode()
    def run(self, plan: StepPlan, x: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Tokens [B] int32 (device) on the current stream.  ``x``: the normed hidden states
        [B, H]; None when they were already received into ``self.x``."""
        B = len(plan.seq_ids)
        if B > self.max_rows:
            raise ValueError(f"head step of {B} rows > {self.max_rows}")
        rows = self._rows(B)
        self._stage(plan, rows)
        if x is not None and x.data_ptr() != self.x.data_ptr():
            self.x[:B].copy_(x[:B], non_blocking=True)
        if rows > B:
            self.x[B:rows].zero_()
        if not self.use_graphs:
            return self._forward(rows)[:B]
        g = self._graphs.get(rows)
        if g is None:
            g = self._capture(rows)
        g.replay()
        return self.out[:B]

    @torch.inference_mode()
    def warmup(self) -> None:
        """Capture every bucket's graph now (dummy greedy rows), before any traffic."""
        if not self.use_graphs:
            return
        for rows in self.graph_sizes:
            if rows in self._graphs:
                continue
            self.x[:rows].zero_()
            plan = StepPlan(0, 0, list(range(rows)), [1] * rows, sample_rows=list(range(rows)),
                            temperature=[0.0] * rows, top_k=[0] * rows, top_p=[1.0] * rows,
                            seeds=[0] * rows)
            self._stage(plan, rows)
            self._capture(rows)
        torch.cuda.synchronize(self.device)

    def _capture(self, rows: int):
        cur = torch.cuda.current_stream()
        s = self.capture_stream or torch.cuda.Stream()
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(2):
                self._forward(rows)
        cur.wait_stream(s)
        prime_graph_rng(torch.cuda.current_device())
        g = torch.cuda.CUDAGraph()
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        # thread_local: publisher threads may synchronise events while this captures
        with capture_guard(), torch.cuda.graph(g, pool=self._pool, stream=s,
                                               capture_error_mode="thread_local"):
            self._forward(rows)
        cur.wait_stream(s)
        self._graphs[rows] = g
        log.info("captured head graph rows=%d", rows)
        return g


class HeadJobs:
    """This rank's share of the rotating head: for every step whose turn it is, receive the
    last stage's normed hidden states, project + sample, and hand the tokens to ``publish``.

    GPU (RCCL): a job is enqueued on a side HIP stream of its own — receive (an RCCL kernel that
    waits for the last stage's send), graph replay, D2H copy — so the host never blocks and the
    head runs concurrently with this rank's layer work.  It is enqueued ``delay`` steps after its
    own step left this rank (``delay`` = stages between this rank and the end of the pipeline),
    i.e. about when its hidden states arrive: posted at once, the waiting receive kernel would sit
    on the GPU (and on whatever hardware queue its stream shares) for a whole pipeline traversal.
    ``flush`` enqueues everything deferred (idle rank, driver collecting, barrier).
    CPU (gloo): the receive is posted at once (``irecv``) and the job runs when this rank is idle
    or its tokens are wanted (``run_oldest`` / ``drain``)."""

    def __init__(self, runner: HeadRunner, transport, last_rank: int, publish, delay: int = 0,
                 stream: Optional["torch.cuda.Stream"] = None):
        self.runner = runner
        self.tr = transport
        self.last = last_rank
        self.publish = publish            # publish(plan, pinned_tokens, event_or_None)
        self.delay = max(0, int(delay))
        self.gpu = runner.device.type == "cuda"
        # the rank's dedicated head stream (runtime/streams.py: a hardware queue of its own, so
        # the waiting receive never sits in front of compute or the stage transfers)
        self.stream = (stream or torch.cuda.Stream(device=runner.device)) if self.gpu else None
        self._pending: Deque[tuple] = collections.deque()    # CPU: (plan, buf, work)
        self._deferred: Deque[list] = collections.deque()    # GPU: [plan, age]
        self.jobs = 0
        self.enqueued = 0

    def submit(self, plan: StepPlan) -> None:
        self.jobs += 1
        if self.gpu:
            self._deferred.append([plan, 0])
            if self.delay == 0:
                self.flush()
            return
        B = len(plan.seq_ids)
        buf = torch.empty(B, self.runner.x.shape[1], dtype=torch.bfloat16)
        work = self.tr.irecv_head(buf, self.last)
        self._pending.append((plan, buf, work))

    def tick(self) -> None:
        """One more step left this rank: enqueue the deferred jobs that are due."""
        for j in self._deferred:
            j[1] += 1
        while self._deferred and self._deferred[0][1] >= self.delay:
            self._enqueue(self._deferred.popleft()[0])

    def flush(self) -> None:
        while self._deferred:
            self._enqueue(self._deferred.popleft()[0])

    @property
    def deferred(self) -> int:
        return len(self._deferred)

    def state(self) -> dict:
        """Snapshot for the watchdog's record: jobs submitted, waiting to be enqueued, enqueued."""
        return {"jobs": self.jobs, "deferred": [(j[0].step, j[1]) for j in self._deferred],
                "enqueued": self.enqueued, "pending_cpu": len(self._pending), "delay": self.delay}

    def _enqueue(self, plan: StepPlan) -> None:
        B = len(plan.seq_ids)
        TRACKER.mark("head-recv", plan.step, plan.mb, peer=self.last, stream="head")
        self.enqueued += 1
        with torch.cuda.stream(self.stream):
            x = self.runner.x[:B]
            self.tr.recv_head(x, self.last, self.stream)
            tok = self.runner.run(plan, None)
            # device -> host by a copy kernel on the head stream (no shared copy engine)
            pinned, ev = token_ring(self.runner.device).take(tok, self.stream)
        TRACKER.device_mark("head", plan.step, self.stream)
        self.publish(plan, pinned, ev)

    @property
    def pending(self) -> int:
        return len(self._pending)

    def poll(self, block: bool = False) -> None:
        """Run the queued jobs whose hidden states have landed (all of them with ``block``).
        (gloo's ``is_completed`` only turns true once ``wait`` ran, so in practice a CPU job runs
        when this rank is idle or its tokens are wanted: ``run_oldest`` / ``drain``.)"""
        if block:
            self.flush()
        while self._pending and (block or self._pending[0][2].is_completed()):
            self.run_oldest()

    def run_oldest(self) -> None:
        """Wait for the oldest queued job's hidden states and run it.  Never deadlocks: the step
        already left this rank, so only the ranks after it stand between it and the last stage's
        send, and the last stage sends to this rank in step order."""
        plan, buf, work = self._pending.popleft()
        work.wait()
        tok = self.runner.run(plan, buf)
        self.publish(plan, tok.clone(), None)

    def drain(self) -> None:
        self.poll(block=True)
        if self.gpu:
            self.stream.synchronize()
