"""Pipeline-parallel execution of stages.

Topology (one node, one process per GPU, launched by ``distribute`` / torchrun):

  rank 0 (driver)  : scheduler + stage 0 (embedding + first layers)
  rank i (0<i<N-1) : middle layers
  rank N-1         : last layers + final norm [+ LM head + sampling kernel]
  every rank       : with the rotating head (runtime/head.py), the vocabulary projection +
                     sampling of the decode steps whose turn it is (step % N)

Per micro-batch step:
  * the driver publishes the step plan (sequence ids, new-token counts, frees, sampling params) on
    a shared-memory broadcast channel (csrc/runtime/shm_channel.cpp) — the *control plane*;
  * hidden states move rank i -> i+1 with RCCL send/recv over xGMI on dedicated streams — the
    *data plane* (parallel/transport.py);
  * the last rank's sampled token ids (B int32) come back to the driver on a second shm channel,
    published by a helper thread once the sampling kernel's event completes, so the last stage
    never stalls its own GPU queue waiting on a device->host copy.
With M >= N micro-batches in flight every stage is busy; the driver plans micro-batch m's next step
as soon as its tokens return (FIFO order == issue order).

The same driver loop also runs an in-process pipeline (:class:`LocalPipeline`) — PP=1 on one GPU,
or several stages in one process for tests / single-GPU rehearsal of PP=2/4/8.
"""
from __future__ import annotations

import collections
import logging
import os
import queue
import sys
import threading
import time
from typing import Deque, Dict, List, Optional, Sequence

import msgpack
import torch
import torch.distributed as dist

from ..runtime.executor import StageExecutor, StepPlan
from ..runtime.faults import FaultInjector, StageStats
from ..runtime.hostclock import HOST
from ..runtime.scheduler import Scheduler
from ..runtime.sequence import SamplingParams, Sequence as Seq
from ..runtime.watchdog import TRACKER, abort_job, wait_event
from .integrity import flush as hop_flush
from .transport import LoopbackTransport, RcclTransport, TorchDistTransport, Transport

log = logging.getLogger(__name__)


def _runtime():
    from .. import _runtime
    return _runtime


# =============================================================================================
# driver loop (shared by the in-process and the multi-process pipeline)
# =============================================================================================
class DriverBase:
    """Owns the scheduler; subclasses implement ``_issue(plan)`` and ``_collect(plan)``."""

    def __init__(self, scheduler: Scheduler):
        self.sched = scheduler
        self.inflight: Deque[StepPlan] = collections.deque()
        self.collect_times: Dict[int, List[float]] = collections.defaultdict(list)
        self.tokens_generated = 0
        self.wait_s = 0.0  # host time blocked on results (the rest of a round is driver work)
        self._tok_wait_ms = 0.0  # of the current _collect: blocked on the tokens
        self.streams = None  # runtime.streams.RankStreams of a multi-process rank

    def activate_streams(self) -> None:
        """Make this rank's compute stream current in the calling thread (a serving loop that
        drives the pipeline from its own thread calls this first)."""
        if self.streams is not None:
            self.streams.activate()

    # -- to implement
    def _issue(self, plan: StepPlan) -> None:
        raise NotImplementedError

    def _collect(self, plan: StepPlan) -> List[int]:
        raise NotImplementedError

    def _broadcast_control(self, kind: str) -> None:
        pass

    # -- loop
    def _collect_front(self) -> None:
        p = self.inflight.popleft()
        t0 = time.perf_counter()
        self._tok_wait_ms = 0.0
        toks = self._collect(p)
        now = time.perf_counter()
        self.wait_s += now - t0
        self.collect_times[p.mb].append(now)
        self.tokens_generated += len(toks)
        self.sched.on_tokens(p.mb, toks, now)
        # host phases (runtime/hostclock.py): blocked on the tokens vs reading / applying them
        HOST.add("tokens_wait", self._tok_wait_ms)
        HOST.add("tokens", (time.perf_counter() - t0) * 1e3 - self._tok_wait_ms)

    def round(self) -> bool:
        """Give every micro-batch one step (collecting results as needed).  Returns False when
        there is nothing left to do."""
        progressed = False
        for mb in range(self.sched.M):
            while self.sched.inflight[mb] is not None:
                self._collect_front()
            t0 = time.perf_counter()
            plan = self.sched.plan(mb)
            HOST.since("plan", t0)
            if plan is None:
                continue
            self._issue(plan)
            if plan.seq_ids:
                self.inflight.append(plan)
            progressed = True
        if not progressed:
            if self.inflight:
                self._collect_front()
                return True
            return False
        return True

    def drain(self) -> None:
        while self.inflight:
            self._collect_front()

    def run_until_done(self) -> List[Seq]:
        while self.round():
            pass
        self.drain()
        return self.sched.pop_finished()

    def generate(self, prompts: Sequence[Sequence[int]], params: Optional[SamplingParams] = None,
                 eos_token_id: Optional[int] = None) -> List[Seq]:
        params = params or SamplingParams()
        seqs = [Seq(list(p), params) for p in prompts]
        for s in seqs:
            self.sched.add(s)
        done = {s.seq_id: s for s in self.run_until_done()}
        return [done.get(s.seq_id, s) for s in seqs]

    def barrier(self) -> None:
        """Drain everything in flight on every stage and synchronise all ranks."""
        self.drain()
        self._broadcast_control("barrier")

    def stop(self) -> None:
        self.drain()
        self._broadcast_control("stop")


def _sample_tokens_to_host(out: torch.Tensor):
    """Async D2H of sampled tokens; returns (host tensor, event).  On the GPU a copy kernel on
    the current stream writes a device-mapped host ring slot (runtime/streams.py
    HostTokenRing): no copy engine shared with the other streams."""
    if out.is_cuda:
        from ..runtime.streams import token_ring
        return token_ring(out.device).take(out)
    return out.clone(), None


# =============================================================================================
# in-process pipeline
# =============================================================================================
class LocalPipeline(DriverBase):
    """All stages in this process (PP=1, or PP>1 loopback on one device / CPU)."""

    def __init__(self, executors: List[StageExecutor], scheduler: Scheduler,
                 lookahead: bool = True):
        super().__init__(scheduler)
        self.executors = executors
        self._results: Dict[int, tuple] = {}
        # one-step lookahead keeps a single micro-batch's GPU queue non-empty while the host
        # consumes the previous step's tokens (see Scheduler.plan_lookahead)
        self.lookahead = lookahead and scheduler.M == 1
        self._last_tokens: Optional[torch.Tensor] = None

    def _issue(self, plan: StepPlan) -> None:
        x = None
        for i, ex in enumerate(self.executors):
            x = ex.execute(plan, x, token_src=self._last_tokens if i == 0 else None)
        if plan.seq_ids:
            # sampled tokens stay referenced on the device for a lookahead step
            self._last_tokens = x
            self._results[plan.step] = _sample_tokens_to_host(x)

    def round(self) -> bool:
        s = self.sched
        if not self.lookahead or s.inflight[0] is None:
            return super().round()
        la = s.plan_lookahead(0)
        if la is not None:
            self._issue(la)
            self.inflight.append(la)
        self._collect_front()  # the older step; its successor (if any) is already queued
        return True

    def _collect(self, plan: StepPlan) -> List[int]:
        pinned, ev = self._results.pop(plan.step)
        if ev is not None:
            t0 = time.perf_counter()
            ev.synchronize()
            self._tok_wait_ms += (time.perf_counter() - t0) * 1e3
        return pinned.tolist()

    def _broadcast_control(self, kind: str) -> None:
        if any(ex.device.type == "cuda" for ex in self.executors):
            torch.cuda.synchronize()

    def close(self) -> None:
        pass


# =============================================================================================
# multi-process pipeline
# =============================================================================================
class _Channels:
    """Shared-memory control (driver -> all) and token (rank r -> driver) channels.  Tokens come
    from the last rank only, or from every rank r >= 1 when the LM head rotates
    (runtime/head.py): ``toks[r]`` on the driver, ``tok`` on a producing rank."""

    def __init__(self, job: str, rank: int, world: int, slot_size: int = 1 << 20,
                 head_rotation: bool = False):
        R = _runtime()
        self.ctrl = None
        self.tok = None
        self.toks: Dict[int, object] = {}
        if world == 1:
            return
        ctrl_name = f"/dli_{job}_ctrl"
        producers = list(range(1, world)) if head_rotation else [world - 1]
        if rank == 0:
            self.ctrl = R.ShmChannel(ctrl_name, -1, 64, slot_size, world - 1, True)
            for r in producers:
                self.toks[r] = R.ShmChannel(f"/dli_{job}_tok{r}", 0, 64, slot_size, 1, False, 120.0)
            self.tok = self.toks[world - 1]
        else:
            self.ctrl = R.ShmChannel(ctrl_name, rank - 1, 64, slot_size, world - 1, False, 120.0)
            if rank in producers:
                self.tok = R.ShmChannel(f"/dli_{job}_tok{rank}", -1, 64, slot_size, 1, True)

    def unlink(self) -> None:
        """Drop the /dev/shm names once every rank has attached (mappings stay valid)."""
        for ch in [self.ctrl, self.tok] + list(self.toks.values()):
            if ch is not None:
                ch.unlink()


class DistributedDriver(DriverBase):
    """Rank 0 of a multi-process pipeline."""

    def __init__(self, executor: StageExecutor, scheduler: Scheduler, transport: Transport,
                 channels: _Channels, world: int, ctrl_group=None, timeout: float = 120.0,
                 policy=None, heads=None):
        super().__init__(scheduler)
        self.ex = executor
        self.tr = transport
        self.ch = channels
        self.world = world
        self.group = ctrl_group
        self.timeout = timeout
        self.faults = FaultInjector(0)
        self.stats = StageStats(0, executor.device)
        self.stats.transport = transport
        self.snapshots: List[dict] = []   # StageStats.snapshot() at every barrier
        self.policy = policy              # runtime.head.HeadPolicy (None: head on the last rank)
        self.heads = heads                # runtime.head.HeadJobs of this rank (rotating head)
        self._head_results: Dict[int, tuple] = {}

    def _head_rank(self, plan: StepPlan) -> int:
        return self.policy.rank_for(plan) if self.policy is not None else self.world - 1

    def publish_local(self, plan: StepPlan, pinned, ev) -> None:
        """HeadJobs callback: tokens of a step whose head ran on this (the driver's) rank."""
        self._head_results[plan.step] = (pinned, ev)

    def _issue(self, plan: StepPlan) -> None:
        t = time.perf_counter()
        TRACKER.mark("ctrl-send", plan.step, plan.mb)
        self.ch.ctrl.send(msgpack.packb(plan.to_wire()), self.timeout)
        t = HOST.since("ctrl", t)
        if plan.seq_ids and self.faults.active:
            self.faults.on_step()
        tok = self.stats.begin(self.faults.delay_ms) if plan.seq_ids else None
        TRACKER.mark("execute", plan.step, plan.mb, stream="compute")
        out = self.ex.execute(plan, None)   # charges stage / staging_wait / launch itself
        self.stats.end(tok)
        t = time.perf_counter()
        if plan.seq_ids:
            _device_mark(self.ex, "compute", plan.step)
            TRACKER.mark("send", plan.step, plan.mb, peer=1, stream="send")
            self.tr.send(out, 1)
            _device_mark(self.ex, "send", plan.step)
            t = HOST.since("send", t)
            if self.heads is not None:
                self.heads.tick()
                if self._head_rank(plan) == 0:
                    self.heads.submit(plan)
        if self.heads is not None:
            self.heads.poll()
            HOST.since("head", t)

    def _collect(self, plan: StepPlan) -> List[int]:
        hr = self._head_rank(plan)
        TRACKER.mark("collect", plan.step, plan.mb, peer=hr)
        if hr == 0:
            t0 = time.perf_counter()
            while plan.step not in self._head_results:
                self.heads.poll(block=True)   # (enqueues any deferred GPU job first)
            pinned, ev = self._head_results.pop(plan.step)
            wait_event(ev, "local head tokens", plan.step, plan.mb)
            self._tok_wait_ms += (time.perf_counter() - t0) * 1e3
            return pinned.tolist()
        t0 = time.perf_counter()
        with TRACKER.waiting("tokens", plan.step, plan.mb, peer=hr):
            raw = self.ch.toks.get(hr, self.ch.tok).recv(self.timeout)
        self._tok_wait_ms += (time.perf_counter() - t0) * 1e3
        msg = msgpack.unpackb(raw)
        if msg["step"] != plan.step:
            raise RuntimeError(f"token stream of rank {hr} out of order: got step {msg['step']}, "
                               f"want {plan.step}")
        return list(msg["tokens"])

    def _broadcast_control(self, kind: str) -> None:
        self.ch.ctrl.send(msgpack.packb({"kind": kind}), self.timeout)
        if self.ex.device.type == "cuda":
            torch.cuda.synchronize()
        if kind == "barrier":
            hop_flush(self.tr)   # the warm-up's payload digests, checked once (integrity.py)
            dist.barrier(group=self.group)
            self.snapshots.append(self.stats.snapshot())

    def close(self) -> None:
        """After :meth:`stop`: wait for every rank to finish, then tear down the RCCL
        communicators explicitly (never from an interpreter-exit destructor)."""
        dist.barrier(group=self.group)
        self.tr.close()


class StageFollower:
    """Ranks 1..N-1: execute plans as they are published."""

    def __init__(self, executor: StageExecutor, transport: Transport, channels: _Channels,
                 rank: int, world: int, ctrl_group=None, timeout: float = 120.0, policy=None,
                 heads=None):
        self.ex, self.tr, self.ch = executor, transport, channels
        self.rank, self.world = rank, world
        self.group = ctrl_group
        self.timeout = timeout
        self.ctrl_timeout = float(os.environ.get("DLI_CTRL_TIMEOUT_S", "0"))
        self.is_last = rank == world - 1
        self.barrier_times: List[float] = []
        self.snapshots: List[dict] = []   # StageStats.snapshot() at every barrier
        self.faults = FaultInjector(rank)
        self.stats = StageStats(rank, executor.device)
        self.stats.transport = transport
        self.policy = policy              # runtime.head.HeadPolicy (None: head on the last rank)
        self.heads = heads                # runtime.head.HeadJobs (rotating head, non-last ranks)
        self._pub_q: "queue.Queue" = queue.Queue()
        self._pub_thread = None
        self.streams = None               # runtime.streams.RankStreams (GPU ranks)
        if self.is_last or heads is not None:
            self._start_publisher()

    def _start_publisher(self) -> None:
        if self._pub_thread is None:
            self._pub_thread = threading.Thread(target=self._publisher, name="dli-publisher",
                                                daemon=True)
            self._pub_thread.start()

    def publish(self, plan: StepPlan, pinned, ev) -> None:
        """Queue a step's sampled tokens for the driver (HeadJobs callback / last stage)."""
        self._pub_q.put((plan.step, plan.mb, pinned, ev))

    def _head_rank(self, plan: StepPlan) -> int:
        return self.policy.rank_for(plan) if self.policy is not None else self.world - 1

    def _next_msg(self) -> bytes:
        """The next control message; a CPU rank with queued head jobs keeps running them while it
        waits (the driver may be waiting for exactly those tokens).  Waiting for the driver is
        idle time, not a stall (a serving pipeline can sit idle for hours): no deadline unless
        ``DLI_CTRL_TIMEOUT_S`` sets one; a failed driver reaches this rank through the watchdog
        (runtime/watchdog.py) or the launcher."""
        TRACKER.mark("ctrl-wait")
        idle = self.ctrl_timeout
        if self.heads is None:
            return self.ch.ctrl.recv(idle)
        if self.heads.gpu:
            if self.heads.deferred and not self.ch.ctrl.poll():
                self.heads.flush()   # idle: the driver may be waiting for these tokens
            return self.ch.ctrl.recv(idle)
        t0 = time.perf_counter()
        while not self.ch.ctrl.poll():
            if self.heads.pending:
                self.heads.run_oldest()   # idle: the driver may be waiting for these tokens
                continue
            if idle > 0 and time.perf_counter() - t0 > idle:
                return self.ch.ctrl.recv(1e-3)   # raises the channel's TimeoutError
            time.sleep(2e-4)
        return self.ch.ctrl.recv(idle)

    # ring of receive buffers: the receive of micro-batch m+1 only waits until the compute that
    # READ the slot (two steps earlier) is done, not for everything queued on the compute stream
    def _recv_slot(self, T: int):
        if not hasattr(self, "_rbufs"):
            n = 3
            H = self.ex.spec.hidden_size
            self._rbufs = [torch.empty(self.ex.max_tokens, H, dtype=torch.bfloat16,
                                       device=self.ex.device) for _ in range(n)]
            self._rfree = [None] * n
            self._rslot = 0
        self._rslot = (self._rslot + 1) % len(self._rbufs)
        return self._rbufs[self._rslot][:T], self._rfree[self._rslot]

    def _release_slot(self) -> None:
        if self.ex.device.type == "cuda":
            ev = self._rfree[self._rslot] or torch.cuda.Event()
            ev.record()
            self._rfree[self._rslot] = ev

    def _publisher(self) -> None:
        while True:
            item = self._pub_q.get()
            if item is None:
                self._pub_q.task_done()
                return
            step, mb, pinned, ev = item
            wait_event(ev, "sampled tokens on the device", step, mb)
            TRACKER.mark("publish", step, mb, peer=0)
            self.ch.tok.send(msgpack.packb({"step": step, "mb": mb, "tokens": pinned.tolist()}),
                             self.timeout)
            self._pub_q.task_done()

    def run(self) -> None:
        try:
            self._run()
        except BaseException as e:
            import traceback
            traceback.print_exc()
            abort_job(f"{type(e).__name__}: {e}")   # every rank leaves, with its last op
            raise

    def _run(self) -> None:
        while True:
            t = time.perf_counter()
            raw = self._next_msg()
            t = HOST.since("ctrl_wait", t)
            msg = msgpack.unpackb(raw)
            kind = msg.get("kind", "run")
            if kind == "stop":
                break
            if kind == "barrier":
                if self.heads is not None:
                    self.heads.drain()
                if self.ex.device.type == "cuda":
                    torch.cuda.synchronize()
                self._pub_q.join()
                hop_flush(self.tr)   # the warm-up's payload digests, checked once (integrity.py)
                dist.barrier(group=self.group)
                self.barrier_times.append(time.perf_counter())
                self.snapshots.append(self.stats.snapshot())
                continue
            plan = StepPlan.from_wire(msg)
            t = HOST.since("unpack", t)
            if not plan.seq_ids:
                self.ex.execute(plan, None)  # frees only
                continue
            hr = self._head_rank(plan)
            buf, free_ev = self._recv_slot(plan.num_tokens)
            TRACKER.mark("recv", plan.step, plan.mb, peer=self.rank - 1, stream="recv")
            x = self.tr.recv(buf, self.rank - 1, free_event=free_ev)
            _device_mark(self.ex, "recv", plan.step)
            HOST.since("recv", t)
            if self.faults.active:
                self.faults.on_step()
            tok = self.stats.begin(self.faults.delay_ms)
            TRACKER.mark("execute", plan.step, plan.mb, stream="compute")
            out = self.ex.execute(plan, x, project=(hr == self.rank))
            self.stats.end(tok)
            t = time.perf_counter()
            self._release_slot()
            _device_mark(self.ex, "compute", plan.step)
            if self.is_last:
                if hr == self.rank:
                    pinned, ev = _sample_tokens_to_host(out)
                    self.publish(plan, pinned, ev)
                else:   # rotating head: normed hidden states to the rank whose turn it is
                    TRACKER.mark("send_head", plan.step, plan.mb, peer=hr, stream="send")
                    self.tr.send_head(out, hr)
                    _device_mark(self.ex, "send", plan.step)
            else:
                TRACKER.mark("send", plan.step, plan.mb, peer=self.rank + 1, stream="send")
                self.tr.send(out, self.rank + 1)
                _device_mark(self.ex, "send", plan.step)
                if self.heads is not None:
                    self.heads.tick()
                    if hr == self.rank:
                        self.heads.submit(plan)
            t = HOST.since("send", t)
            if self.heads is not None:
                self.heads.poll()
                HOST.since("head", t)
        if self.heads is not None:
            self.heads.drain()
        if self._pub_thread is not None:
            self._pub_q.join()
            self._pub_q.put(None)
            self._pub_thread.join()
        if self.ex.device.type == "cuda":
            torch.cuda.synchronize()

    def close(self) -> None:
        """Counterpart of :meth:`DistributedDriver.close` (call after :meth:`run` returns)."""
        dist.barrier(group=self.group)
        self.tr.close()


def _device_mark(ex, role: str, step: int) -> None:
    """Device progress mark of ``role``'s stream after this step's work (watchdog record)."""
    if TRACKER._words is None:
        return
    from ..runtime.streams import rank_streams
    stream = (torch.cuda.current_stream(ex.device) if role == "compute"
              else rank_streams(ex.device).streams.get(role))
    TRACKER.device_mark(role, step, stream)


def device_identity(device: torch.device) -> str:
    """A string naming the physical device ``device`` is on, equal for two processes exactly when
    they drive the same GPU: host name + PCI domain:bus:device + the device UUID (CPU ranks: the
    host and process)."""
    import socket
    host = socket.gethostname()
    if device.type != "cuda":
        return f"{host}/cpu/{os.getpid()}"
    p = torch.cuda.get_device_properties(device)
    return f"{host}/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}/{p.uuid}"


def choose_data_plane(kind: str, device_ids: Sequence[str]) -> tuple:
    """``(plane, reason)`` for a ``DLI_TRANSPORT`` kind and every stage's :func:`device_identity`.

    ``rccl-or-ipc`` (the default) is RCCL whenever every stage has a GPU of its own - then an RCCL
    failure fails the job loudly, it never silently becomes another transport - and the IPC device
    transport only when two stages share a GPU (RCCL refuses two ranks on one device; that is the
    one-GPU rehearsal of a pipeline).  Every other kind is taken as given: ``rccl`` (strict),
    ``rccl-or-host`` (RCCL, agreed fallback to host staging), ``ipc``, ``host``."""
    if kind != "rccl-or-ipc":
        return kind, ""
    seen: Dict[str, List[int]] = collections.defaultdict(list)
    for r, d in enumerate(device_ids):
        seen[d].append(r)
    shared = [rs for rs in seen.values() if len(rs) > 1]
    if shared:
        return "ipc", f"stages share a GPU (ranks {shared}): RCCL needs one device per rank"
    return "rccl", ""


def _exchange_device_ids(store, key: str, rank: int, world: int, device: torch.device,
                         timeout_s: float) -> List[str]:
    store.set(f"{key}/{rank}", device_identity(device))
    keys = [f"{key}/{r}" for r in range(world)]
    deadline = time.monotonic() + timeout_s
    while not all(_store_has(store, k) for k in keys):
        if time.monotonic() > deadline:
            missing = [r for r, k in enumerate(keys) if not _store_has(store, k)]
            raise TransportInitError(f"[rank {rank}] ranks {missing} never published their "
                                     f"device within {timeout_s:.0f} s")
        time.sleep(0.002)
    return [store.get(k).decode() for k in keys]


def make_transport(rank: int, world: int, device: torch.device, job: str = "0",
                   rccl_timeout_s: float = 120.0, rank_offset: int = 0,
                   head_pairs: bool = False, streams=None, max_bytes: int = 0,
                   head_bytes: int = 0) -> Transport:
    """The data plane of one pipeline replica (``DLI_TRANSPORT``, see :func:`choose_data_plane`):

    * RCCL P2P on GPUs, one 2-rank communicator per stage pair (+ head pairs) — the production
      path whenever every stage has its own GPU;
    * the IPC device transport (parallel/ipc_transport.py: cross-process device memory with
      spinning device waits, the production stream structure and the rotating head) when stages
      share a GPU — chosen by comparing every rank's published PCI device, never as the fallback of
      a failed RCCL bring-up on distinct GPUs;
    * host staging through gloo (``DLI_TRANSPORT=host`` / ``rccl-or-host``, explicit opt-ins);
    * gloo on the CPU (tests).

    RCCL initialisation is agreed on by all ranks (:func:`_agree`): every rank publishes whether
    its communicators came up (a failure or a peer that never arrives ends in a timeout, not a
    hang), and if ANY rank failed, EVERY rank raises :class:`TransportInitError` with the failing
    ranks and the error (``rccl-or-host``: every rank switches to host staging instead).

    ``rank`` / ``world`` are the stage index and stage count of ONE pipeline replica; with several
    replicas (data parallel) ``rank_offset`` is the replica's first global rank and ``job`` names
    the replica, so every replica gets its own RCCL pair communicators."""
    tr = _make_transport(rank, world, device, job, rccl_timeout_s, rank_offset, head_pairs,
                         streams, max_bytes, head_bytes)
    if world > 1:
        from ..runtime.faults import raw_store
        from .integrity import attach
        attach(tr, raw_store(), rank, job)
    return tr


def _make_transport(rank, world, device, job, rccl_timeout_s, rank_offset, head_pairs, streams,
                    max_bytes, head_bytes) -> Transport:
    if world == 1:
        return LoopbackTransport(1)
    from .transport import transport_kind
    kind = transport_kind(device)
    if kind == "gloo":
        return TorchDistTransport(rank_offset=rank_offset)
    from ..runtime.faults import raw_store
    if kind == "rccl-or-ipc":
        ids = _exchange_device_ids(raw_store(), f"dli_dev_{job}", rank, world, device,
                                   rccl_timeout_s)
        kind, why = choose_data_plane(kind, ids)
        if kind == "ipc" and max_bytes <= 0:
            raise ValueError(f"{why}; the IPC transport needs the largest message size (max_bytes)")
        if kind == "ipc":
            print(f"[rank {rank}] data plane: IPC device transport ({why})", file=sys.stderr,
                  flush=True)
            tr = _ipc(raw_store(), rank, world, device, streams, max_bytes, head_bytes, job,
                      head_pairs)
            tr.fallback_from = why
            return tr
    if kind == "ipc":
        if max_bytes <= 0:
            raise ValueError("DLI_TRANSPORT=ipc needs the largest message size (max_bytes)")
        return _ipc(raw_store(), rank, world, device, streams, max_bytes, head_bytes, job,
                    head_pairs)
    if kind == "host":
        from .transport import HostStagedTransport
        return HostStagedTransport(rank_offset=rank_offset)
    # kind in ("rccl", "rccl-or-host")
    store = raw_store()
    prefix = f"dli_rccl_{job}"
    tr, err = None, ""
    try:
        tr = RcclTransport(store, rank, world, device, prefix=prefix, timeout_s=rccl_timeout_s,
                           head_pairs=head_pairs, streams=streams)
    except Exception as e:  # noqa: BLE001 - reported and agreed on below
        err = repr(e)
        store.set(f"{prefix}/err/{rank}", err[:2000])
        store.set(f"{prefix}/failed", f"rank {rank}: {err[:500]}")   # peers stop early
    mine = _publish_ok(store, f"{prefix}/ok/{rank}", tr is not None)
    if not mine and tr is not None:   # declared dead by a peer's deadline before answering
        store.set(f"{prefix}/failed", f"rank {rank}: answered after the agreement deadline")
    ok = _agree(store, prefix, world, rank, rccl_timeout_s)
    if all(ok):
        return tr
    if tr is not None:
        tr.abort()
    bad = [r for r, o in enumerate(ok) if not o]
    errs = {r: store.get(f"{prefix}/err/{r}").decode(errors="replace") for r in bad
            if r != rank and _store_has(store, f"{prefix}/err/{r}")}
    if err:
        errs[rank] = err
    msg = (f"[rank {rank}] RCCL transport unavailable: communicators failed on ranks {bad}"
           f" (device {device}, HSA_ENABLE_IPC_MODE_LEGACY="
           f"{os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '<unset>')}); errors: {errs}")
    print(msg, file=sys.stderr, flush=True)
    if kind != "rccl-or-host":
        raise TransportInitError(msg)
    log.warning(msg + "; DLI_TRANSPORT=rccl-or-host: falling back to host-staged transport")
    from .transport import HostStagedTransport
    return HostStagedTransport(rank_offset=rank_offset)


def _ipc(store, rank, world, device, streams, max_bytes, head_bytes, job, head_pairs):
    from .ipc_transport import IpcTransport
    if streams is None:
        from ..runtime.streams import rank_streams
        streams = rank_streams(device)
    return IpcTransport(store, rank, world, device, streams, max_bytes, head_bytes,
                        prefix=f"dli_ipc_{job}", head_pairs=head_pairs)


def _publish_ok(store, key: str, ok: bool) -> bool:
    """Publish this rank's bring-up outcome unless a peer already declared it failed (a
    ``compare_set`` on the missing key, see :func:`_agree`); returns the value that stands."""
    return _compare_set(store, key, "1" if ok else "0") == b"1"


def _compare_set(store, key: str, value: str) -> bytes:
    """Set ``key`` to ``value`` if it does not exist; returns the value the key holds."""
    return bytes(store.compare_set(key, "", value))


def _agree(store, prefix: str, world: int, rank: int, timeout_s: float) -> List[bool]:
    """Every rank's RCCL bring-up outcome; every rank decides the same.

    * no failure published and every rank answered: their answers;
    * a failure published (by a failing rank, or by a rank whose deadline passed): each rank that
      has not answered is declared failed with a ``compare_set`` of its key to "0" - whichever
      of that and the rank's own ``compare_set`` comes first stands, for every reader, so a late
      rank can never turn "1" after another rank decided without it."""
    fail_key = f"{prefix}/failed"
    keys = [f"{prefix}/ok/{r}" for r in range(world)]
    deadline = time.monotonic() + timeout_s
    failed_at: Optional[float] = None
    while True:
        if failed_at is None and _store_has(store, fail_key):
            failed_at = time.monotonic()
        # after a failure, live ranks answer within milliseconds (their bring-up stops at the
        # published failure): give them a short grace so the reported set is the ranks that
        # really failed, then settle every missing answer as failed - sticky, the same everywhere
        if failed_at is not None and (all(_store_has(store, k) for k in keys)
                                      or time.monotonic() - failed_at > min(timeout_s, 5.0)):
            return [_compare_set(store, k, "0") == b"1" for k in keys]
        if failed_at is None and all(_store_has(store, k) for k in keys):
            vals = [store.get(k) == b"1" for k in keys]
            if all(vals):
                return vals
            # a "0" is always preceded by its rank's failure key: decide on the sticky path
            continue
        if time.monotonic() > deadline:
            missing = [r for r, k in enumerate(keys) if not _store_has(store, k)]
            store.set(f"{prefix}/err/{missing[0]}", f"no answer within {timeout_s:.0f} s")
            store.set(fail_key, f"rank {rank}: ranks {missing} never answered")
        time.sleep(0.002)


class TransportInitError(RuntimeError):
    """The RCCL data plane could not be brought up on every rank."""


def _store_has(store, key: str) -> bool:
    try:
        return bool(store.check([key]))
    except Exception:  # noqa: BLE001
        return False
