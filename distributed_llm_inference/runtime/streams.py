"""Every HIP stream a pipeline rank uses, created once, each on a hardware queue of its own.

A rank keeps kernels that wait on OTHER ranks next to its own compute: the RCCL (or IPC) receive
of the next micro-batch, the send of the previous one (it completes only once the peer has posted
its receive), and the rotating LM head's receive (runtime/head.py).  HIP maps streams onto a
small pool of HSA hardware queues per priority (``GPU_MAX_HW_QUEUES``, 4 by default; PyTorch's
stream pool alone creates 32 streams per priority, RCCL two internal streams per communicator),
and the packets of one hardware queue run in order: a waiting kernel - or RCCL's cross-stream
barrier packet behind it - that lands on the compute stream's queue stalls the stage for as long
as the peer takes, and at worst closes a wait cycle between ranks.

So the roles that ever hold such work get DEDICATED streams: created with a (full) CU mask, which
makes HIP give the stream a hardware queue of its own instead of a shared pool queue, while its
kernels still run on every CU.  Roles:

  ``compute``  every stage kernel and graph replay (made the thread's current stream)
  ``send``     stage -> stage+1 sends; on the last stage the rotating head's sends
  ``recv``     stage-1 -> stage receives
  ``head``     the rotating head's receive + projection + sampling (runtime/head.py)
  ``capture``  hipGraph warm-up / capture (idle afterwards)

``DLI_STREAMS=pool`` restores ordinary pool streams (the isolation test shows what that risks).
``tests/test_streams_gpu.py`` proves the isolation on the hardware: a kernel spinning on each
waiting role in turn must not keep any other role - a decode-graph replay on ``compute``, copies
on the others - from completing, with RCCL-style barrier packets queued on pool streams as well.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

ROLES = ("compute", "send", "recv", "head", "capture")
WAITING_ROLES = ("send", "recv", "head")


def _native():
    from .. import ops
    return ops.native()


class RankStreams:
    """The streams of one rank on one device (see module docstring)."""

    def __init__(self, device: torch.device, mode: Optional[str] = None):
        self.device = torch.device(device)
        self.mode = mode or os.environ.get("DLI_STREAMS", "dedicated")
        if self.mode not in ("dedicated", "pool"):
            raise ValueError(f"DLI_STREAMS={self.mode!r}: expected dedicated or pool")
        self.gpu = self.device.type == "cuda"
        self._handles = []
        self.streams: Dict[str, Optional[torch.cuda.Stream]] = {}
        if not self.gpu:
            self.streams = {r: None for r in ROLES}
            return
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.index = idx
        C = _native()
        for role in ROLES:
            if self.mode == "dedicated":
                h = C.stream_create(idx, 1, 0)
                self._handles.append(h)
                self.streams[role] = torch.cuda.ExternalStream(h, device=self.device)
            else:
                self.streams[role] = torch.cuda.Stream(device=self.device)

    def __getattr__(self, role: str):
        if role in ROLES:
            return self.__dict__["streams"][role]
        raise AttributeError(role)

    def activate(self) -> None:
        """Make ``compute`` the calling thread's current stream (torch's current stream is
        per thread: call this in every thread that launches stage work)."""
        if self.gpu:
            torch.cuda.set_stream(self.streams["compute"])

    def describe(self) -> dict:
        d = {"mode": self.mode}
        if self.gpu and self.mode == "dedicated":
            C = _native()
            d["cu_per_stream"] = {r: int(C.stream_cu_count(s.cuda_stream))
                                  for r, s in self.streams.items()}
        return d

    def synchronize(self) -> None:
        if self.gpu:
            for s in self.streams.values():
                s.synchronize()

    def close(self) -> None:
        """Destroy the dedicated streams (after every stream has drained)."""
        if not self._handles:
            return
        self.synchronize()
        if torch.cuda.current_stream(self.device).cuda_stream in self._handles:
            torch.cuda.set_stream(torch.cuda.default_stream(self.device))
        C = _native()
        for h in self._handles:
            C.stream_destroy(h)
        self._handles.clear()


class TokenSlot:
    """One take of a :class:`HostTokenRing`: the host view of the copied tokens and the ring slot
    behind it.  The consumer reads it ONCE with :meth:`tolist`, which also frees the slot; a take
    that is never read (an aborted step) frees its slot with :meth:`release` or when the handle is
    garbage-collected.  ``view`` peeks without freeing (tests)."""

    __slots__ = ("view", "_ledger", "_k")

    def __init__(self, view: torch.Tensor, ledger: "SlotLedger", k: int):
        self.view, self._ledger, self._k = view, ledger, k

    def tolist(self) -> List[int]:
        out = self.view.tolist()
        self.release()
        return out

    def release(self) -> None:
        if self._ledger is not None:
            self._ledger.release(self._k)
            self._ledger = None

    def __len__(self) -> int:
        return self.view.numel()

    def __del__(self):
        self.release()


class SlotLedger:
    """Which slots of a ring are held by an unread :class:`TokenSlot` (round-robin hand-out; a
    hand-out onto a held slot raises instead of overwriting tokens nobody has read yet)."""

    def __init__(self, slots: int):
        self.held = [False] * int(slots)
        self.i = 0

    def acquire(self) -> int:
        k = self.i % len(self.held)
        if self.held[k]:
            raise RuntimeError(f"HostTokenRing overflow: slot {k} is still held by its consumer "
                               f"({self.in_use()} of {len(self.held)} slots unread); size the "
                               "ring with token_ring(device, max_items, slots)")
        self.held[k] = True
        self.i += 1
        return k

    def release(self, k: int) -> None:
        self.held[k] = False

    def in_use(self) -> int:
        return sum(self.held)


class HostTokenRing:
    """Device -> host returns of sampled token ids without a copy engine: a ring of slots in
    coherent, device-mapped host memory written by a copy kernel on the caller's stream
    (``copy_segments``), followed by an event.  (A device -> host ``copy_`` goes through a copy
    queue shared by the process's streams - see csrc/comm/streams.hip - where it can wait behind
    another stream's copy that is ordered after a spinning receive.)

    Slots are released explicitly: :meth:`take` returns a :class:`TokenSlot` that frees its slot
    when the consumer reads it (``tolist()``), releases it, or drops it.  A take that would
    overwrite a slot still held -- more unread takes than ``slots`` -- raises instead of silently
    corrupting tokens; size the ring from the in-flight micro-batch count at init."""

    def __init__(self, device: torch.device, max_items: int, slots: int = 64):
        from .. import ops
        self.C = ops.native()
        self.device = torch.device(device)
        self.item_bytes = (int(max_items) * 4 + 255) // 256 * 256
        self.slots = int(slots)
        self.buf = self.C.HostBuffer(self.item_bytes * self.slots)
        self.view = self.buf.tensor()
        self.ledger = SlotLedger(self.slots)

    def in_use(self) -> int:
        """Slots held by an unread take."""
        return self.ledger.in_use()

    def take(self, tok: torch.Tensor, stream=None):
        """Copy ``tok`` (int32 [B], device) into the next slot on ``stream`` (default: current);
        returns (:class:`TokenSlot`, event recorded after the copy)."""
        if tok.dtype != torch.int32 or not tok.is_contiguous():
            tok = tok.to(torch.int32).contiguous()
        nb = tok.numel() * 4
        if nb > self.item_bytes:
            raise ValueError(f"{tok.numel()} tokens > ring slot of {self.item_bytes // 4}")
        k = self.ledger.acquire()
        off = k * self.item_bytes
        s = stream or torch.cuda.current_stream(self.device)
        if nb:   # (an empty step samples nothing: no copy, just the event)
            self.C.copy_segments(self.buf.dev_ptr + off, tok.data_ptr(), [(0, nb)], s.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(s)
        return TokenSlot(self.view[off: off + nb].view(torch.int32), self.ledger, k), ev


_TOKEN_RINGS: Dict[int, HostTokenRing] = {}
_RETIRED_RINGS: List[HostTokenRing] = []   # replaced rings: views into them may still be read


def token_ring(device: torch.device, max_items: int = 4096, slots: int = 64) -> HostTokenRing:
    """The process-wide token ring of ``device`` (up to ``max_items`` tokens a take, ``slots``
    takes unconsumed at once).  Call it at init with the largest sizes (engine.py does): a later
    request for a larger ring replaces it, keeping the old buffer alive for views into it."""
    device = torch.device(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    r = _TOKEN_RINGS.get(key)
    if r is None or r.item_bytes < max_items * 4 or r.slots < slots:
        if r is not None:
            _RETIRED_RINGS.append(r)
            max_items = max(max_items, r.item_bytes // 4)
            slots = max(slots, r.slots)
        r = HostTokenRing(device, max_items, slots)
        _TOKEN_RINGS[key] = r
    return r


_RANK_STREAMS: Dict[int, RankStreams] = {}


def rank_streams(device: torch.device) -> RankStreams:
    """The process-wide :class:`RankStreams` of ``device`` (created on first use)."""
    device = torch.device(device)
    key = device.index if device.index is not None else (
        torch.cuda.current_device() if device.type == "cuda" else -1)
    rs = _RANK_STREAMS.get(key)
    if rs is None:
        rs = RankStreams(device)
        _RANK_STREAMS[key] = rs
    return rs


# ------------------------------------------------------------------------------ isolation probe
def isolation_matrix(streams: Dict[str, torch.cuda.Stream], waiters, device: torch.device,
                     barrier_streams=(), graph=None, graph_role: str = "compute",
                     window_s: float = 1.5, spin_timeout_s: float = 20.0,
                     host_copies: bool = False, copy_kernels: bool = False
                     ) -> Dict[str, Dict[str, bool]]:
    """For each role in ``waiters``: spin a kernel on it (waiting on a host flag, as a receive
    waits for its peer), queue RCCL-style barrier packets behind it on ``barrier_streams`` (RCCL
    makes an internal stream wait on every send / receive it launches), then queue work on every
    other stream - ``graph`` replayed on ``graph_role``, a small kernel + copy elsewhere - and
    record whether each completed within ``window_s`` while the spinner still spins.  Returns
    ``{waiter: {other: progressed}}``.  The spinner always exits (host release or its deadline).

    ``host_copies``: the waiting stream also queues a host -> device copy behind its spinner (as
    the head stream's staging uploads sit behind its receive), and every other stream's work is
    a host -> device copy too: copies a runtime hands to a copy engine queue shared by the
    process's streams would then wait behind the spinner's copy.  ``copy_kernels``: those copies
    are made the runtime's way instead - a ``copy_segments`` kernel reading device-mapped host
    memory on the stream itself (executor staging, HostTokenRing)."""
    import time
    C = _native()
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    names = list(streams)
    flags = C.HostWords(2)
    out = torch.zeros(len(names), dtype=torch.int32, device=dev)
    src = torch.ones(1 << 16, dtype=torch.float32, device=dev)
    dsts = {n: torch.empty_like(src) for n in names}
    hsrc = torch.ones(1 << 16, dtype=torch.float32).pin_memory() if host_copies else None
    hbuf = C.HostBuffer(1 << 18) if copy_kernels else None

    def host_copy(dst: torch.Tensor, s) -> None:
        if copy_kernels:
            C.copy_segments(dst.data_ptr(), hbuf.dev_ptr, [(0, dst.numel() * 4)], s.cuda_stream)
        else:
            with torch.cuda.stream(s):
                dst.copy_(hsrc, non_blocking=True)
    torch.cuda.synchronize(dev)
    res: Dict[str, Dict[str, bool]] = {}
    for w in waiters:
        flags.set(0, 0)
        flags.set(1, 0)
        C.wait_geq(flags.dev_ptr(0), 1, spin_timeout_s, flags.dev_ptr(1), 1,
                   streams[w].cuda_stream, idx)
        if host_copies:
            host_copy(dsts[w], streams[w])
        ev = torch.cuda.Event()
        ev.record(streams[w])
        for b in barrier_streams:
            b.wait_event(ev)
        evs = {}
        for i, n in enumerate(names):
            if n == w:
                continue
            s = streams[n]
            with torch.cuda.stream(s):
                if graph is not None and n == graph_role:
                    graph.replay()
                else:
                    C.touch(out[i:i + 1], s.cuda_stream)
                    if host_copies:
                        host_copy(dsts[n], s)
                    else:
                        dsts[n].copy_(src, non_blocking=True)
            e = torch.cuda.Event()
            e.record(s)
            evs[n] = e
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < window_s and not all(e.query() for e in evs.values()):
            time.sleep(1e-3)
        res[w] = {n: bool(e.query()) for n, e in evs.items()}
        flags.set(0, 1)   # release the spinner
        streams[w].synchronize()
        torch.cuda.synchronize(dev)
        if flags.get(1) != 0:
            raise RuntimeError(f"isolation probe: spinner on {w!r} hit its deadline")
    return res
