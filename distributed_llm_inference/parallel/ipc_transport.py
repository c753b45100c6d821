"""Device-side P2P transport over cross-process GPU memory (HIP IPC) with device signals.

RCCL refuses two ranks on one device, so on a one-GPU box the multi-process pipeline used to run
over the host-staged transport - which blocks the HOST on every receive and cannot carry the
rotating LM head.  That left the production stream structure untested: kernels that wait on
other ranks sitting on side streams next to compute, the head's deferred receive + graph replay on
its own stream.  This transport reproduces that structure exactly, on one GPU or several:

* every directed channel (stage r -> r+1, and last stage -> r for the rotating head) owns
  ``slots`` message buffers in the RECEIVER's memory plus a ``ready`` word per slot next to them,
  and a ``free`` word per slot in the SENDER's memory; both ends open the other's allocation with
  ``hipIpcOpenMemHandle`` (handles exchanged through the job's TCP store);
* message n uses slot s = n % slots, round u = n // slots.  Sender, on its send stream (after the
  compute that produced the data): wait ``free[s] >= u`` -> copy into the peer's slot -> release
  ``ready[s] = u + 1``.  Receiver, on its receive (or head) stream: wait ``ready[s] >= u + 1`` ->
  copy out -> release ``free[s] = u + 1`` in the sender's memory.  The copies are kernels on the
  same stream, never hipMemcpyAsync: a memcpy runs on a copy queue the process's streams share
  (measured, profiles/streams/copies_*.json), where one copy held behind a spinning wait blocks
  every other stream's copies.  (The 8-rank rehearsal's stall in its third decode round came
  from exactly that coupling - the executor's host -> device step uploads stuck behind the head
  stream's; those are copy kernels now as well, runtime/executor.py _Staging);
* the waits are spinning kernels (csrc/comm/streams.hip), like RCCL's: they hold their stream -
  and, if it were shared, that stream's hardware queue - until the peer arrives.  That is the
  point: the GPU tests run the real HeadJobs / executor stream schedule against them.  Each wait
  has a deadline; an expired one leaves a code in a host-mapped status word and :meth:`check`
  raises with the channel and message number, instead of a wave spinning forever.

Not the production data plane on a multi-GPU node (RcclTransport is), but it works across GPUs
as well (the copy then crosses xGMI).
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Tuple

import torch

from .transport import Transport

_FLAG_BYTES = 256   # ready / free words region (64 slots max)


class _Channel:
    def __init__(self, cid: int, kind: str, src: int, dst: int, slot_bytes: int, slots: int):
        self.cid, self.kind, self.src, self.dst = cid, kind, src, dst
        self.slot_bytes, self.slots = slot_bytes, slots
        self.n = 0            # messages issued on this end
        self.data = None      # receiver's slots (owned by the receiver, opened by the sender)
        self.peer_flags = None  # the other end's flag words (ready at the receiver / free at the sender)
        self.own = None       # this end's own allocation (kept alive)

    def describe(self) -> str:
        return f"{self.kind} {self.src}->{self.dst}"


_PROG = 6   # progress words per channel (see IpcTransport.__init__)


class IpcTransport(Transport):
    """See module docstring.  ``max_bytes``: largest stage message (max tokens x hidden x 2)."""

    supports_head = True

    def __init__(self, store, rank: int, world: int, device: torch.device, streams,
                 max_bytes: int, head_bytes: int = 0, prefix: str = "dli_ipc",
                 timeout_s: float = 120.0, slots: int = 2, head_pairs: bool = False):
        from .. import ops
        C = ops.native()
        self.C = C
        self.rank, self.world, self.device = rank, world, device
        self.idx = device.index if device.index is not None else torch.cuda.current_device()
        self.streams = streams
        self.send_stream = streams.send
        self.recv_stream = streams.recv
        self.timeout_s = float(os.environ.get("DLI_P2P_TIMEOUT_S", timeout_s))
        # host-mapped words: [0] code of the first expired wait (0 = none), [1] abort (nonzero
        # ends every pending device wait and stops every release), then 6 progress words per
        # channel, written by the device: sender (credit wait entered, credit seen, ready
        # released), receiver (ready wait entered, ready seen, credit released) - a stuck
        # pipeline's record names the wait each stream reached and never passed, read without
        # any GPU operation (releases stop after a failure, so the words stay frozen there)
        self.status = C.HostWords(2 + _PROG * 64)
        self.prefix = prefix
        self._ch: Dict[Tuple[str, int, int], _Channel] = {}
        edges: List[Tuple[str, int, int, int]] = [("stage", r, r + 1, max_bytes)
                                                   for r in range(world - 1)]
        if head_pairs and world > 1:
            edges += [("head", world - 1, r, head_bytes or max_bytes) for r in range(world - 1)]
        # every rank publishes its side first, then opens the peers' (the store's get blocks)
        mine = []
        for cid, (kind, src, dst, nbytes) in enumerate(edges):
            if rank not in (src, dst):
                continue
            slot_bytes = (int(nbytes) + 255) // 256 * 256
            ch = _Channel(cid, kind, src, dst, slot_bytes, slots)
            if rank == dst:   # receiver: slots + ready words
                ch.own = C.IpcBuffer(slot_bytes * slots + _FLAG_BYTES, self.idx)
                store.set(f"{prefix}/c{cid}/rx", bytes(ch.own.handle()))
            else:             # sender: free words
                ch.own = C.IpcBuffer(_FLAG_BYTES, self.idx)
                store.set(f"{prefix}/c{cid}/tx", bytes(ch.own.handle()))
            self._ch[(kind, src, dst)] = ch
            mine.append(ch)
        for ch in mine:
            if rank == ch.dst:
                h = store.get(f"{prefix}/c{ch.cid}/tx")
                ch.peer_flags = C.IpcBuffer(bytes(h), _FLAG_BYTES, self.idx)      # sender's free
            else:
                h = store.get(f"{prefix}/c{ch.cid}/rx")
                ch.data = C.IpcBuffer(bytes(h), ch.slot_bytes * ch.slots + _FLAG_BYTES, self.idx)
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ protocol
    def _flag(self, buf, offset_bytes: int, s: int) -> int:
        return buf.ptr + offset_bytes + 4 * s

    def _prog(self, ch: _Channel, k: int) -> int:
        return self.status.dev_ptr(2 + _PROG * ch.cid + k)

    def _signal(self, ptr: int, value: int, stream, progress: int) -> None:
        self.C.signal(ptr, value, stream.cuda_stream, progress, self.status.dev_ptr(0),
                      self.status.dev_ptr(1))

    def _wait(self, ptr: int, target: int, code: int, stream, progress: int = 0) -> None:
        self.C.wait_geq(ptr, target, self.timeout_s, self.status.dev_ptr(0), code,
                        stream.cuda_stream, self.idx, self.status.dev_ptr(1), progress)

    def _code(self, ch: _Channel, recv: bool) -> int:
        return 1 + 2 * ch.cid + (1 if recv else 0)

    def _send_on(self, ch: _Channel, t: torch.Tensor, stream) -> None:
        if not t.is_contiguous():   # callers make it contiguous before ordering the streams
            raise ValueError("IPC send buffers must be contiguous")
        nb = t.numel() * t.element_size()
        if nb > ch.slot_bytes:
            raise ValueError(f"IPC {ch.describe()}: message of {nb} B > slot of {ch.slot_bytes} B")
        s, u = ch.n % ch.slots, ch.n // ch.slots
        ch.n += 1
        free_ptr = self._flag(ch.own, 0, s)                               # my free words
        ready_ptr = self._flag(ch.data, ch.slot_bytes * ch.slots, s)      # peer's ready words
        with torch.cuda.stream(stream):
            self._wait(free_ptr, u, self._code(ch, False), stream, self._prog(ch, 0))
            # copy KERNEL on this stream (not hipMemcpyAsync: see csrc/comm/streams.hip dev_copy)
            self.C.dev_copy(ch.data.ptr + s * ch.slot_bytes, t.data_ptr(), nb, stream.cuda_stream)
            self._signal(ready_ptr, u + 1, stream, self._prog(ch, 2))

    def _recv_on(self, ch: _Channel, t: torch.Tensor, stream) -> None:
        if not t.is_contiguous():
            raise ValueError("IPC receive buffers must be contiguous")
        nb = t.numel() * t.element_size()
        if nb > ch.slot_bytes:
            raise ValueError(f"IPC {ch.describe()}: message of {nb} B > slot of {ch.slot_bytes} B")
        s, u = ch.n % ch.slots, ch.n // ch.slots
        ch.n += 1
        ready_ptr = self._flag(ch.own, ch.slot_bytes * ch.slots, s)       # my ready words
        free_ptr = self._flag(ch.peer_flags, 0, s)                         # sender's free words
        with torch.cuda.stream(stream):
            self._wait(ready_ptr, u + 1, self._code(ch, True), stream, self._prog(ch, 3))
            self.C.dev_copy(t.data_ptr(), ch.own.ptr + s * ch.slot_bytes, nb, stream.cuda_stream)
            self._signal(free_ptr, u + 1, stream, self._prog(ch, 5))

    # ------------------------------------------------------------------ Transport API
    def send(self, t: torch.Tensor, peer: int) -> None:
        self.check()
        cur = torch.cuda.current_stream(self.device)
        # a contiguous copy is made on the compute stream BEFORE the send stream is ordered
        # after it, and that copy is the tensor kept alive for the send stream
        t = t.contiguous()
        self.send_stream.wait_stream(cur)
        t.record_stream(self.send_stream)
        self._ig_send("stage", peer, t, self.send_stream)   # the bytes the send reads
        self._send_on(self._ch[("stage", self.rank, peer)], t, self.send_stream)
        self._count(t, True)

    def recv(self, t: torch.Tensor, peer: int, free_event=None) -> torch.Tensor:
        self.check()
        cur = torch.cuda.current_stream(self.device)
        if free_event is not None:
            self.recv_stream.wait_event(free_event)
        else:
            self.recv_stream.wait_stream(cur)
        t.record_stream(self.recv_stream)
        self._recv_on(self._ch[("stage", peer, self.rank)], t, self.recv_stream)
        self._ig_recv("stage", peer, t, self.recv_stream)   # the bytes the next stage reads
        cur.wait_stream(self.recv_stream)
        self._count(t, False)
        return t

    def send_head(self, t: torch.Tensor, peer: int) -> None:
        self.check()
        cur = torch.cuda.current_stream(self.device)
        # a contiguous copy is made on the compute stream BEFORE the send stream is ordered
        # after it, and that copy is the tensor kept alive for the send stream
        t = t.contiguous()
        self.send_stream.wait_stream(cur)
        t.record_stream(self.send_stream)
        self._ig_send("head", peer, t, self.send_stream)
        self._send_on(self._ch[("head", self.rank, peer)], t, self.send_stream)
        self._count(t, True)

    def recv_head(self, t: torch.Tensor, peer: int, stream) -> torch.Tensor:
        self.check()
        self._recv_on(self._ch[("head", peer, self.rank)], t, stream)
        self._count(t, False)
        self._ig_recv("head", peer, t, stream)
        return t

    def check(self) -> None:
        """Raise if any device-side wait of this rank expired (a peer never arrived)."""
        code = self.status.get(0)
        if code:
            cid, recv = (code - 1) // 2, (code - 1) % 2
            ch = next((c for c in self._ch.values() if c.cid == cid), None)
            what = ch.describe() if ch is not None else f"channel {cid}"
            raise TimeoutError(f"[rank {self.rank}] IPC transport: {'receive' if recv else 'send'} "
                               f"on {what} waited > {self.timeout_s} s for its peer")

    def counters(self) -> dict:
        """Per channel: messages issued on this end (host) and the device's progress words
        (message n uses slot n % slots, round u = n // slots): sender - credit wait entered /
        passed (target u), ready released (u + 1); receiver - ready wait entered / passed
        (target u + 1), credit released (u + 1).  "entered" > "seen" = the stream sits in that
        wait; "entered" == "seen" with fewer issued = the stream is held up before it."""
        out = {}
        for c in self._ch.values():
            b = 2 + _PROG * c.cid
            g = self.status.get
            if self.rank == c.src:
                dev = {"credit_wait": g(b), "credit_seen": g(b + 1), "ready_released": g(b + 2)}
            else:
                dev = {"ready_wait": g(b + 3), "ready_seen": g(b + 4),
                       "credit_released": g(b + 5)}
            out[c.describe()] = {"issued": c.n, **dev}
        return out

    fallback_from = ""   # set by make_transport: why the default kind took IPC (a shared GPU)

    def describe(self) -> dict:
        d = {"transport": "IpcTransport",
             "channels": sorted(c.describe() for c in self._ch.values()),
             "timeout_s": self.timeout_s}
        if self.fallback_from:
            d["fallback_from"] = self.fallback_from
        return d

    def close(self) -> None:
        if not self._ch:
            return
        torch.cuda.synchronize(self.device)
        for ch in self._ch.values():
            for b in (ch.data, ch.peer_flags):
                if b is not None:
                    b.close()
        # owners free last (peers closed their mappings before the closing barrier)
        for ch in self._ch.values():
            ch.own.close()
        self._ch.clear()

    def abort(self) -> None:
        """Leaving after a failure: raise the abort word (every pending device wait of this rank
        exits at its next poll), no device synchronisation; the process exit releases the
        mappings."""
        self.status.set(1, 1)
        time.sleep(0.05)
        self._ch.clear()
