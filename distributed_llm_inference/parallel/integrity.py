"""Hop integrity: prove, in the run that matters, that the data plane delivers every payload intact.

The reference's whole purpose is to ship activations between block servers
(/root/reference/distributed_llm_inference/server/backend.py:42, server/server.py:7-8), and a
pipeline whose bytes arrive corrupted or at the wrong stage still produces a tokens/s number.  So
during a run's warm-up (prefill + warm-up steps; never inside a timed window) every message on
every stage pair and rotating-head pair is digested twice:

* on the sending rank, on its send stream, right before the send is enqueued (the exact bytes
  the transport reads);
* on the receiving rank, on the stream the data landed on, right after the receive (the exact
  bytes the next stage computes on).

The digest is csrc/kernels/digest.hip (two order-sensitive 64-bit sums over the payload's words;
one workgroup partial pair each, folded on the host).  Message n of a link is keyed
``{prefix}/{kind}/{src}-{dst}/{n}`` on both ends, so a dropped, duplicated, re-ordered or
mis-routed message shows up as a mismatch too.  At the first barrier every rank synchronises its
digests, publishes the ones it sent through the job's store, compares the ones it received with
the sender's, and turns the check off (:meth:`HopIntegrity.flush`).  bench.py reports
``hop_integrity: {checked, mismatch, missing}`` per rank and for the job, and exits non-zero on
any mismatch (``DLI_HOP_CHECK``, docs/env.md).
"""
from __future__ import annotations

import collections
import contextlib
import logging
import os
import time
from typing import List, Optional, Tuple

import torch

log = logging.getLogger(__name__)


def hop_check_enabled() -> bool:
    return os.environ.get("DLI_HOP_CHECK", "0").strip() not in ("", "0")


class HopIntegrity:
    def __init__(self, store, rank: int, prefix: str = "dli_hop", timeout_s: float = 60.0):
        self.store, self.rank, self.prefix = store, int(rank), prefix
        self.timeout_s = float(timeout_s)
        self.active = True
        self._seq: collections.Counter = collections.Counter()
        self._sent: List[Tuple[str, torch.Tensor, object]] = []
        self._recv: List[Tuple[str, torch.Tensor, object]] = []
        self.checked = self.mismatch = self.missing = self.published = 0
        self.failures: List[str] = []

    # ------------------------------------------------------------------ recording
    def _key(self, kind: str, src: int, dst: int, side: str) -> str:
        n = self._seq[(side, kind, src, dst)]
        self._seq[(side, kind, src, dst)] += 1
        return f"{self.prefix}/{kind}/{src}-{dst}/{n}"

    @staticmethod
    def _digest(t: torch.Tensor, stream) -> Tuple[torch.Tensor, object]:
        from .. import ops
        if not t.is_cuda:
            return ops.digest(t), None
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            parts = ops.digest(t)
            ev = torch.cuda.Event()
            ev.record()
        return parts, ev

    def on_send(self, kind: str, src: int, dst: int, t: torch.Tensor, stream=None) -> None:
        """Before the send of ``t`` is enqueued on ``stream`` (which already waits for ``t``)."""
        if self.active:
            self._sent.append((self._key(kind, src, dst, "s"),) + self._digest(t, stream))

    def on_recv(self, kind: str, src: int, dst: int, t: torch.Tensor, stream=None) -> None:
        """After the receive into ``t`` was enqueued on ``stream`` (CPU: after it completed)."""
        if self.active:
            self._recv.append((self._key(kind, src, dst, "r"),) + self._digest(t, stream))

    # ------------------------------------------------------------------ verification
    def flush(self) -> dict:
        """Publish the sent digests, check the received ones against their senders', and stop
        recording.  Every rank calls this at the same barrier (messages drained)."""
        from .. import ops
        if not self.active:
            return self.summary()
        self.active = False
        for key, parts, ev in self._sent:
            if ev is not None:
                ev.synchronize()
            a, b = ops.digest_fold(parts)
            self.store.set(key, f"{a}:{b}")
            self.published += 1
        deadline = time.monotonic() + self.timeout_s
        for key, parts, ev in self._recv:
            if ev is not None:
                ev.synchronize()
            a, b = ops.digest_fold(parts)
            while not self.store.check([key]):
                if time.monotonic() > deadline:
                    break
                time.sleep(0.002)
            if not self.store.check([key]):
                self.missing += 1
                self.failures.append(f"{key}: the sender published no digest")
                continue
            want = self.store.get(key).decode()
            self.checked += 1
            if want != f"{a}:{b}":
                self.mismatch += 1
                self.failures.append(f"{key}: received {a}:{b}, sent {want}")
        self._sent.clear()
        self._recv.clear()
        s = self.summary()
        if self.mismatch or self.missing:
            log.error("rank %d hop integrity FAILED: %s; first: %s", self.rank, s,
                      self.failures[:4])
        return s

    def summary(self) -> dict:
        d = {"checked": self.checked, "mismatch": self.mismatch, "missing": self.missing,
             "sent": self.published}
        if self.failures:
            d["failures"] = self.failures[:8]
        return d


def attach(tr, store, rank: int, job: str = "0") -> None:
    """Give transport ``tr`` a :class:`HopIntegrity` when ``DLI_HOP_CHECK`` is on."""
    if hop_check_enabled():
        tr.integrity = HopIntegrity(store, rank, prefix=f"dli_hop_{job}")


def flush(tr) -> Optional[dict]:
    """The barrier-time check of ``tr`` (no-op without integrity or after the first flush)."""
    ig = getattr(tr, "integrity", None)
    if ig is None:
        return None
    return ig.flush()
