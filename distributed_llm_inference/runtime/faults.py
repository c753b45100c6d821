"""Fault injection and per-stage performance stats (used by the server's health / rebalance loop).

``DLI_FAULT`` (comma-separated specs, read once per process):
  * ``kill:<rank>:<after_steps>``  — the rank exits abruptly (``os._exit(17)``) after N steps;
  * ``delay:<rank>:<ms>``          — the rank sleeps <ms> before every step (a slow GPU);
  * ``hang:<rank>:<after_steps>``  — the rank stops making progress (sleeps forever).
``DLI_PUBLISH_STATS=1`` makes every rank publish ``{"step_ms", "steps"}`` (EWMA of device time per
step, measured with HIP events, read back lazily without synchronising) to the job's TCP store.
"""
from __future__ import annotations

import collections
import json
import os
import time
from typing import Deque, List, Optional, Tuple

import torch


def raw_store():
    """The job's TCPStore without torch's PrefixStore wrappers (so external supervisors that
    connect to MASTER_PORT see the same keys)."""
    import torch.distributed as dist
    s = dist.distributed_c10d._get_default_store()
    while hasattr(s, "underlying_store"):
        s = s.underlying_store
    return s


class FaultInjector:
    def __init__(self, rank: int, spec: Optional[str] = None):
        self.rank = rank
        self.kill_after: Optional[int] = None
        self.hang_after: Optional[int] = None
        self.delay_ms = 0.0
        self.steps = 0
        for item in (spec if spec is not None else os.environ.get("DLI_FAULT", "")).split(","):
            if not item.strip():
                continue
            kind, r, v = item.strip().split(":")
            if int(r) != rank:
                continue
            if kind == "kill":
                self.kill_after = int(v)
            elif kind == "delay":
                self.delay_ms = float(v)
            elif kind == "hang":
                self.hang_after = int(v)
            else:
                raise ValueError(f"unknown fault kind {kind!r}")

    @property
    def active(self) -> bool:
        return self.kill_after is not None or self.hang_after is not None or self.delay_ms > 0

    def on_step(self) -> None:
        self.steps += 1
        if self.delay_ms > 0:
            time.sleep(self.delay_ms / 1e3)
        if self.kill_after is not None and self.steps >= self.kill_after:
            os._exit(17)
        if self.hang_after is not None and self.steps >= self.hang_after:
            while True:
                time.sleep(3600)


class StageStats:
    """Per-step device time of this rank: an EWMA published to the torch.distributed store
    (``DLI_PUBLISH_STATS=1``, read by the server's rebalance loop) and cumulative totals that
    :meth:`snapshot` reports (``DLI_STAGE_TIMING=1``, used by bench.py's per-rank fields)."""

    def __init__(self, rank: int, device: torch.device, publish_every: int = 20, alpha: float = 0.1):
        self.rank = rank
        self.device = device
        self.publishing = os.environ.get("DLI_PUBLISH_STATS", "0") == "1"
        self.enabled = self.publishing or os.environ.get("DLI_STAGE_TIMING", "0") == "1"
        self.every = publish_every
        self.alpha = alpha
        self.ewma: Optional[float] = None
        self.steps = 0
        self.total_ms = 0.0
        self._pending: Deque[Tuple] = collections.deque()
        self._t0 = 0.0
        self._store = None
        self.transport = None   # set by the pipeline: its traffic counters are published too

    def begin(self, extra_ms: float = 0.0):
        if not self.enabled:
            return None
        if self.device.type == "cuda":
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            return (s, e, extra_ms)
        return (time.perf_counter(), None, extra_ms)

    def end(self, tok) -> None:
        if tok is None:
            return
        s, e, extra = tok
        if e is not None:
            e.record()
            self._pending.append((s, e, extra))
        else:
            self._add((time.perf_counter() - s) * 1e3 + extra)
        self._poll(block=False)

    def _poll(self, block: bool) -> None:
        while self._pending and (block or self._pending[0][1].query()):
            s, e, extra = self._pending.popleft()
            e.synchronize()
            self._add(s.elapsed_time(e) + extra)

    def _add(self, ms: float) -> None:
        self.ewma = ms if self.ewma is None else (1 - self.alpha) * self.ewma + self.alpha * ms
        self.steps += 1
        self.total_ms += ms
        if self.publishing and self.steps % self.every == 0:
            self.publish()

    def snapshot(self) -> dict:
        """Cumulative counters now (waits for the timing events still in flight)."""
        self._poll(block=True)
        from .hostclock import HOST
        rec = {"t": time.perf_counter(), "steps": self.steps, "device_ms": self.total_ms}
        rec.update(HOST.snapshot())
        if self.transport is not None:
            rec.update(self.transport.traffic())
        return rec

    def publish(self) -> None:
        try:
            if self._store is None:
                self._store = raw_store()
            rec = {"step_ms": self.ewma, "steps": self.steps}
            if self.transport is not None:
                rec.update(self.transport.traffic())
            # keyed by GLOBAL rank: with several pipeline replicas stage indices repeat
            self._store.set(f"dli_stats/{os.environ.get('RANK', self.rank)}", json.dumps(rec))
        except Exception:
            pass


def snapshot_delta(a: dict, b: dict) -> dict:
    """Counters accumulated between two :meth:`StageStats.snapshot` records."""
    return {k: b[k] - a[k] for k in b if k in a and isinstance(b[k], (int, float))}
