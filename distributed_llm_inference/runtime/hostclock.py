"""Host time of a pipeline rank, split by phase.

A pipeline rank's host thread is on the critical path once per micro-batch step: the driver plans,
publishes the plan, stages metadata, launches stage 0 and collects tokens; a follower receives the
plan, stages metadata and launches its graph.  At PP = 8 the budget for all of it is one stage time
(~9 ms for 10 Llama-3-70B layers at 512 rows), so every phase is counted separately, and the
phases that WAIT on something (the device behind a staging slot, the token channel, the control
channel) are kept apart from the phases that are pure host work.

``HOST`` is the process-wide clock; :class:`~runtime.faults.StageStats` snapshots it at every
barrier and bench.py reports the per-micro-batch-step breakdown of the timed window per rank.
"""
from __future__ import annotations

import collections
import time
from typing import Dict

# phases in which the host thread waits for another agent instead of working
WAIT_PHASES = ("staging_wait", "tokens_wait", "ctrl_wait", "ring_wait")


class HostClock:
    __slots__ = ("ms", "n")

    def __init__(self):
        self.ms: Dict[str, float] = collections.defaultdict(float)
        self.n: Dict[str, int] = collections.defaultdict(int)

    def since(self, phase: str, t0: float) -> float:
        """Charge ``now - t0`` to ``phase``; returns now (the next phase's start)."""
        now = time.perf_counter()
        self.ms[phase] += (now - t0) * 1e3
        self.n[phase] += 1
        return now

    def add(self, phase: str, ms: float) -> None:
        self.ms[phase] += ms
        self.n[phase] += 1

    def snapshot(self) -> Dict[str, float]:
        return {f"host_{k}_ms": v for k, v in self.ms.items()}

    def reset(self) -> None:
        self.ms.clear()
        self.n.clear()


HOST = HostClock()


def per_step(delta: Dict[str, float], steps: int) -> Dict[str, object]:
    """From a :func:`~runtime.faults.snapshot_delta` record: host ms per micro-batch step, by
    phase, plus the busy (non-waiting) and waiting totals."""
    n = max(int(steps), 1)
    phases = {k[len("host_"):-len("_ms")]: v / n for k, v in delta.items()
              if k.startswith("host_") and k.endswith("_ms")}
    busy = sum(v for k, v in phases.items() if k not in WAIT_PHASES)
    wait = sum(v for k, v in phases.items() if k in WAIT_PHASES)
    return {"host_busy_ms_per_mb_step": round(busy, 3),
            "host_wait_ms_per_mb_step": round(wait, 3),
            "host_ms_per_mb_step": {k: round(v, 3) for k, v in sorted(phases.items())}}
