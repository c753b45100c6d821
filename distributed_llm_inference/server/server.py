"""Server lifecycle: block placement, health checks, rebalance and restart.

Reference: ``Server.run()`` (/root/reference/distributed_llm_inference/server/server.py:4-24) — a
commented skeleton: choose "optimal block ids", build the module, then loop { wait; sleep a random
jitter; break if not healthy or should rebalance } and restart.  This is that loop, implemented for
one MI355X node:

* **placement** (``choose_blocks``): contiguous, cost-balanced layer ranges over the GPUs
  (``plan_stages``), weighted by each stage's measured speed once measurements exist;
* **launch**: one process per GPU running the pipeline stage + (rank 0) the HTTP front-end;
* **health** (``is_healthy``): every stage process alive, rank 0's ``/health`` answering and the
  engine loop not wedged;
* **rebalance** (``should_rebalance``): per-stage device time per step, published by every rank to
  the job's TCP store, differs by more than ``imbalance_threshold`` -> re-plan with the measured
  speeds;
* **restart**: tear the job down (terminate -> kill) and start it again with the new placement;
  bounded by ``max_restarts``.
Fault injection for tests: ``DLI_FAULT="kill:<rank>:<after_steps>"`` or
``"delay:<rank>:<ms>"`` in the workers' environment (see ``runtime/faults.py``).
"""
from __future__ import annotations

import json
import logging
import os
import random
import signal
import subprocess
import sys
import time
import urllib.request
from typing import Dict, List, Optional, Sequence, Tuple

from ..config import plan_stages, resolve_model
from ..launcher import _shutdown, free_port, package_pythonpath

log = logging.getLogger(__name__)


class Server:
    def __init__(self, model: str = "llama-3-8b", num_gpus: int = 1, port: int = 8000,
                 checkpoint: Optional[str] = None, extra_args: Sequence[str] = (),
                 health_interval: float = 2.0, max_restarts: int = 3,
                 imbalance_threshold: float = 1.3, startup_timeout: float = 900.0,
                 env: Optional[Dict[str, str]] = None):
        self.model = model
        self.spec = resolve_model(checkpoint or model)
        self.num_gpus = num_gpus
        self.port = port
        self.checkpoint = checkpoint
        self.extra_args = list(extra_args)
        self.health_interval = health_interval
        self.max_restarts = max_restarts
        self.imbalance_threshold = imbalance_threshold
        self.startup_timeout = startup_timeout
        self.env = dict(env or {})
        self.procs: List[subprocess.Popen] = []
        self.ranges: List[Tuple[int, int]] = []
        self.speeds: Optional[List[float]] = None
        self.restarts = 0
        self.store_port: Optional[int] = None
        self.events: List[str] = []

    # ------------------------------------------------------------------ placement
    def choose_blocks(self) -> List[Tuple[int, int]]:
        """The reference's "optimal block ids": cost-balanced contiguous ranges."""
        self.ranges = plan_stages(self.spec, self.num_gpus, self.speeds)
        return self.ranges

    # ------------------------------------------------------------------ process management
    def start(self) -> None:
        ranges = self.choose_blocks()
        self.store_port = free_port()
        base = dict(os.environ)
        base.update(self.env)
        base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(self.store_port),
                    WORLD_SIZE=str(self.num_gpus), LOCAL_WORLD_SIZE=str(self.num_gpus),
                    DLI_STAGE_RANGES=json.dumps(ranges), DLI_PUBLISH_STATS="1")
        base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        base["PYTHONPATH"] = package_pythonpath(base.get("PYTHONPATH"))
        args = [sys.executable, "-m", "distributed_llm_inference.cli", "worker", "--action", "serve",
                "--model", self.model, "--gpus", str(self.num_gpus), "--port", str(self.port)]
        if self.checkpoint:
            args += ["--checkpoint", self.checkpoint]
        args += self.extra_args
        self.procs = []
        for r in range(self.num_gpus):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            self.procs.append(subprocess.Popen(args, env=e))
        self._event(f"started {self.num_gpus} stages with placement {ranges}")
        self._wait_ready()

    def _wait_ready(self) -> None:
        deadline = time.time() + self.startup_timeout
        while time.time() < deadline:
            if any(p.poll() not in (None,) for p in self.procs):
                return  # a process died during startup: health check will report it
            if self._http_health() is not None:
                self._event("ready")
                return
            time.sleep(0.5)

    def stop(self) -> None:
        if self.procs:
            _shutdown(self.procs, grace_s=10.0)
            self._event("stopped")
        self.procs = []

    def restart(self) -> None:
        self.stop()
        self.restarts += 1
        self.start()

    # ------------------------------------------------------------------ health
    def _http_health(self) -> Optional[dict]:
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{self.port}/health", timeout=2.0) as r:
                return json.loads(r.read())
        except Exception:
            return None

    def stage_stats(self) -> List[Optional[dict]]:
        """Per-rank ``{"step_ms": ewma device ms per step, "steps": n}`` from the job store."""
        out: List[Optional[dict]] = []
        try:
            import torch.distributed as dist
            store = dist.TCPStore("127.0.0.1", self.store_port, is_master=False,
                                  timeout=__import__("datetime").timedelta(seconds=2))
            for r in range(self.num_gpus):
                key = f"dli_stats/{r}"
                try:
                    if store.check([key]):
                        out.append(json.loads(store.get(key)))
                    else:
                        out.append(None)
                except Exception:
                    out.append(None)
        except Exception:
            return [None] * self.num_gpus
        return out

    def is_healthy(self) -> bool:
        for r, p in enumerate(self.procs):
            if p.poll() is not None:
                self._event(f"stage {r} exited with code {p.returncode}")
                return False
        h = self._http_health()
        if h is None or not h.get("healthy", False):
            self._event("rank-0 health endpoint unhealthy")
            return False
        if h.get("running", 0) > 0 and h.get("seconds_since_last_step", 0) > 60:
            self._event("engine loop stalled")
            return False
        return True

    def should_rebalance(self) -> bool:
        st = self.stage_stats()
        if any(s is None or s.get("steps", 0) < 20 for s in st) or len(st) < 2:
            return False
        per_layer = [s["step_ms"] / max(1, e - b) for s, (b, e) in zip(st, self.ranges)]
        ratio = max(per_layer) / max(1e-9, min(per_layer))
        if ratio > self.imbalance_threshold:
            # stage speed ~ layers per ms; next placement gives slow stages fewer layers
            self.speeds = [1.0 / x for x in per_layer]
            self._event(f"imbalance {ratio:.2f} -> rebalance with speeds "
                        f"{[round(x, 3) for x in self.speeds]}")
            return True
        return False

    # ------------------------------------------------------------------ main loop
    def run(self, max_iterations: Optional[int] = None) -> None:
        it = 0
        while True:
            if not self.procs:
                self.start()
            try:
                while True:
                    time.sleep(self.health_interval * random.uniform(0.5, 1.0))  # jittered
                    it += 1
                    if not self.is_healthy():
                        break
                    if self.should_rebalance():
                        break
                    if max_iterations is not None and it >= max_iterations:
                        return
            finally:
                if max_iterations is not None and it >= max_iterations:
                    self.stop()
            if self.restarts >= self.max_restarts:
                self._event("max restarts reached; giving up")
                self.stop()
                raise RuntimeError("server failed: " + "; ".join(self.events[-5:]))
            self.restart()

    def _event(self, msg: str) -> None:
        log.warning("server: %s", msg)
        self.events.append(msg)
