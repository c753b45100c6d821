"""Online serving on top of a pipeline driver: request queue, engine loop thread, streaming.

Runs on rank 0 (the driver).  Requests arrive from any thread (HTTP handlers); the engine loop
thread owns the scheduler/driver and gives every in-flight micro-batch one step per round
(continuous batching: new requests join at their micro-batch's next step, finished sequences free
their KV blocks immediately).
"""
from __future__ import annotations

import collections
import json
import os
import logging
import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..runtime.sequence import SamplingParams, Sequence, SeqStatus

log = logging.getLogger(__name__)


@dataclass
class Completion:
    seq_id: int
    prompt_len: int
    output_ids: List[int]
    finish_reason: Optional[str]
    latency_s: float
    ttft_s: Optional[float]
    token_latencies_ms: List[float] = field(default_factory=list)


class EngineService:
    def __init__(self, driver, eos_token_id: Optional[int] = None, idle_wait_s: float = 0.02):
        self.driver = driver
        self.eos = eos_token_id
        self._new: "queue.Queue" = queue.Queue()
        self._futs: Dict[int, Future] = {}
        self._streams: Dict[int, "queue.Queue"] = {}
        self._sent: Dict[int, int] = {}
        self._seqs: Dict[int, Sequence] = {}
        self._stop = threading.Event()
        self._idle = idle_wait_s
        self.started = time.time()
        self.total_tokens = 0
        self.total_requests = 0
        self.last_step_time = time.time()
        self.error: Optional[BaseException] = None
        # rolling windows for /metrics: per-token latency, time to first token
        self._tok_lat_ms: "collections.deque" = collections.deque(maxlen=8192)
        self._ttft_ms: "collections.deque" = collections.deque(maxlen=1024)
        self.completed = 0
        self.aborted = 0
        self._thread = threading.Thread(target=self._loop, name="dli-engine", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ client API
    def submit(self, prompt_ids: List[int], params: SamplingParams,
               stream: bool = False) -> "tuple[Future, Optional[queue.Queue]]":
        if self.error is not None:
            raise RuntimeError(f"engine failed: {self.error!r}")
        seq = Sequence(list(prompt_ids), params)
        fut: Future = Future()
        fut.seq_id = seq.seq_id  # type: ignore[attr-defined]  (for abort on timeout / disconnect)
        q = queue.Queue() if stream else None
        self._new.put((seq, fut, q))
        return fut, q

    def generate(self, prompt_ids: List[int], params: SamplingParams,
                 timeout: Optional[float] = None) -> Completion:
        fut, _ = self.submit(prompt_ids, params)
        return fut.result(timeout)

    def abort(self, seq_id: int) -> None:
        """Stop generating for ``seq_id`` (request timeout, client gone); its KV blocks are freed
        at the next step and its future resolves with ``finish_reason="abort"``."""
        self._new.put(("abort", seq_id, None))

    @staticmethod
    def _pct(xs, q: float) -> float:
        if not xs:
            return 0.0
        v = sorted(xs)
        return round(v[min(len(v) - 1, int(q * len(v)))], 3)

    def stats(self) -> dict:
        s = self.driver.sched
        up = time.time() - self.started
        lat, ttft = list(self._tok_lat_ms), list(self._ttft_ms)
        return dict(running=s.num_running(), waiting=len(s.waiting), uptime_s=round(up, 1),
                    total_tokens=self.total_tokens, total_requests=self.total_requests,
                    completed_requests=self.completed, aborted_requests=self.aborted,
                    tokens_per_s=round(self.total_tokens / up, 2) if up > 0 else 0.0,
                    token_latency_p50_ms=self._pct(lat, 0.5),
                    token_latency_p90_ms=self._pct(lat, 0.9),
                    token_latency_p99_ms=self._pct(lat, 0.99),
                    ttft_p50_ms=self._pct(ttft, 0.5), ttft_p90_ms=self._pct(ttft, 0.9),
                    kv_reserved_blocks=s.reserved_blocks, kv_total_blocks=s.total_blocks,
                    kv_occupancy=round(s.reserved_blocks / s.total_blocks, 4) if s.total_blocks else 0.0,
                    seconds_since_last_step=round(time.time() - self.last_step_time, 3),
                    healthy=self.error is None and self._thread.is_alive())

    def stage_stats(self) -> list:
        """Per-rank ``{"step_ms", "steps", "bytes_sent", "bytes_recv", ...}`` that every stage
        publishes to the job store when ``DLI_PUBLISH_STATS=1`` (empty otherwise)."""
        if os.environ.get("DLI_PUBLISH_STATS", "0") != "1":
            return []
        try:
            from ..runtime.faults import raw_store
            store = raw_store()
            out = []
            for r in range(int(os.environ.get("WORLD_SIZE", "1"))):
                key = f"dli_stats/{r}"
                out.append(json.loads(store.get(key)) if store.check([key]) else None)
            return out
        except Exception:  # pragma: no cover - store unavailable (single process)
            return []

    def shutdown(self, stop_driver: bool = True) -> None:
        self._stop.set()
        self._thread.join(timeout=30)
        if stop_driver:
            try:
                self.driver.stop()
            except Exception as e:  # pragma: no cover
                log.warning("driver stop failed: %s", e)

    # ------------------------------------------------------------------ engine loop
    def _ingest(self, block: bool) -> None:
        try:
            item = self._new.get(timeout=self._idle) if block else self._new.get_nowait()
        except queue.Empty:
            return
        while True:
            seq, fut, q = item
            if seq == "abort":
                self.driver.sched.abort(fut)
            else:
                try:
                    self.driver.sched.add(seq)
                    self._futs[seq.seq_id] = fut
                    self._seqs[seq.seq_id] = seq
                    self._sent[seq.seq_id] = 0
                    if q is not None:
                        self._streams[seq.seq_id] = q
                    self.total_requests += 1
                except Exception as e:
                    fut.set_exception(e)
            try:
                item = self._new.get_nowait()
            except queue.Empty:
                return

    def _publish(self) -> None:
        for sid, q in list(self._streams.items()):
            s = self._seqs[sid]
            n = len(s.output)
            if n > self._sent[sid]:
                for t in s.output[self._sent[sid]:n]:
                    q.put(t)
                self._sent[sid] = n
        for s in self.driver.sched.pop_finished():
            fut = self._futs.pop(s.seq_id, None)
            self._seqs.pop(s.seq_id, None)
            q = self._streams.pop(s.seq_id, None)
            if q is not None:
                for t in s.output[self._sent.get(s.seq_id, 0):]:
                    q.put(t)
                q.put(None)
            self._sent.pop(s.seq_id, None)
            self.total_tokens += len(s.output)
            tt = s.token_times
            self._tok_lat_ms.extend((tt[i + 1] - tt[i]) * 1e3 for i in range(len(tt) - 1))
            if s.first_token_time:
                self._ttft_ms.append((s.first_token_time - s.arrival) * 1e3)
            if s.finish_reason == "abort":
                self.aborted += 1
            else:
                self.completed += 1
            if fut is not None and not fut.done():
                tt = s.token_times
                fut.set_result(Completion(
                    seq_id=s.seq_id, prompt_len=len(s.prompt), output_ids=list(s.output),
                    finish_reason=s.finish_reason, latency_s=time.perf_counter() - s.arrival,
                    ttft_s=(s.first_token_time - s.arrival) if s.first_token_time else None,
                    token_latencies_ms=[(tt[i + 1] - tt[i]) * 1e3 for i in range(len(tt) - 1)]))

    def _loop(self) -> None:
        try:
            act = getattr(self.driver, "activate_streams", None)
            if act is not None:
                act()   # the rank's compute stream is per thread (runtime/streams.py)
            while not self._stop.is_set():
                sched = self.driver.sched
                self._ingest(block=not sched.has_work())
                if sched.has_work():
                    self.driver.round()
                    self.last_step_time = time.time()
                self._publish()
            self.driver.drain()
            self._publish()
        except BaseException as e:  # surface engine failures to every waiter
            log.exception("engine loop failed")
            self.error = e
            for fut in self._futs.values():
                if not fut.done():
                    fut.set_exception(RuntimeError(f"engine failed: {e!r}"))
            for q in self._streams.values():
                q.put(None)
