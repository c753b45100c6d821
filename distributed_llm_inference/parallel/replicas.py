"""Data-parallel pipeline replicas (DP x PP) on one node.

The reference's swarm lets several servers host the same blocks (reference server/server.py:7-8,20:
"choose optimal block ids" / rebalance; server/worker.py:9-20: a worker owns a block range, any
number of workers may own the same range) and clients pick among them.  On one MI355X node the
equivalent is ``dp`` independent pipelines of ``pp`` stages each (``runtime.engine.ReplicaLayout``:
replica r = ranks [r*pp, (r+1)*pp), its own driver, shm control plane and RCCL pair communicators).
Llama-3-70B in bf16 (140 GB) fits on one 288 GB GPU, so dp8 x pp1 (no activation traffic at all)
and dp2 x pp4 are first-class layouts next to the pp8 headline.

This module is the part above the replicas:

* :func:`replica_generate` — offline generation: prompts are dealt round-robin to the replica
  drivers, each generates its share, rank 0 reassembles them in prompt order (gloo group over
  the drivers).
* :class:`ReplicaRouter` — online serving: one HTTP front end (rank 0) over every replica.
  Replica 0's :class:`EngineService` is in-process; every other replica driver runs a
  :class:`ReplicaServer` that takes requests from rank 0 over a shared-memory channel
  (csrc/runtime/shm_channel.cpp) and streams tokens / completions / stats back on another one;
  :class:`RemoteReplica` is rank 0's proxy for it.  Requests go to the replica with the fewest
  outstanding requests; ``abort`` follows the request to its replica.
"""
from __future__ import annotations

import dataclasses
import itertools
import logging
import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Sequence

import msgpack

from ..runtime.sequence import SamplingParams

log = logging.getLogger(__name__)


# ============================================================================ offline generate
def deal(items: Sequence, dp: int, replica: int) -> List:
    """Round-robin share of ``items`` for ``replica`` (item i goes to replica i % dp)."""
    return [x for i, x in enumerate(items) if i % dp == replica]


def undeal(shares: Sequence[Sequence], n: int) -> List:
    """Inverse of :func:`deal`: ``shares[r]`` holds items r, r+dp, ... -> the ``n`` items in order."""
    dp = len(shares)
    out = [None] * n
    for r, sh in enumerate(shares):
        for j, x in enumerate(sh):
            out[r + j * dp] = x
    return out


def replica_generate(drv, prompts: Sequence[Sequence[int]], params: SamplingParams):
    """Generate ``prompts`` over every replica; returns the Sequences in prompt order on the
    driver of replica 0 and None on the other replica drivers (call on every replica driver)."""
    import torch.distributed as dist
    layout = getattr(drv, "layout", None)
    group = getattr(drv, "drivers_group", None)
    if layout is None or layout.dp == 1 or group is None:
        return drv.generate(prompts, params)
    rep = drv.replica
    mine = deal(list(prompts), layout.dp, rep)
    outs = drv.generate(mine, params) if mine else []
    rec = [(s.prompt, s.output, s.finish_reason) for s in outs]
    shares = [None] * layout.dp
    dist.all_gather_object(shares, rec, group=group)
    if rep != 0:
        return None
    from ..runtime.sequence import Sequence as Seq
    res = []
    for prompt, output, reason in undeal(shares, len(prompts)):
        s = Seq(list(prompt), params)
        s.output, s.finish_reason = list(output), reason
        res.append(s)
    return res


# ============================================================================ online serving
def _channel_names(job: str, replica: int):
    return f"/dli_{job}_req{replica}", f"/dli_{job}_evt{replica}"


def _params_to_wire(p: SamplingParams) -> dict:
    return dataclasses.asdict(p)


class ReplicaServer:
    """Runs on a replica driver (replica > 0): serves rank 0's requests with the local
    :class:`EngineService` until rank 0 sends ``stop``."""

    def __init__(self, service, job: str, replica: int, timeout: float = 120.0,
                 stats_every_s: float = 1.0):
        from .. import _runtime as R
        self.svc = service
        req, evt = _channel_names(job, replica)
        self.evt = R.ShmChannel(evt, -1, 256, 1 << 20, 1, True)
        self.req = R.ShmChannel(req, 0, 256, 1 << 20, 1, False, timeout)
        self._lock = threading.Lock()      # one producer ring, several sender threads
        self._rid2sid: Dict[int, int] = {}
        self.stats_every_s = stats_every_s

    def _send(self, msg: dict) -> None:
        data = msgpack.packb(msg)
        with self._lock:
            self.evt.send(data, 60.0)

    def _forward_stream(self, rid: int, q: "queue.Queue", fut: Future) -> None:
        """Forward a streaming request's tokens, then its completion - from THIS thread, after
        the stream's end sentinel, so 'done' can never overtake a token still being forwarded
        (the proxy ends the stream on 'done')."""
        while True:
            tok = q.get()
            if tok is None:
                break
            self._send({"op": "tok", "rid": rid, "tok": int(tok)})
        try:
            fut.result()
        except Exception:  # noqa: BLE001 - reported by _on_done
            pass
        self._on_done(rid, fut)

    def _on_done(self, rid: int, fut: Future) -> None:
        self._rid2sid.pop(rid, None)
        try:
            c = fut.result()
            self._send({"op": "done", "rid": rid, "res": dataclasses.asdict(c)})
        except Exception as e:  # noqa: BLE001 - forwarded to the client
            self._send({"op": "err", "rid": rid, "err": repr(e)})

    def serve_forever(self) -> None:
        last_stats = 0.0
        while True:
            now = time.time()
            if now - last_stats >= self.stats_every_s:
                self._send({"op": "stats", "stats": self.svc.stats()})
                last_stats = now
            if not self.req.poll():
                time.sleep(0.002)
                continue
            msg = msgpack.unpackb(self.req.recv(5.0))
            op = msg["op"]
            if op == "stop":
                self._send({"op": "stats", "stats": self.svc.stats()})
                return
            if op == "abort":
                sid = self._rid2sid.get(msg["rid"])
                if sid is not None:
                    self.svc.abort(sid)
                continue
            rid = msg["rid"]
            try:
                fut, q = self.svc.submit(msg["prompt"], SamplingParams(**msg["params"]),
                                         stream=bool(msg.get("stream")))
            except Exception as e:  # noqa: BLE001
                self._send({"op": "err", "rid": rid, "err": repr(e)})
                continue
            self._rid2sid[rid] = fut.seq_id
            if q is not None:
                threading.Thread(target=self._forward_stream, args=(rid, q, fut),
                                 daemon=True).start()
            else:
                fut.add_done_callback(lambda f, rid=rid: self._on_done(rid, f))

    def close(self) -> None:
        for ch in (self.req, self.evt):
            try:
                ch.unlink()
            except Exception:  # noqa: BLE001
                pass


class RemoteReplica:
    """Rank 0's proxy for the :class:`ReplicaServer` of one replica (EngineService interface)."""

    def __init__(self, job: str, replica: int, timeout: float = 120.0):
        from .. import _runtime as R
        from ..server.service import Completion
        self._Completion = Completion
        self.replica = replica
        req, evt = _channel_names(job, replica)
        self.req = R.ShmChannel(req, -1, 256, 1 << 20, 1, True)
        self.evt = R.ShmChannel(evt, 0, 256, 1 << 20, 1, False, timeout)
        self._lock = threading.Lock()
        self._futs: Dict[int, Future] = {}
        self._streams: Dict[int, "queue.Queue"] = {}
        self._ids = itertools.count()
        self.last_stats: dict = {}
        self.error: Optional[str] = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._reader, daemon=True)
        self._thread.start()

    def submit(self, prompt_ids: List[int], params: SamplingParams, stream: bool = False):
        if self.error is not None:
            raise RuntimeError(f"replica {self.replica} failed: {self.error}")
        rid = next(self._ids)
        fut: Future = Future()
        fut.seq_id = rid  # type: ignore[attr-defined]
        q = queue.Queue() if stream else None
        self._futs[rid] = fut
        if q is not None:
            self._streams[rid] = q
        self._send({"op": "submit", "rid": rid, "prompt": list(prompt_ids),
                    "params": _params_to_wire(params), "stream": stream})
        return fut, q

    def abort(self, rid: int) -> None:
        self._send({"op": "abort", "rid": rid})

    def outstanding(self) -> int:
        return len(self._futs)

    def stats(self) -> dict:
        return dict(self.last_stats)

    def stop(self) -> None:
        self._send({"op": "stop"})
        self._thread.join(timeout=10)
        self._stop.set()

    def _send(self, msg: dict) -> None:
        data = msgpack.packb(msg)
        with self._lock:
            self.req.send(data, 60.0)

    def _reader(self) -> None:
        try:
            while not self._stop.is_set():
                if not self.evt.poll():
                    time.sleep(0.001)
                    continue
                msg = msgpack.unpackb(self.evt.recv(5.0), strict_map_key=False)
                op = msg["op"]
                if op == "stats":
                    self.last_stats = msg["stats"]
                    if self._stop.is_set():
                        return
                    continue
                rid = msg["rid"]
                if op == "tok":
                    q = self._streams.get(rid)
                    if q is not None:
                        q.put(msg["tok"])
                    continue
                fut = self._futs.pop(rid, None)
                q = self._streams.pop(rid, None)
                if q is not None:
                    q.put(None)
                if fut is None or fut.done():
                    continue
                if op == "done":
                    fut.set_result(self._Completion(**msg["res"]))
                else:
                    fut.set_exception(RuntimeError(msg.get("err", "replica error")))
        except Exception as e:  # noqa: BLE001 - a dead replica fails its waiters
            self.error = repr(e)
            for f in self._futs.values():
                if not f.done():
                    f.set_exception(RuntimeError(f"replica {self.replica} failed: {e!r}"))
            for q in self._streams.values():
                q.put(None)


class ReplicaRouter:
    """EngineService facade over several replicas (``services[i]`` has ``submit`` / ``abort`` /
    ``stats``): least-outstanding-requests dispatch, per-request replica affinity for abort,
    node-wide stats (sums of counters, max of latency percentiles)."""

    SUM_KEYS = ("running", "waiting", "total_tokens", "total_requests", "completed_requests",
                "aborted_requests", "tokens_per_s", "kv_reserved_blocks", "kv_total_blocks")
    MAX_KEYS = ("token_latency_p50_ms", "token_latency_p90_ms", "token_latency_p99_ms",
                "ttft_p50_ms", "ttft_p90_ms", "seconds_since_last_step", "uptime_s")

    def __init__(self, services: Sequence):
        self.services = list(services)
        self._route: Dict[int, tuple] = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._load = [0] * len(self.services)
        self._rr = 0   # rotating tie-break: equal loads do not all land on replica 0

    @property
    def error(self):
        for s in self.services:
            if getattr(s, "error", None) is not None:
                return s.error
        return None

    def submit(self, prompt_ids: List[int], params: SamplingParams, stream: bool = False):
        with self._lock:
            n = len(self.services)
            r = min(range(n), key=lambda i: (self._load[i], (i - self._rr) % n))
            self._rr = (r + 1) % n
            self._load[r] += 1
        try:
            fut, q = self.services[r].submit(prompt_ids, params, stream=stream)
        except Exception:
            with self._lock:
                self._load[r] -= 1
            raise
        gid = next(self._ids)
        self._route[gid] = (r, fut.seq_id)
        fut.seq_id = gid  # type: ignore[attr-defined]
        fut.replica = r   # type: ignore[attr-defined]

        def _done(_f, gid=gid, r=r):
            with self._lock:
                self._load[r] -= 1
            self._route.pop(gid, None)
        fut.add_done_callback(_done)
        return fut, q

    def generate(self, prompt_ids: List[int], params: SamplingParams, timeout=None):
        fut, _ = self.submit(prompt_ids, params)
        return fut.result(timeout)

    def abort(self, gid: int) -> None:
        rt = self._route.get(gid)
        if rt is not None:
            self.services[rt[0]].abort(rt[1])

    def stats(self) -> dict:
        per = [s.stats() or {} for s in self.services]
        out: dict = {"replicas": len(per)}
        for k in self.SUM_KEYS:
            out[k] = round(sum(p.get(k, 0) or 0 for p in per), 3)
        for k in self.MAX_KEYS:
            out[k] = max((p.get(k, 0) or 0 for p in per), default=0)
        out["kv_occupancy"] = (round(out["kv_reserved_blocks"] / out["kv_total_blocks"], 4)
                               if out["kv_total_blocks"] else 0.0)
        out["healthy"] = bool(per) and all(p.get("healthy", False) for p in per)
        for i, p in enumerate(per):
            out[f"replica{i}_healthy"] = bool(p.get("healthy", False))
            out[f"replica{i}_running"] = p.get("running", 0)
        return out

    def stage_stats(self) -> list:
        first = self.services[0]
        return first.stage_stats() if hasattr(first, "stage_stats") else []

    def shutdown(self, stop_driver: bool = False) -> None:
        for s in self.services[1:]:
            try:
                s.stop()
            except Exception as e:  # noqa: BLE001
                log.warning("replica stop failed: %s", e)
