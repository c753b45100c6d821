"""Bounded, diagnosable failure for multi-process pipelines.

A stuck RCCL kernel raises no host error: the rank that notices is whichever one next waits on
the host for something that depends on it (the driver collecting tokens, the last stage's token
publisher), and until then every rank just waits.  Here:

* :class:`OpTracker` (one per process, :data:`TRACKER`) keeps the rank's LAST pipeline operation
  - op name, step, micro-batch, peer, stream - and the blocking wait it is in, if any.  The
  pipeline loops, transports and the head runner mark every operation (a few attribute writes).
* :class:`Watchdog` (a daemon thread per rank, on its own TCP-store client) aborts the job when
  a host wait that should progress - tokens of an in-flight step, a device event behind stage
  work - exceeds ``DLI_WATCHDOG_S`` (default 90 s), or when any rank raised: it publishes an abort
  key; every rank's watchdog sees it within a second, writes its last op to the store and to
  stderr, aborts its communicators (RCCL kernels waiting on a dead peer exit) and leaves with
  exit code 3.  The rank that flagged the stall prints the table of every rank's last op, so a
  hung 8-GPU run ends non-zero in ~watchdog + 10 s and says where each rank was.
"""
from __future__ import annotations

import collections
import contextlib
import json
import os
import sys
import threading
import time
from typing import Callable, List, Optional

EXIT_CODE = 3


# compute_in: this step's inputs uploaded, its graph about to run; compute: graph done
_MARK_ROLES = ("compute_in", "compute", "send", "recv", "head")


class OpTracker:
    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.last = {"op": "init", "step": -1, "mb": -1, "peer": -1, "stream": ""}
        self.by_thread: dict = {}   # thread name -> its last op (the pipeline loop, publisher...)
        self.t_last = time.monotonic()
        self.ops = 0
        self._waits: dict = {}      # thread name -> the blocking host wait it is in
        self.plans: "collections.deque" = collections.deque(maxlen=12)   # recent step shapes
        self._state: dict = {}      # name -> callable returning a JSON-able snapshot
        self._words = None          # device marks (enable_device_marks)

    def mark(self, op: str, step: int = -1, mb: int = -1, peer: int = -1, stream: str = "") -> None:
        rec = {"op": op, "step": step, "mb": mb, "peer": peer, "stream": stream}
        self.by_thread[threading.current_thread().name] = rec
        if threading.current_thread() is threading.main_thread():
            self.last = rec
        self.t_last = time.monotonic()
        self.ops += 1

    def enable_device_marks(self, device) -> None:
        """Per-stream device progress in the record: after each step's work on a role's stream
        (compute / send / recv / head) a one-lane kernel stores ``step + 1`` into host-mapped
        memory, next to the host's count of what it enqueued - a stuck rank then shows which
        stream is behind, and by how many steps, without any GPU call."""
        from .. import ops
        self._C = ops.native()
        self._words = self._C.HostWords(len(_MARK_ROLES))
        self._enq = {r: 0 for r in _MARK_ROLES}
        self.add_state("device", self.device_state)

    def device_mark(self, role: str, step: int, stream) -> None:
        if self._words is None or stream is None:
            return
        i = _MARK_ROLES.index(role)
        self._enq[role] = step + 1
        self._C.signal(self._words.dev_ptr(i), step + 1, stream.cuda_stream)

    def device_state(self) -> dict:
        """{role: [last step enqueued, last step the device finished]} (0 = none yet)."""
        return {r: [self._enq[r] - 1, self._words.get(i) - 1] for i, r in enumerate(_MARK_ROLES)
                if self._enq[r]}

    def add_state(self, name: str, fn) -> None:
        """Register a snapshot provider (transport counters, head-job queue...) for the record."""
        self._state[name] = fn

    @contextlib.contextmanager
    def waiting(self, what: str, step: int = -1, mb: int = -1, peer: int = -1):
        """A host wait that must end while the job is healthy (the watchdog times it)."""
        name = threading.current_thread().name
        self._waits[name] = {"what": what, "step": step, "mb": mb, "peer": peer,
                             "t0": time.monotonic()}
        try:
            yield
        finally:
            self._waits.pop(name, None)

    def current_wait(self) -> Optional[dict]:
        """The longest-running host wait of any thread (None: no thread is waiting)."""
        ws = list(self._waits.values())
        return min(ws, key=lambda w: w["t0"]) if ws else None

    def note_plan(self, step: int, **shape) -> None:
        """Shape of a step this rank executes (B, T, graph rows, longest sequence) for the
        record: a step whose kernels never finish can be told apart by its inputs."""
        self.plans.append({"step": step, **shape})

    def record(self) -> dict:
        now = time.monotonic()
        r = {"rank": self.rank, "last_op": dict(self.last), "ops": self.ops,
             "s_since_last_op": round(now - self.t_last, 1)}
        others = {k: v for k, v in self.by_thread.items() if k != threading.main_thread().name}
        if others:
            r["threads"] = others
        waits = {}
        for name, w in list(self._waits.items()):
            waits[name] = {k: v for k, v in w.items() if k != "t0"}
            waits[name]["for_s"] = round(now - w["t0"], 1)
        if waits:
            r["waiting"] = waits
        if self.plans:
            r["plans"] = list(self.plans)
        for name, fn in list(self._state.items()):
            try:
                r[name] = fn()
            except Exception as e:  # noqa: BLE001 - a snapshot must never block the abort
                r[name] = repr(e)
        return r


TRACKER = OpTracker()


def wait_event(ev, what: str, step: int = -1, mb: int = -1, poll_s: float = 5e-5) -> None:
    """``ev.synchronize()`` that the watchdog can see (polls ``query``; the GPU may be stuck
    behind a kernel waiting for another rank, which a blocking synchronize never reports)."""
    if ev is None or ev.query():
        return
    with TRACKER.waiting(what, step, mb):
        while not ev.query():
            time.sleep(poll_s)


class Watchdog:
    def __init__(self, job: str, world: int, stall_s: Optional[float] = None,
                 on_abort: Optional[Callable[[], None]] = None, poll_s: float = 1.0):
        self.job, self.world = job, world
        self.rank = TRACKER.rank
        self.stall_s = float(stall_s if stall_s is not None else os.environ.get("DLI_WATCHDOG_S", 90))
        self.on_abort = on_abort
        self.poll_s = poll_s
        self._store = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="dli-watchdog", daemon=True)
        self.key = f"dli_abort/{job}"

    # a private client connection: the main thread's store is not shared across threads
    def _client(self):
        if self._store is None:
            import datetime
            import torch.distributed as dist
            self._store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"),
                                        int(os.environ["MASTER_PORT"]), is_master=False,
                                        timeout=datetime.timedelta(seconds=10),
                                        wait_for_workers=False)
        return self._store

    def start(self) -> "Watchdog":
        self._client()
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def abort(self, reason: str) -> None:
        """Raise the job-wide alarm (this rank failed or saw a stall) and leave."""
        try:
            st = self._client()
            if not st.check([self.key]):
                st.set(self.key, json.dumps({"rank": self.rank, "reason": reason[:2000]}))
        except Exception:  # noqa: BLE001 - the alarm is best effort, the exit is not
            pass
        self._leave(flagger=True, reason=reason)

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            try:
                if self._client().check([self.key]):
                    info = json.loads(self._client().get(self.key))
                    self._leave(flagger=False, reason=f"rank {info['rank']}: {info['reason']}")
                w = TRACKER.current_wait()
                if w is not None and time.monotonic() - w["t0"] > self.stall_s:
                    self.abort(f"stalled {time.monotonic() - w['t0']:.0f} s (> DLI_WATCHDOG_S="
                               f"{self.stall_s:g}) waiting for {w['what']} (step {w['step']}, "
                               f"mb {w['mb']}, peer {w['peer']})")
            except SystemExit:
                raise
            except Exception:  # noqa: BLE001 - a store hiccup must not kill the watchdog
                continue

    def _leave(self, flagger: bool, reason: str) -> None:
        rec = TRACKER.record()
        try:
            self._client().set(f"dli_lastop/{self.job}/{self.rank}", json.dumps(rec))
        except Exception:  # noqa: BLE001
            pass
        print(f"[dli watchdog] rank {self.rank} aborting: {reason}\n[dli watchdog] rank "
              f"{self.rank} last op: {json.dumps(rec)}", file=sys.stderr, flush=True)
        if flagger:
            self._print_table()
            try:
                self._client().set(f"dli_abort_done/{self.job}", "1")
            except Exception:  # noqa: BLE001
                pass
        else:
            # stay until the flagging rank has printed the table: a launcher such as torchrun
            # kills the remaining ranks as soon as one of them exits
            t0 = time.monotonic()
            while time.monotonic() - t0 < 10.0:
                try:
                    if self._client().check([f"dli_abort_done/{self.job}"]):
                        break
                except Exception:  # noqa: BLE001
                    break
                time.sleep(0.2)
        if self.on_abort is not None:
            t = threading.Thread(target=self.on_abort, daemon=True)
            t.start()
            t.join(10.0)   # aborting communicators lets RCCL kernels waiting on a peer exit
        os._exit(EXIT_CODE)

    def _print_table(self, wait_s: float = 5.0) -> None:
        t0 = time.monotonic()
        recs: List[Optional[str]] = [None] * self.world
        while time.monotonic() - t0 < wait_s and any(r is None for r in recs):
            for r in range(self.world):
                if recs[r] is None:
                    try:
                        k = f"dli_lastop/{self.job}/{r}"
                        if self._client().check([k]):
                            recs[r] = self._client().get(k).decode()
                    except Exception:  # noqa: BLE001
                        pass
            time.sleep(0.2)
        lines = [f"  rank {r}: {rec if rec is not None else '<no record: process gone or stuck>'}"
                 for r, rec in enumerate(recs)]
        print("[dli watchdog] last op of every rank:\n" + "\n".join(lines), file=sys.stderr,
              flush=True)


_WATCHDOG: Optional[Watchdog] = None


def start_watchdog(job: str, world: int, on_abort=None) -> Optional[Watchdog]:
    """Start this process's watchdog (once; ``DLI_WATCHDOG_S=0`` disables it)."""
    global _WATCHDOG
    if _WATCHDOG is None and float(os.environ.get("DLI_WATCHDOG_S", 90)) > 0:
        _WATCHDOG = Watchdog(job, world, on_abort=on_abort).start()
    return _WATCHDOG


def abort_job(reason: str) -> None:
    """Called on an exception in a pipeline rank: every rank leaves promptly with its last op."""
    if _WATCHDOG is not None:
        _WATCHDOG.abort(reason)
