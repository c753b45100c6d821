"""Request-batching pool.

Reference: ``TaskPool(func)`` stub (/root/reference/distributed_llm_inference/server/task_pool.py:4-8)
and hivemind's TaskPool used by ``InferenceBackend`` (server/backend.py:42): independent tasks are
aggregated up to ``max_batch_size`` rows and processed by one call.

Here a pool is a background thread (the GPU work it triggers is asynchronous anyway; no extra
processes or pipes): ``submit_task(*tensors, **meta)`` returns a ``Future``; the pool gathers
tasks until ``max_batch_size`` rows are pending or ``timeout`` elapses, then calls
``process_func``.  With ``collate=True`` the tasks' tensors are concatenated along dim 0 and the
outputs split back; with ``collate=False`` the raw task list is passed (used by the block backend
to pack variable-length sessions into one varlen forward).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

log = logging.getLogger(__name__)


@dataclass
class Task:
    args: Tuple[Any, ...]
    meta: Dict[str, Any]
    future: Future = field(default_factory=Future)
    size: int = 1
    t_submit: float = field(default_factory=time.perf_counter)


class TaskPool:
    def __init__(self, process_func: Callable, max_batch_size: int = 256, name: str = "pool",
                 timeout: float = 0.002, collate: bool = True, start: bool = True):
        if max_batch_size < 1:
            raise ValueError("max_batch_size must be >= 1")
        self.process_func = process_func
        self.max_batch_size = max_batch_size
        self.name = name
        self.timeout = timeout
        self.collate = collate
        self._q: "queue.Queue[Optional[Task]]" = queue.Queue()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.batches_processed = 0
        self.tasks_processed = 0
        if start:
            self.start()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        if self._thread is None or not self._thread.is_alive():
            self._stop.clear()
            self._thread = threading.Thread(target=self._run, name=self.name, daemon=True)
            self._thread.start()

    def shutdown(self, timeout: float = 10.0) -> None:
        self._stop.set()
        self._q.put(None)
        if self._thread is not None:
            self._thread.join(timeout)

    @property
    def is_alive(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    # ------------------------------------------------------------------ client
    def submit_task(self, *args, **meta) -> Future:
        size = 1
        for a in args:
            if isinstance(a, torch.Tensor) and a.dim() > 0:
                size = int(a.shape[0])
                break
        if size > self.max_batch_size:
            raise ValueError(f"task batch {size} exceeds max_batch_size {self.max_batch_size}")
        t = Task(args, meta, size=size)
        self._q.put(t)
        return t.future

    def __call__(self, *args, **meta):
        return self.submit_task(*args, **meta).result()

    # ------------------------------------------------------------------ worker
    def _gather(self) -> List[Task]:
        first = self._q.get()
        if first is None:
            return []
        batch, rows = [first], first.size
        deadline = time.perf_counter() + self.timeout
        while rows < self.max_batch_size:
            rem = deadline - time.perf_counter()
            try:
                t = self._q.get(timeout=max(0.0, rem)) if rem > 0 else self._q.get_nowait()
            except queue.Empty:
                break
            if t is None:
                self._stop.set()
                break
            if rows + t.size > self.max_batch_size:
                self._q.put(t)  # next batch
                break
            batch.append(t)
            rows += t.size
        return batch

    def _run(self) -> None:
        while not self._stop.is_set():
            batch = self._gather()
            if not batch:
                continue
            try:
                if self.collate:
                    nargs = len(batch[0].args)
                    cat = [torch.cat([t.args[i] for t in batch], 0) for i in range(nargs)]
                    out = self.process_func(*cat)
                    outs = out if isinstance(out, (tuple, list)) else (out,)
                    sizes = [t.size for t in batch]
                    pieces = [torch.split(o, sizes, 0) for o in outs]
                    for j, t in enumerate(batch):
                        res = tuple(p[j] for p in pieces)
                        t.future.set_result(res if isinstance(out, (tuple, list)) else res[0])
                else:
                    # a result that is an exception fails that task alone (e.g. a session whose
                    # KV reservation did not fit); the rest of the batch completes
                    results = self.process_func(batch)
                    for t, r in zip(batch, results):
                        if isinstance(r, BaseException):
                            t.future.set_exception(r)
                        else:
                            t.future.set_result(r)
                self.batches_processed += 1
                self.tasks_processed += len(batch)
            except BaseException as e:  # deliver the failure to every waiter
                log.exception("%s: batch failed", self.name)
                for t in batch:
                    if not t.future.done():
                        t.future.set_exception(e)
