"""RCCL bring-up failure handling with more than two ranks (parallel/transport.py RcclTransport),
simulated on the CPU: one thread per rank, a blocking in-memory store, and a fake native module
whose 2-rank communicator init blocks until both members arrive (like ncclCommInitRank) or its
deadline passes, and fails immediately on a chosen rank.

The failure path used to hang with > 2 ranks: a rank whose first communicator init raised never
published the unique id of its next pair, so that peer blocked in ``store.get`` forever (seen as
a 900 s hang of an 8-rank bench on a shared GPU).  Now every rank publishes the ids it owns before
initialising anything, and stops at the next init once any rank has published a failure."""
import threading
import time

import pytest
import torch

from distributed_llm_inference.parallel import transport as tmod


class _Store:
    def __init__(self):
        self.d, self.cv = {}, threading.Condition()

    def set(self, k, v):
        with self.cv:
            self.d[k] = v if isinstance(v, bytes) else str(v).encode()
            self.cv.notify_all()

    def get(self, k):
        with self.cv:
            if not self.cv.wait_for(lambda: k in self.d, timeout=10.0):
                raise TimeoutError(f"store.get({k!r}) blocked")   # the old hang
            return self.d[k]

    def check(self, keys):
        with self.cv:
            return all(k in self.d for k in keys)

    def compare_set(self, k, expected, desired):
        with self.cv:
            cur = self.d.get(k)
            if (cur is None and expected == "") or (cur is not None and cur == expected.encode()):
                self.d[k] = desired.encode()
                self.cv.notify_all()
            return self.d[k]


class _Comm:
    """A 2-rank communicator whose (non-blocking) init completes once both members arrived,
    never if either member is the hung rank."""

    def __init__(self, ev, idx, hung):
        self.ev, self.idx, self.hung = ev, idx, hung

    def ready(self):
        return not self.hung[0] and self.ev[1 - self.idx].is_set()

    def abort(self):
        pass


class _Native:
    """ncclGetUniqueId / 2-rank ncclCommInitRank stand-ins."""

    def __init__(self, fail_rank, hung_rank=None):
        self.fail_rank, self.lock, self.arrived, self.n = fail_rank, threading.Lock(), {}, 0
        self.hung_rank, self.members = hung_rank, {}

    def rccl_version(self):
        return 22606

    def rccl_unique_id(self):
        with self.lock:
            self.n += 1
            return f"uid{self.n}".encode()

    def RcclComm(self, uid, idx, world, dev, timeout_s, wait=True):
        me = threading.current_thread().name
        if me == f"rank{self.fail_rank}":
            raise RuntimeError("RCCL error: invalid usage (duplicate GPU)")
        with self.lock:
            ev = self.arrived.setdefault(uid, [threading.Event(), threading.Event()])
            hung = self.members.setdefault(uid, [False])
            if me == f"rank{self.hung_rank}":
                hung[0] = True      # this pair's init never completes, on either end
        ev[idx].set()
        if wait and not ev[1 - idx].wait(timeout=min(timeout_s, 1.0)):
            raise RuntimeError("ncclCommInitRankConfig timed out")
        return _Comm(ev, idx, hung)


class _Streams:
    send = recv = None


@pytest.mark.parametrize("world,fail_rank,head", [(4, 1, False), (8, 1, True), (8, 6, True),
                                                   (8, 7, True), (8, 0, False)])
def test_rccl_bringup_failure_never_blocks_peers(monkeypatch, world, fail_rank, head):
    nat = _Native(fail_rank)
    from distributed_llm_inference import ops
    monkeypatch.setattr(ops, "native", lambda: nat)
    store = _Store()
    errs = {}

    def rank_main(r):
        try:
            tmod.RcclTransport(store, r, world, torch.device("cuda", 0), prefix="t",
                               timeout_s=1.0, head_pairs=head, streams=_Streams())
            errs[r] = None
        except Exception as e:  # noqa: BLE001
            errs[r] = e
            store.set("t/failed", f"rank {r}")   # what make_transport publishes

    th = [threading.Thread(target=rank_main, args=(r,), name=f"rank{r}") for r in range(world)]
    t0 = time.monotonic()
    for t in th:
        t.start()
    for t in th:
        t.join(30.0)
    assert not any(t.is_alive() for t in th), "a rank is still blocked"
    assert time.monotonic() - t0 < 20.0
    assert not any(isinstance(e, TimeoutError) for e in errs.values()), errs
    assert isinstance(errs[fail_rank], RuntimeError) and "duplicate" in str(errs[fail_rank])
    # nobody completes a transport when a rank failed: every other rank either stopped at a
    # published failure, timed out on the failed peer, or (CPU box) failed its CUDA connect probe
    assert len(errs) == world


def _ids(shared: bool):
    """Simulated device identities (parallel/pipeline.py device_identity) per rank thread."""
    return lambda device: ("host/0000:05:00/gpu0" if shared else
                           f"host/0000:{5 + int(threading.current_thread().name[4:]):02x}:00/gpu")


@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("env", [None, "rccl-or-ipc", "rccl", "rccl-or-host", "ipc", "host"])
@pytest.mark.parametrize("rccl_fails", [False, True])
def test_data_plane_choice_by_device(monkeypatch, shared, env, rccl_fails):
    """make_transport on two GPU ranks (threads over one in-memory store, stand-in transports):
    the default (``rccl-or-ipc``) takes the IPC device transport ONLY when the ranks' published
    devices coincide - without trying RCCL - and strict RCCL on distinct GPUs, where an RCCL
    failure fails every rank (TransportInitError) instead of silently becoming IPC; the explicit
    kinds are taken as given (``rccl-or-host`` falls back to host staging when RCCL fails)."""
    from distributed_llm_inference.parallel import ipc_transport, pipeline
    from distributed_llm_inference.runtime import faults

    store = _Store()
    monkeypatch.setattr(faults, "raw_store", lambda: store)
    monkeypatch.setattr(pipeline, "device_identity", _ids(shared))
    tried = []

    class FakeRccl:
        def __init__(self, store, rank, world, device, **kw):
            tried.append(rank)
            if rccl_fails and rank == 1:
                raise RuntimeError("RCCL error: invalid usage")

        def abort(self):
            pass

    class FakeIpc:
        def __init__(self, store, rank, world, device, streams, max_bytes, head_bytes, **kw):
            self.rank = rank

    class FakeHost:
        def __init__(self, rank_offset=0):
            pass

    monkeypatch.setattr(pipeline, "RcclTransport", FakeRccl)
    monkeypatch.setattr(ipc_transport, "IpcTransport", FakeIpc)
    monkeypatch.setattr(tmod, "HostStagedTransport", FakeHost)
    if env is None:
        monkeypatch.delenv("DLI_TRANSPORT", raising=False)
    else:
        monkeypatch.setenv("DLI_TRANSPORT", env)
    res = {}

    def rank_main(r):
        try:
            res[r] = pipeline.make_transport(r, 2, torch.device("cuda", 0), job="j",
                                             rccl_timeout_s=5.0, streams=_Streams(),
                                             max_bytes=1 << 20, head_bytes=1 << 16)
        except Exception as e:  # noqa: BLE001
            res[r] = e

    th = [threading.Thread(target=rank_main, args=(r,), name=f"rank{r}") for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(20.0)
    assert not any(t.is_alive() for t in th)
    kind = env or "rccl-or-ipc"
    if kind == "rccl-or-ipc":
        expect = "ipc" if shared else ("raise" if rccl_fails else "rccl")
    elif kind in ("rccl", "rccl-or-host"):
        expect = "rccl" if not rccl_fails else ("raise" if kind == "rccl" else "host")
    else:
        expect = kind
    for r in range(2):
        if expect == "ipc":
            assert isinstance(res[r], FakeIpc), res
        elif expect == "host":
            assert isinstance(res[r], FakeHost), res
        elif expect == "rccl":
            assert isinstance(res[r], FakeRccl), res
        else:
            assert isinstance(res[r], pipeline.TransportInitError), res
            assert "failed on ranks [1]" in str(res[r])
    if kind == "rccl-or-ipc" and shared:
        assert tried == [], "RCCL must not be tried on a shared GPU"
        assert all("share a GPU" in res[r].fallback_from for r in range(2))


def test_agreement_is_sticky_for_a_late_rank():
    """a rank answering after another rank published a failure must not flip the
    decision - ranks that decided without it and the late rank itself agree it failed."""
    from distributed_llm_inference.parallel import pipeline
    store = _Store()
    store.set("p/ok/0", "1")
    store.set("p/ok/1", "1")
    store.set("p/failed", "rank 0: ranks [2] never answered")
    assert pipeline._agree(store, "p", 3, 0, 1.0) == [True, True, False]
    # rank 2 finally comes up and answers ok: the key was already settled at "0"
    assert pipeline._publish_ok(store, "p/ok/2", True) is False
    assert pipeline._agree(store, "p", 3, 2, 1.0) == [True, True, False]
    assert pipeline._agree(store, "p", 3, 1, 1.0) == [True, True, False]


@pytest.mark.parametrize("hung_rank,head", [(3, True), (7, True), (0, False), (5, False)])
def test_hung_rank_ends_bringup_within_seconds(monkeypatch, hung_rank, head):
    """One of 8 ranks (distinct GPUs, strict RCCL) enters its RCCL inits but they never complete.
    Its peers see the pair pending a probe window after both ends entered it, publish the
    failure, and every rank -- the hung one included -- raises TransportInitError with the same
    set of failed ranks within seconds, not after the 120 s init deadline."""
    from distributed_llm_inference.parallel import pipeline
    from distributed_llm_inference.runtime import faults
    nat = _Native(fail_rank=None, hung_rank=hung_rank)
    from distributed_llm_inference import ops
    monkeypatch.setattr(ops, "native", lambda: nat)
    monkeypatch.setattr(tmod.RcclTransport, "_connect", lambda self: 0.0)   # no CUDA probe here
    store = _Store()
    monkeypatch.setattr(faults, "raw_store", lambda: store)
    monkeypatch.setattr(pipeline, "device_identity", _ids(False))
    monkeypatch.delenv("DLI_TRANSPORT", raising=False)
    monkeypatch.setenv("DLI_RCCL_PROBE_S", "3")
    world, res = 8, {}

    def rank_main(r):
        try:
            res[r] = pipeline.make_transport(r, world, torch.device("cuda", 0), job="h",
                                             rccl_timeout_s=120.0, head_pairs=head,
                                             streams=_Streams(), max_bytes=1 << 20,
                                             head_bytes=1 << 16)
        except Exception as e:  # noqa: BLE001
            res[r] = e

    th = [threading.Thread(target=rank_main, args=(r,), name=f"rank{r}") for r in range(world)]
    t0 = time.monotonic()
    for t in th:
        t.start()
    for t in th:
        t.join(60.0)
    took = time.monotonic() - t0
    assert not any(t.is_alive() for t in th), "a rank is still blocked"
    assert took <= 15.0, took
    assert all(isinstance(res[r], pipeline.TransportInitError) for r in range(world)), res
    failed_sets = {str(res[r]).split("failed on ranks ")[1].split("]")[0] for r in range(world)}
    assert len(failed_sets) == 1, failed_sets   # one agreed set of failed ranks


def test_healthy_bringup_agrees_on_rccl(monkeypatch):
    """No failure: every rank returns its RcclTransport, and a slow rank (still loading weights)
    is waited for rather than declared failed."""
    from distributed_llm_inference.parallel import pipeline
    from distributed_llm_inference.runtime import faults
    nat = _Native(fail_rank=None)
    from distributed_llm_inference import ops
    monkeypatch.setattr(ops, "native", lambda: nat)
    monkeypatch.setattr(tmod.RcclTransport, "_connect", lambda self: 0.0)
    store = _Store()
    monkeypatch.setattr(faults, "raw_store", lambda: store)
    monkeypatch.setattr(pipeline, "device_identity", _ids(False))
    monkeypatch.delenv("DLI_TRANSPORT", raising=False)
    monkeypatch.setenv("DLI_RCCL_PROBE_S", "1")
    world, res = 4, {}

    def rank_main(r):
        if r == 2:
            time.sleep(2.5)    # longer than the probe window: not a failure, it never entered
        res[r] = pipeline.make_transport(r, world, torch.device("cuda", 0), job="ok",
                                         head_pairs=True, streams=_Streams(), max_bytes=1 << 20,
                                         head_bytes=1 << 16)

    th = [threading.Thread(target=rank_main, args=(r,), name=f"rank{r}") for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(30.0)
    assert all(isinstance(res.get(r), tmod.RcclTransport) for r in range(world)), res
