"""The RCCL data plane end to end on the CPU: a PP=4 / PP=8 multi-process pipeline whose hidden
states and rotating-head traffic go through :class:`RcclTransport` itself - its pair and head
communicators, the peer index inside every 2-rank pair, the connect plan, ``describe()`` - over a
SIMULATED communicator (a one-GPU box cannot run two RCCL ranks, and round 4 had only simulated
failed bring-ups).  Generated tokens must equal the single-stage engine's.

The fake stands in for csrc/comm/rccl_p2p.hip's ``rccl_unique_id`` / ``RcclComm``: a 2-rank
communicator keyed by its unique id, whose members register in the job's TCP store; ``send`` is
asynchronous (the message is posted to the store, like an RCCL send enqueued on a stream) and
``recv`` blocks until the message with the next sequence number in that direction exists.  It
checks what a real communicator would reject or silently mis-route: a peer index that is not the
other member, a size mismatch between the send and the receive, and a send in the wrong direction
of a pipeline pair."""
import multiprocessing as mp
import os
import socket

import pytest
import torch

from distributed_llm_inference.config import CacheConfig, ServeConfig, resolve_model
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
from distributed_llm_inference.runtime.sequence import SamplingParams

SPEC = resolve_model("tiny-llama-8l")
PROMPTS = [list(range(3, 40)), [7, 8, 9], list(range(100, 190)), [11], list(range(20, 33))]


class _FakeComm:
    def __init__(self, native, uid: bytes, idx: int, nranks: int):
        assert nranks == 2 and idx in (0, 1)
        self.n, self.uid, self.idx = native, uid.hex(), idx
        self.sent = self.recvd = 0
        self.n.store.set(f"fk/{self.uid}/member/{idx}", str(self.n.global_rank))
        self.n.comms.append(self)

    # -- RcclComm API
    @property
    def rank(self):
        return self.idx

    @property
    def world(self):
        return 2

    def ready(self) -> bool:
        return bool(self.n.store.check([f"fk/{self.uid}/member/{1 - self.idx}"]))

    def peer_rank(self) -> int:
        return int(self.n.store.get(f"fk/{self.uid}/member/{1 - self.idx}"))

    def send(self, t: torch.Tensor, peer: int, stream: int) -> None:
        assert peer == 1 - self.idx, f"send to peer index {peer} from index {self.idx}"
        assert stream == 0, "the CPU path is host-synchronous"
        assert t.device.type == "cpu" and t.is_contiguous()
        key = f"fk/{self.uid}/{self.idx}->{peer}/{self.sent}"
        self.sent += 1
        raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
        flip = os.environ.get("FAKE_FLIP")   # "<global rank>:<n>": corrupt this rank's n-th send
        if flip and raw and int(flip.split(":")[0]) == self.n.global_rank:
            self.n.sends += 1
            if self.n.sends == int(flip.split(":")[1]):
                b = bytearray(raw)
                b[len(b) // 2] ^= 0x10          # one bit of one byte, mid-payload
                raw = bytes(b)
        self.n.store.set(key, raw if raw else b"\0")
        self.n.log.append(("send", self.peer_rank(), t.numel()))

    def recv(self, t: torch.Tensor, peer: int, stream: int) -> None:
        assert peer == 1 - self.idx, f"recv from peer index {peer} at index {self.idx}"
        key = f"fk/{self.uid}/{peer}->{self.idx}/{self.recvd}"
        self.recvd += 1
        raw = self.n.store.get(key)
        self.n.store.delete_key(key)
        nb = t.numel() * t.element_size()
        if nb == 0:
            return
        assert len(raw) == nb, f"receive of {nb} bytes matched a send of {len(raw)}"
        t.view(torch.uint8).view(-1).copy_(torch.frombuffer(bytearray(raw), dtype=torch.uint8))
        self.n.log.append(("recv", self.peer_rank(), t.numel()))

    def destroy(self):
        self.n.destroyed += 1

    def abort(self):
        pass


class _FakeNative:
    """The slice of the ``_C`` extension that RcclTransport uses."""

    def __init__(self, global_rank: int):
        from distributed_llm_inference.runtime.faults import raw_store
        self.store = raw_store()
        self.global_rank = global_rank
        self.comms, self.log, self.destroyed, self.sends = [], [], 0, 0

    def rccl_version(self):
        return 22606

    def rccl_unique_id(self):
        return os.urandom(16)

    def RcclComm(self, uid, idx, nranks, dev, timeout_s, wait=True):
        return _FakeComm(self, bytes(uid), idx, nranks)


def _cfg(pp):
    return EngineConfig(model=SPEC, pp=pp, seed=3,
                        cache=CacheConfig(num_blocks=256, block_size=32, max_chunk=64),
                        serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=64,
                                          max_seq_len=512, use_graphs=False))


def _worker(rank, world, port, q, params, env=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLI_HEAD_ROTATION="1")
    os.environ.update(env or {})
    import torch.distributed as dist
    from distributed_llm_inference import ops
    from distributed_llm_inference.parallel import transport as tmod
    from distributed_llm_inference.runtime.engine import init_pipeline_rank
    # the CPU default is gloo: take the RCCL data plane instead, over the simulated communicator
    tmod.transport_kind = lambda device: "rccl"
    natives = []

    def native():
        if not natives:
            natives.append(_FakeNative(rank))
        return natives[0]
    ops.native = native
    role, obj = init_pipeline_rank(_cfg(world))
    tr = obj.tr
    rep = {"rank": rank, "type": type(tr).__name__, "describe": tr.describe(),
           "rotation": obj.head_rotation}
    if role == "driver":
        out = obj.generate(PROMPTS, params)
        obj.barrier()   # the hop-integrity check runs here (DLI_HOP_CHECK)
        obj.stop()
        rep["tokens"] = [s.output for s in out]
    else:
        obj.run()
    ig = getattr(tr, "integrity", None)
    rep["hop"] = ig.summary() if ig is not None else None
    rep["traffic"] = tr.traffic()
    rep["log"] = natives[0].log
    obj.close()
    rep["destroyed"] = natives[0].destroyed
    q.put(rep)
    dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, params, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, params, env))
          for r in range(world)]
    for p in ps:
        p.start()
    reps = {}
    for _ in range(world):
        r = q.get(timeout=300)
        reps[r["rank"]] = r
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return reps


@pytest.mark.parametrize("world", [4, 8])
def test_rccl_transport_dataplane_pipeline_equals_pp1(world):
    params = SamplingParams(max_tokens=6, temperature=0.8, top_k=30, seed=11, ignore_eos=True)
    ref = [s.output for s in LLMEngine(SPEC, cfg=_cfg(1)).generate(PROMPTS, params)]
    reps = _run(world, params, {"DLI_HOP_CHECK": "1"})
    assert reps[0]["tokens"] == ref
    # every hop of the run was digested on both ends and matched
    hops = [rep["hop"] for rep in reps.values()]
    assert all(h is not None and h["mismatch"] == 0 and h["missing"] == 0 for h in hops), hops
    assert sum(h["checked"] for h in hops) == sum(h["sent"] for h in hops) > 0
    assert all(reps[r]["hop"]["checked"] > 0 for r in range(1, world)), hops   # stage + head
    last = world - 1
    for r, rep in reps.items():
        assert rep["type"] == "RcclTransport" and rep["rotation"], rep
        d = rep["describe"]
        assert d["transport"] == "RcclTransport" and d["connect_ms"] >= 0
        # stage pairs: (r-1, r) and (r, r+1), this rank's index inside each
        want = {}
        if r > 0:
            want[str(r - 1)] = {"rank": 1, "size": 2}
        if r < last:
            want[str(r + 1)] = {"rank": 0, "size": 2}
        assert d["pair_comms"] == want, d
        # head pairs: the last stage holds one per other rank, every other rank one with the last
        assert d["head_comms"] == (list(range(last)) if r == last else [last]), d
        # every communicator was torn down by close()
        assert rep["destroyed"] == len(want) + len(d["head_comms"])
    # the rotating head really moved traffic over the head pairs: a rank r < last never has a
    # stage pair it RECEIVES on from the last stage, so every such receive is head traffic
    # (normed hidden states, whole decode micro-batches); each rank got its turns
    H = SPEC.hidden_size
    for r in range(last):
        head_recvs = [e for e in reps[r]["log"] if e[0] == "recv" and e[1] == last]
        assert head_recvs[0][2] == 64, head_recvs   # the connect probe (RcclTransport._connect)
        assert len(head_recvs) > 1 and all(e[2] % H == 0 for e in head_recvs[1:]), (r, head_recvs)
    to_heads = {e[1] for e in reps[last]["log"] if e[0] == "send"}
    assert to_heads == set(range(last)), to_heads
    # stage bytes balance: everything sent was received
    tot_sent = sum(rep["traffic"]["bytes_sent"] for rep in reps.values())
    tot_recv = sum(rep["traffic"]["bytes_recv"] for rep in reps.values())
    assert tot_sent == tot_recv > 0


def test_hop_integrity_catches_one_flipped_byte():
    """The simulated communicator corrupts ONE bit of ONE message (rank 1's third send, a stage
    hop to rank 2): the receiving rank's digest disagrees with the sender's and the run reports
    exactly that mismatch; every other hop still matches."""
    params = SamplingParams(max_tokens=4, ignore_eos=True)
    reps = _run(4, params, {"DLI_HOP_CHECK": "1", "FAKE_FLIP": "1:3"})
    hops = {r: rep["hop"] for r, rep in reps.items()}
    assert sum(h["mismatch"] for h in hops.values()) == 1, hops
    assert hops[2]["mismatch"] == 1 and "stage/1-2/" in hops[2]["failures"][0], hops[2]
    assert all(h["missing"] == 0 for h in hops.values()), hops
