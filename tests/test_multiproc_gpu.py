"""Multi-process pipeline on the GPU (one process per stage).

On a ONE-GPU box stage processes share the card (``DLI_SHARE_GPU=1``).  RCCL refuses two ranks on
the same device, so there the full driver/follower GPU path (graphs, shm control plane, token
feedback, micro-batching) runs over the host-staged transport, the RCCL binding is exercised with
a 1-rank communicator, and the RCCL-failure path (all ranks agree, fall back together) is tested
by asking for RCCL on a shared GPU: with an explicit ``DLI_TRANSPORT=rccl`` every rank fails
loudly and ``DLI_TRANSPORT=rccl-or-host`` falls back to host staging.  The default (unset:
``rccl-or-ipc``) compares the ranks' PCI devices and takes the IPC device transport on a shared
GPU without trying RCCL (strict RCCL on distinct GPUs).  RCCL itself also runs on the one GPU
when every rank claims its own host (``NCCL_HOSTID``, :func:`_rank_hosts`): real communicators,
bytes over RCCL's loopback socket transport (the PP=2/4 strict-RCCL pipeline tests).  With two or
more GPUs the RCCL P2P transport and a PP=2 RCCL pipeline are tested over xGMI.
"""
import multiprocessing as mp
import os
import socket
import traceback

import pytest
import torch

pytestmark = pytest.mark.gpu

PROMPTS = [list(range(3, 40)), [7, 8, 9], list(range(200, 330)), [11], [5, 5, 5, 5]]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(world, mbs):
    from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig
    from distributed_llm_inference.runtime.engine import EngineConfig
    spec = ModelSpec(name="t", vocab_size=1000, hidden_size=256, intermediate_size=512,
                     num_layers=4, num_heads=8, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                     max_position_embeddings=4096)
    cfg = EngineConfig(model=spec, pp=world, seed=5,  # type: ignore[arg-type]
                       cache=CacheConfig(num_blocks=256, block_size=64),
                       serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=512,
                                         max_seq_len=1024, num_micro_batches=mbs,
                                         graph_batch_sizes=[1, 2, 4, 8]))
    return spec, cfg


def _rank_hosts(rank):
    """Each rank claims a host of its own (``NCCL_HOSTID``).  RCCL's duplicate-device check
    compares (host, PCI bus id) pairs, so ranks that share the one GPU are then accepted and
    connected through RCCL's network transport.  Here that is TCP sockets on loopback, not xGMI,
    but the communicators, the grouped send/recv on the transport's streams and the hop digests
    are the production code.  Must be set before the process makes any RCCL call."""
    os.environ.update(NCCL_HOSTID=f"dli-rehearsal-host-{rank}", NCCL_SOCKET_IFNAME="lo",
                      NCCL_IB_DISABLE="1")


def _pipeline_worker(rank, world, port, mbs, q, transport="host", rotation=None,
                     rank_hosts=False):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLI_SHARE_GPU="1",
                          DLI_TUNING_DIR="off", DLI_WATCHDOG_S="60")
        if rank_hosts:
            _rank_hosts(rank)
        if transport is None:   # the default
            os.environ.pop("DLI_TRANSPORT", None)
        else:
            os.environ["DLI_TRANSPORT"] = transport
        if rotation is not None:
            os.environ["DLI_HEAD_ROTATION"] = "1" if rotation else "0"
        import torch.distributed as dist
        from distributed_llm_inference.runtime.engine import init_pipeline_rank
        from distributed_llm_inference.runtime.sequence import SamplingParams
        _, cfg = _cfg(world, mbs)
        role, obj = init_pipeline_rank(cfg)
        if role == "driver":
            out = obj.generate(PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))
            obj.stop()
            kind = type(obj.tr).__name__
            obj.close()
            q.put(("ok", [s.output for s in out], kind))
        else:
            obj.run()
            obj.close()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc(), None))
        raise


@pytest.mark.parametrize("world,mbs", [(2, 3), (4, 5)])
def test_multiprocess_pipeline_on_gpu(gpu, world, mbs):
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    os.environ["DLI_TUNING_DIR"] = "off"
    spec, cfg = _cfg(1, mbs)
    ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
        PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_pipeline_worker, args=(r, world, port, mbs, q)) for r in range(world)]
    for p in ps:
        p.start()
    status, got, *_ = q.get(timeout=600)
    for p in ps:
        p.join(120)
    assert status == "ok", got
    assert all(p.exitcode == 0 for p in ps)
    assert got == ref


@pytest.mark.parametrize("world,mbs,rotation", [(2, 3, True), (4, 5, True), (4, 5, False)])
def test_multiprocess_pipeline_ipc_transport(gpu, world, mbs, rotation):
    """Stage processes sharing the GPU over the IPC device transport (parallel/ipc_transport.py):
    receives are spinning device waits on the rank's dedicated recv / head streams, exactly the
    production RCCL stream schedule, and with ``rotation`` the rotating LM head's GPU branch runs
    (HeadJobs deferred enqueue, head-stream receive + graph replay, per-rank token channels).
    Tokens must equal PP=1's."""
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    os.environ["DLI_TUNING_DIR"] = "off"
    spec, cfg = _cfg(1, mbs)
    ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
        PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_pipeline_worker, args=(r, world, port, mbs, q, "ipc", rotation))
          for r in range(world)]
    for p in ps:
        p.start()
    status, got, kind = q.get(timeout=600)
    for p in ps:
        p.join(120)
    assert status == "ok", got
    assert kind == "IpcTransport"
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    assert got == ref


def _ipc_timeout_worker(rank, port, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), DLI_P2P_TIMEOUT_S="2")
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from distributed_llm_inference.parallel.ipc_transport import IpcTransport
        from distributed_llm_inference.runtime.faults import raw_store
        from distributed_llm_inference.runtime.streams import RankStreams
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        rs = RankStreams(dev)
        tr = IpcTransport(raw_store(), rank, 2, dev, rs, max_bytes=1 << 16)
        if rank == 0:   # one message, then silence
            tr.send(torch.ones(1024, device=dev, dtype=torch.bfloat16), 1)
            torch.cuda.synchronize()
            q.put(("sent", None))
        else:
            x = torch.empty(1024, device=dev, dtype=torch.bfloat16)
            tr.recv(x, 0)
            torch.cuda.synchronize()
            ok = bool((x == 1).all())
            tr.recv(x, 0)            # never sent: the device wait hits its 2 s deadline
            torch.cuda.synchronize()
            try:
                tr.check()
                q.put(("no-timeout", ok))
            except TimeoutError as e:
                q.put(("timeout", (ok, str(e))))
        dist.barrier()
        tr.close()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc()))


def test_ipc_transport_wait_deadline_is_reported(gpu):
    """A receive whose sender never arrives: the spinning device wait exits at its deadline
    (DLI_P2P_TIMEOUT_S) and the transport raises TimeoutError naming the channel - no wave is
    left spinning, the process exits normally."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_ipc_timeout_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    assert "sent" in res, res
    assert "timeout" in res, res
    ok, msg = res["timeout"]
    assert ok and "stage 0->1" in msg and "receive" in msg, res
    assert all(p.exitcode == 0 for p in ps)


def _run_pair(transport, timeout=600):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_pipeline_worker, args=(r, 2, port, 3, q, transport)) for r in range(2)]
    for p in ps:
        p.start()
    msgs = [q.get(timeout=timeout)]
    for p in ps:
        p.join(120)
    while not q.empty():
        msgs.append(q.get(timeout=5))
    return msgs, ps


def test_rccl_failure_is_loud_when_strict(gpu):
    """Two ranks on ONE GPU with ``DLI_TRANSPORT=rccl``: RCCL rejects the duplicate device and
    EVERY rank must raise TransportInitError (agreed through the store: no hang, no silent
    host-staged fallback, non-zero exit codes)."""
    msgs, ps = _run_pair("rccl")
    assert msgs and all(m[0] == "err" for m in msgs), msgs
    assert any("TransportInitError" in m[1] and "RCCL transport unavailable" in m[1] for m in msgs)
    assert all(p.exitcode not in (0, None) for p in ps), [p.exitcode for p in ps]


def test_rccl_failure_falls_back_with_opt_in(gpu):
    """``DLI_TRANSPORT=rccl-or-host``: the same RCCL failure, agreed on by all ranks, falls back
    together to the host-staged transport, producing the same tokens as PP=1."""
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    os.environ["DLI_TUNING_DIR"] = "off"
    spec, cfg = _cfg(1, 3)
    ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
        PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))]
    msgs, ps = _run_pair("rccl-or-host")
    status, got, *rest = msgs[0]
    assert status == "ok", got
    assert all(p.exitcode == 0 for p in ps)
    assert got == ref
    assert rest and rest[0] == "HostStagedTransport", rest


def test_default_transport_on_a_shared_gpu_is_ipc(gpu):
    """``DLI_TRANSPORT`` unset: both ranks publish the same PCI device, so every rank brings up the
    IPC device transport (rotating head kept) without trying RCCL, producing PP=1's tokens."""
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    os.environ["DLI_TUNING_DIR"] = "off"
    spec, cfg = _cfg(1, 3)
    ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
        PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))]
    msgs, ps = _run_pair(None)
    status, got, *rest = msgs[0]
    assert status == "ok", got
    assert all(p.exitcode == 0 for p in ps)
    assert got == ref
    assert rest and rest[0] == "IpcTransport", rest


def _rccl_worker(rank, port, q, rank_hosts=False):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        if rank_hosts:
            _rank_hosts(rank)
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from distributed_llm_inference.parallel.transport import RcclTransport
        from distributed_llm_inference.runtime.faults import raw_store
        dev = torch.device("cuda", 0 if rank_hosts else rank)
        torch.cuda.set_device(dev)
        tr = RcclTransport(raw_store(), rank, 2, dev, timeout_s=120.0)
        for n in (1 << 10, 8 << 20):  # a decode-sized and a prefill-sized hidden-state message
            x = torch.arange(n, device=dev, dtype=torch.float32) * (rank + 1)
            if rank == 0:
                tr.send(x, 1)
                torch.cuda.synchronize()
            else:
                y = torch.empty_like(x)
                tr.recv(y, 0)
                torch.cuda.synchronize()
                if not torch.equal(y, torch.arange(n, device=dev, dtype=torch.float32)):
                    q.put(("bad", n))
                    break
        else:
            q.put(("ok", None))
        dist.barrier()
        tr.close()
        dist.destroy_process_group()
    except Exception as e:
        q.put(("err", repr(e)))


two_gpus = pytest.mark.skipif(torch.cuda.device_count() < 2,
                              reason="needs 2 GPUs (RCCL refuses two ranks on one device; the "
                                     "1-GPU box covers the fallback path instead)")


@two_gpus
def test_rccl_p2p_two_gpus(gpu):
    """RcclTransport between two real GPUs (xGMI): send/recv of decode- and prefill-sized
    messages on the transport's dedicated streams."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rccl_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
    assert all(s == "ok" for s, _ in res), res


def test_rccl_p2p_one_gpu_rank_hosts(gpu):
    """RcclTransport with two ranks on the ONE GPU, each claiming its own host (_rank_hosts): real
    RCCL communicators and send/recv of decode- and prefill-sized messages on the transport's
    streams (bytes over RCCL's loopback socket transport)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rccl_worker, args=(r, port, q, True)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
    assert all(s == "ok" for s, _ in res), res
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]


@pytest.mark.parametrize("world,mbs", [(2, 3), (4, 5)])
def test_multiprocess_pipeline_rccl_one_gpu_rank_hosts(gpu, world, mbs):
    """The PP pipeline over strict RCCL (``DLI_TRANSPORT=rccl``) on the one GPU, each rank its own
    RCCL host: RCCL pair and rotating-head communicators, hop digests checked, tokens equal
    PP=1's."""
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    os.environ["DLI_TUNING_DIR"] = "off"
    spec, cfg = _cfg(1, mbs)
    ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
        PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_pipeline_worker, args=(r, world, port, mbs, q, "rccl", None, True))
          for r in range(world)]
    for p in ps:
        p.start()
    status, got, kind = q.get(timeout=600)
    for p in ps:
        p.join(120)
    assert status == "ok", got
    assert kind == "RcclTransport", kind
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    assert got == ref


def _pipeline_worker_gpus(rank, world, port, q):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLI_TUNING_DIR="off",
                          DLI_TRANSPORT="rccl")
        os.environ.pop("DLI_SHARE_GPU", None)
        import torch.distributed as dist
        from distributed_llm_inference.runtime.engine import init_pipeline_rank
        from distributed_llm_inference.runtime.sequence import SamplingParams
        _, cfg = _cfg(world, world + 1)
        role, obj = init_pipeline_rank(cfg)
        if role == "driver":
            out = obj.generate(PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))
            obj.stop()
            kind = type(obj.tr).__name__
            obj.close()
            q.put(("ok", [s.output for s in out], kind))
        else:
            obj.run()
            obj.close()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", traceback.format_exc(), None))
        raise


@two_gpus
def test_multiprocess_pipeline_rccl_two_gpus(gpu):
    """PP=2 over RCCL P2P between two GPUs equals PP=1 (same micro-batch count)."""
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    os.environ["DLI_TUNING_DIR"] = "off"
    spec, cfg = _cfg(1, 3)
    ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
        PROMPTS, SamplingParams(max_tokens=8, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_pipeline_worker_gpus, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    status, got, *rest = q.get(timeout=600)
    for p in ps:
        p.join(120)
    assert status == "ok", got
    assert rest and rest[0] == "RcclTransport", rest
    assert got == ref


def test_rccl_single_rank_self_p2p_and_collectives(gpu):
    """The RCCL binding on real hardware with a 1-rank communicator: send/recv to self inside a
    group on explicit streams, all_reduce / broadcast / all_gather."""
    from distributed_llm_inference import ops
    C = ops.native()
    assert C.rccl_version() > 0
    comm = C.RcclComm(bytes(C.rccl_unique_id()), 0, 1, 0)
    s = torch.cuda.Stream()
    x = torch.arange(4096, device=gpu, dtype=torch.bfloat16)
    y = torch.zeros_like(x)
    comm.group_start()
    comm.send(x, 0, s.cuda_stream)
    comm.recv(y, 0, s.cuda_stream)
    comm.group_end()
    s.synchronize()
    assert torch.equal(x, y)
    z = torch.ones(1000, device=gpu)
    comm.all_reduce(z)
    comm.broadcast(z, 0)
    out = torch.empty(1000, device=gpu)
    comm.all_gather(z, out)
    torch.cuda.synchronize()
    assert torch.equal(out, z)
    comm.destroy()
