"""DP x PP replica placement (parallel/replicas.py, runtime/engine.py ReplicaLayout) on the CPU:
layout arithmetic, 2 replicas x PP=2 over gloo producing the PP=1 tokens, the shared-memory
request bridge between rank 0's router and a remote replica's EngineService, and the CLI plan."""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import threading
import time
import uuid

import pytest

from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig
from distributed_llm_inference.parallel.replicas import (RemoteReplica, ReplicaRouter, ReplicaServer,
                                                        deal, undeal)
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine, ReplicaLayout
from distributed_llm_inference.runtime.sequence import SamplingParams

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPEC = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=4,
                 num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                 max_position_embeddings=4096)
PROMPTS = [list(range(3, 40)), [7, 8, 9], list(range(100, 190)), [11], [5, 6], [1, 2, 3, 4, 5]]


def _cfg(pp=1, dp=1):
    return EngineConfig(model="t", pp=pp, dp=dp, seed=3,
                        cache=CacheConfig(num_blocks=256, block_size=32, max_chunk=64),
                        serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=64,
                                          max_seq_len=512, use_graphs=False))


def test_layout_and_deal():
    lay = ReplicaLayout.for_world(8, 2)
    assert (lay.dp, lay.pp) == (2, 4)
    assert lay.ranks(1) == [4, 5, 6, 7] and lay.drivers() == [0, 4]
    assert [lay.replica(r) for r in range(8)] == [0] * 4 + [1] * 4
    assert [lay.stage(r) for r in range(8)] == [0, 1, 2, 3] * 2
    d = lay.describe(ModelSpec(name="x", num_layers=80))
    assert len(d["replicas"]) == 2 and d["replicas"][1]["stages"][0]["rank"] == 4
    with pytest.raises(ValueError):
        ReplicaLayout.for_world(6, 4)
    items = list(range(11))
    shares = [deal(items, 3, r) for r in range(3)]
    assert shares[1] == [1, 4, 7, 10] and undeal(shares, 11) == items


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, dp, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from distributed_llm_inference.parallel.replicas import replica_generate
    from distributed_llm_inference.runtime.engine import init_pipeline_rank
    cfg = _cfg(pp=world // dp, dp=dp)
    cfg.model = SPEC  # type: ignore[assignment]
    role, obj = init_pipeline_rank(cfg)
    if role == "driver":
        out = replica_generate(obj, PROMPTS, SamplingParams(max_tokens=6, ignore_eos=True))
        kind = type(obj).__name__
        obj.stop()
        obj.close()
        if out is not None:
            q.put(([s.output for s in out], kind, obj.replica))
    else:
        obj.run()
        obj.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,dp", [(4, 2), (2, 2)])
def test_replicas_generate_equals_single_stage(world, dp):
    """2 replicas x PP=2 (and 2 single-stage replicas): prompts dealt over the replicas, every
    replica's tokens identical to one PP=1 engine's, reassembled in prompt order on rank 0."""
    ref = [s.output for s in LLMEngine(SPEC, cfg=_cfg()).generate(
        PROMPTS, SamplingParams(max_tokens=6, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_dp_worker, args=(r, world, dp, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got, kind, rep = q.get(timeout=240)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert rep == 0 and got == ref
    assert kind == ("DistributedDriver" if world // dp > 1 else "LocalPipeline")


def _engine():
    cfg = EngineConfig(model="t", cache=CacheConfig(num_blocks=128, block_size=32),
                       serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=128,
                                         max_seq_len=256, use_graphs=False))
    return LLMEngine(SPEC, cfg=cfg)


def test_router_over_local_and_remote_replica():
    """ReplicaRouter over an in-process EngineService and a RemoteReplica whose ReplicaServer
    (another EngineService) is reached through the shm request / event channels: requests are
    spread over both, outputs equal a direct generation, streaming, abort and stats work."""
    from distributed_llm_inference.server.service import EngineService
    job = uuid.uuid4().hex[:10]
    svc0 = EngineService(_engine().pipeline)
    svc1 = EngineService(_engine().pipeline)
    server = {}

    def run_server():
        server["rs"] = ReplicaServer(svc1, job, 1, stats_every_s=0.05)
        server["rs"].serve_forever()

    th = threading.Thread(target=run_server, daemon=True)
    th.start()
    remote = RemoteReplica(job, 1)
    router = ReplicaRouter([svc0, remote])
    p = SamplingParams(max_tokens=5, ignore_eos=True)
    ref = [c.output_ids for c in [svc0.generate(pr, p, 60) for pr in PROMPTS]]
    futs = [router.submit(pr, p)[0] for pr in PROMPTS]
    res = [f.result(60) for f in futs]
    assert [r.output_ids for r in res] == ref
    assert {f.replica for f in futs} == {0, 1}            # both replicas served requests
    fut, q = router.submit([1, 2, 3], SamplingParams(max_tokens=4, ignore_eos=True), stream=True)
    toks = []
    while True:
        t = q.get(timeout=60)
        if t is None:
            break
        toks.append(t)
    assert toks == fut.result(60).output_ids and len(toks) == 4
    # streaming straight through the remote replica: every token arrives before the stream ends
    # ('done' is sent by the forwarding thread after the last token, never ahead of it)
    for n in (1, 3, 6):
        fut, q = remote.submit([4, 5, 6, n], SamplingParams(max_tokens=n, ignore_eos=True),
                               stream=True)
        toks = []
        while True:
            t = q.get(timeout=60)
            if t is None:
                break
            toks.append(t)
        assert toks == fut.result(60).output_ids and len(toks) == n, (n, toks)
    # equal loads rotate over the replicas instead of always picking replica 0
    seen = set()
    for _ in range(2):
        f, _ = router.submit([3, 3], SamplingParams(max_tokens=1, ignore_eos=True))
        f.result(60)
        seen.add(f.replica)
    assert seen == {0, 1}
    # abort a long request on whichever replica it landed
    fut, _ = router.submit([9, 9], SamplingParams(max_tokens=250, ignore_eos=True))
    time.sleep(0.2)
    router.abort(fut.seq_id)
    assert fut.result(60).finish_reason == "abort"
    deadline = time.time() + 10
    st = router.stats()
    while st["replica1_healthy"] is False and time.time() < deadline:
        time.sleep(0.05)
        st = router.stats()
    assert st["replicas"] == 2 and st["healthy"], st
    assert st["total_requests"] >= len(PROMPTS) + 2
    router.shutdown()
    th.join(10)
    assert not th.is_alive()
    server["rs"].close()
    svc0.shutdown()
    svc1.shutdown()


def test_cli_plan_dp():
    r = subprocess.run([sys.executable, "-m", "distributed_llm_inference.cli", "plan", "--model",
                        "llama-3-70b", "--gpus", "8", "--dp", "2"], capture_output=True, text=True,
                       timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["layout"] == "dp2xpp4" and len(d["replicas"]) == 2
    assert [s["rank"] for s in d["replicas"][1]["stages"]] == [4, 5, 6, 7]
    assert d["replicas"][1]["stages"][-1]["layers"][1] == 80


def test_cli_generate_dp():
    """``distribute generate --gpus 2 --dp 2`` (two single-stage replicas over gloo)."""
    r = subprocess.run([sys.executable, "-m", "distributed_llm_inference.cli", "generate",
                        "--model", "tiny-llama", "--gpus", "2", "--dp", "2", "--no-graphs",
                        "--max-seq-len", "128", "--max-batched-tokens", "64", "--max-batch", "4",
                        "--prompt-ids", "1,2,3", "--prompt-ids", "4,5", "--prompt-ids", "6",
                        "--max-tokens", "3", "--ignore-eos"],
                       capture_output=True, text=True, timeout=240, cwd=REPO,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [x["prompt_ids"] for x in recs] == [[1, 2, 3], [4, 5], [6]]
    assert all(len(x["output_ids"]) == 3 for x in recs)
