"""Server layer on CPU: batching pool, inference backend, worker, HTTP service and the
supervisor's health / restart / rebalance loop with injected faults (multi-process, gloo)."""
import json
import os
import threading
import time
import urllib.request

import pytest
import torch

from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig
from distributed_llm_inference.models import LlamaBlock
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
from distributed_llm_inference.runtime.sequence import SamplingParams
from distributed_llm_inference.server.backend import BatchTensorDescriptor, InferenceBackend
from distributed_llm_inference.server.task_pool import TaskPool
from distributed_llm_inference.server.worker import InferenceWorker

SPEC = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=4,
                 num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                 max_position_embeddings=4096)


def test_task_pool_batches_and_splits():
    calls = []

    def f(x):
        calls.append(x.shape[0])
        return x * 2, x + 1

    pool = TaskPool(f, max_batch_size=8, timeout=0.05)
    futs = [pool.submit_task(torch.full((2, 3), float(i))) for i in range(4)]
    res = [fu.result(5) for fu in futs]
    for i, (a, b) in enumerate(res):
        assert torch.equal(a, torch.full((2, 3), 2.0 * i)) and torch.equal(b, torch.full((2, 3), i + 1.0))
    assert sum(calls) == 8 and max(calls) <= 8 and len(calls) < 4
    with pytest.raises(ValueError):
        pool.submit_task(torch.zeros(9, 1))
    pool.shutdown()


def test_task_pool_propagates_errors():
    pool = TaskPool(lambda x: (_ for _ in ()).throw(RuntimeError("boom")), max_batch_size=4)
    with pytest.raises(RuntimeError):
        pool.submit_task(torch.zeros(1, 1)).result(5)
    pool.shutdown()


def test_backend_plain_module_and_disabled_backward():
    lin = torch.nn.Linear(4, 3)
    be = InferenceBackend("lin", lin, args_schema=(BatchTensorDescriptor((4,), torch.float32),),
                          max_batch_size=8)
    assert be.outputs_schema == BatchTensorDescriptor((3,), torch.float32)
    assert isinstance(be.get_pools(), tuple) and be.get_pools()[0] is be.inference_pool
    x = torch.randn(2, 4)
    assert torch.allclose(be.submit(x).result(5), lin(x).detach())
    with pytest.raises(NotImplementedError):
        be.backward(x)
    with pytest.raises(NotImplementedError):
        be.on_backward(1)
    be.shutdown()


def test_block_backend_batches_sessions_like_individual_calls():
    blk = LlamaBlock(SPEC, [0, 1]).init_random(4)
    be = InferenceBackend("blk", blk, args_schema=(BatchTensorDescriptor((1, 128)),),
                          max_batch_size=64, pool_timeout=0.05)
    ref_blk = LlamaBlock(SPEC, [0, 1]).init_random(4)
    ref_cache = ref_blk.new_cache(num_blocks=64)
    xs = {g: torch.randn(1, n, 128, dtype=torch.bfloat16) for g, n in (("a", 5), ("b", 9), ("c", 2))}
    futs = {g: be.submit(x, generation_id=g) for g, x in xs.items()}
    got = {g: f.result(10)[0] for g, f in futs.items()}
    for g, x in xs.items():
        (ref,) = ref_blk(g, x, past_key_value=ref_cache)
        assert torch.allclose(got[g].float(), ref.float(), atol=3e-2, rtol=3e-2)
    # a decode step for two sessions at once
    d = {g: torch.randn(1, 1, 128, dtype=torch.bfloat16) for g in ("a", "b")}
    futs = {g: be.submit(x, generation_id=g) for g, x in d.items()}
    for g, x in d.items():
        (ref,) = ref_blk(g, x, past_key_value=ref_cache)
        assert torch.allclose(futs[g].result(10)[0].float(), ref.float(), atol=3e-2, rtol=3e-2)
    assert be.cache.get_seq_length(0, "a") == 6
    be.shutdown()


def test_inference_worker_routes_blocks():
    w = InferenceWorker(SPEC, 1, 4, layers_per_block=2, device="cpu")
    assert [b["block_index"] for b in w.block_ids] == [1, 3]
    w.run()
    assert w.is_healthy()
    h = torch.randn(2, 3, 128, dtype=torch.bfloat16)
    out = w.forward_range("s", h)
    assert out.shape == h.shape and torch.isfinite(out.float()).all()
    w.close_session("s")
    w.shutdown()


def test_worker_move_refuses_new_sessions_and_abandons_when_not_idle():
    """ADVICE r5 (rebalance race): while a move loads its layers no new session is admitted
    (WorkerMoving -> HTTP 409 at the block server); a session that slips in before the move
    started makes the move abandon at the swap (checked under the swap lock); an idle worker
    moves; a range walk keeps one snapshot of the blocks."""
    from distributed_llm_inference.server.worker import WorkerMoving
    w = InferenceWorker(SPEC, 0, 2, device="cpu")
    w.run()
    h = torch.randn(1, 2, 128, dtype=torch.bfloat16)
    real_load = w._load_range
    gate = threading.Event()
    entered = threading.Event()

    def slow_load(a, b):
        entered.set()
        gate.wait(30)
        return real_load(a, b)

    w._load_range = slow_load
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("moved", w.move_to(2, 4, require_idle=True)))
    th.start()
    assert entered.wait(30)
    with pytest.raises(WorkerMoving):
        w.forward_range("new", h)
    # a session that was admitted before the move: simulate it appearing during the load
    w.moving = False
    w.forward_range("early", h)
    w.moving = True
    gate.set()
    th.join(60)
    assert res["moved"] is False and (w.start, w.end) == (0, 2)
    assert w.sessions() == ["early"] and not w.moving
    w.close_session("early")
    w._load_range = real_load
    assert w.move_to(2, 4, require_idle=True) is True and (w.start, w.end) == (2, 4)
    out = w.forward_range("after", h)
    assert out.shape == h.shape
    w.close_session("after")
    w.shutdown()


def _engine():
    cfg = EngineConfig(model="t", cache=CacheConfig(num_blocks=128, block_size=32),
                       serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=128,
                                         max_seq_len=256, use_graphs=False))
    return LLMEngine(SPEC, cfg=cfg)


def test_engine_service_and_http():
    from fastapi.testclient import TestClient
    from distributed_llm_inference.server.http import build_app
    from distributed_llm_inference.server.service import EngineService
    eng = _engine()
    svc = EngineService(eng.pipeline)
    # concurrent clients join the running batch
    outs = [None] * 6
    def client(i):
        outs[i] = svc.generate([1 + i, 2, 3], SamplingParams(max_tokens=4 + i, ignore_eos=True), 60)
    ts = [threading.Thread(target=client, args=(i,)) for i in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert [len(o.output_ids) for o in outs] == [4, 5, 6, 7, 8, 9]
    app = TestClient(build_app(svc, model_name="t"))
    r = app.post("/generate", json={"prompt_ids": [5, 6, 7], "max_tokens": 3, "ignore_eos": True})
    assert r.status_code == 200 and len(r.json()["output_ids"]) == 3
    r = app.post("/v1/completions", json={"prompt": [9, 9], "max_tokens": 2, "ignore_eos": True})
    assert r.json()["usage"]["completion_tokens"] == 2
    with app.stream("POST", "/generate", json={"prompt_ids": [1], "max_tokens": 3,
                                                "ignore_eos": True, "stream": True}) as s:
        events = [l for l in s.iter_lines() if l.startswith("data:")]
    assert events[-1] == "data: [DONE]" and len(events) == 4
    assert app.get("/health").json()["healthy"]
    m = app.get("/metrics").text
    assert "dli_total_tokens" in m and "dli_token_latency_p50_ms" in m and "dli_ttft_p90_ms" in m
    assert app.post("/generate", json={"max_tokens": 3}).status_code == 400
    # request timeout: 504, and the sequence is aborted (its KV blocks come back)
    r = app.post("/generate", json={"prompt_ids": [4, 4], "max_tokens": 200, "ignore_eos": True,
                                    "timeout_s": 0.05})
    assert r.status_code == 504
    deadline = time.time() + 30
    while (svc.stats()["running"] or svc.stats()["waiting"]) and time.time() < deadline:
        time.sleep(0.05)
    st = svc.stats()
    assert st["running"] == 0 and st["aborted_requests"] >= 1 and st["kv_reserved_blocks"] == 0
    # a stream that times out also aborts its sequence
    with app.stream("POST", "/generate", json={"prompt_ids": [2], "max_tokens": 200,
                                                "ignore_eos": True, "stream": True,
                                                "timeout_s": 0.05}) as s:
        events = [l for l in s.iter_lines() if l.startswith("data:")]
    assert "timeout" in events[-1]
    deadline = time.time() + 30
    while svc.stats()["aborted_requests"] < 2 and time.time() < deadline:
        time.sleep(0.05)
    assert svc.stats()["aborted_requests"] >= 2
    svc.shutdown()


# ------------------------------------------------------------------------------ supervisor
def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _post(port, body, timeout=60):
    req = urllib.request.Request(f"http://127.0.0.1:{port}/generate", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


SERVER_ARGS = ["--max-seq-len", "256", "--max-batched-tokens", "128", "--max-batch", "8",
               "--no-graphs"]


@pytest.mark.slow
def test_server_restarts_after_stage_crash():
    from distributed_llm_inference.server.server import Server
    port = _free_port()
    srv = Server("tiny-llama", num_gpus=2, port=port, extra_args=SERVER_ARGS, health_interval=0.5,
                 env={"DLI_FAULT": "kill:1:6"}, startup_timeout=120)
    try:
        srv.start()
        assert srv.is_healthy()
        with pytest.raises(Exception):
            for _ in range(10):  # stage 1 dies after 6 steps -> requests fail / hang up
                _post(port, {"prompt_ids": [1, 2, 3], "max_tokens": 4, "ignore_eos": True}, 15)
        deadline = time.time() + 30
        while srv.is_healthy() and time.time() < deadline:
            time.sleep(0.2)
        assert not srv.is_healthy()
        srv.env.pop("DLI_FAULT")  # transient fault: the restarted job is clean
        srv.restart()
        assert srv.is_healthy() and srv.restarts == 1
        out = _post(port, {"prompt_ids": [1, 2, 3], "max_tokens": 4, "ignore_eos": True})
        assert len(out["output_ids"]) == 4
    finally:
        srv.stop()


@pytest.mark.slow
def test_server_rebalances_slow_stage():
    from distributed_llm_inference.server.server import Server
    port = _free_port()
    srv = Server("tiny-llama", num_gpus=2, port=port, extra_args=SERVER_ARGS, health_interval=0.5,
                 env={"DLI_FAULT": "delay:1:15"}, startup_timeout=120)
    try:
        srv.start()
        assert srv.choose_blocks() == [(0, 2), (2, 4)]
        for _ in range(4):
            _post(port, {"prompt_ids": [1, 2], "max_tokens": 12, "ignore_eos": True})
        deadline = time.time() + 30
        reb = False
        while time.time() < deadline and not reb:
            reb = srv.should_rebalance()
            time.sleep(0.3)
        assert reb
        st = srv.stage_stats()
        # traffic counters ride along with the step times: stage 0 sends, stage 1 receives
        assert st[0]["bytes_sent"] > 0 and st[1]["bytes_recv"] > 0
        m = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
        assert 'dli_stage_step_ms{stage="1"}' in m and 'dli_stage_bytes_sent{stage="0"}' in m
        new = srv.choose_blocks()
        assert new[1][1] - new[1][0] < 2  # the slow stage gets fewer layers
    finally:
        srv.stop()
