"""Block registry (VERDICT r3 missing #3): block servers started WITHOUT --start/--end claim the
least-served layers from a registry, together tile [0, L), and a client builds its chain from
the registry alone; the chain matches one LlamaBlock over all layers.

Reference: the intended "choose optimal block ids" step of the server loop
(/root/reference/distributed_llm_inference/server/server.py:7-8) over hivemind's DHT."""
import os
import socket
import subprocess
import sys
import time

import pytest
import torch

from distributed_llm_inference.server.registry import Registry, choose_range, find_chain

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_choose_range_prefers_gaps_then_least_served():
    assert choose_range(8, 3, []) == (0, 3)
    assert choose_range(8, 3, [(0, 3)]) == (3, 6)
    assert choose_range(8, 3, [(0, 3), (3, 6)]) == (6, 8)
    assert choose_range(8, 3, [(0, 3), (6, 8)]) == (3, 6)
    assert choose_range(8, 8, [(2, 4)]) == (0, 2)          # the first gap, not past a served layer
    # everything covered: the window with the lowest coverage
    assert choose_range(8, 3, [(0, 3), (3, 6), (6, 8)]) == (0, 3)
    assert choose_range(8, 3, [(0, 3), (3, 6), (6, 8), (0, 3)]) == (3, 6)
    assert choose_range(8, 2, [(0, 8), (0, 4)]) == (4, 6)
    assert choose_range(4, 10, []) == (0, 4)


def test_find_chain_fewest_hops():
    es = [{"start": 0, "end": 3, "url": "a"}, {"start": 3, "end": 8, "url": "b"},
          {"start": 0, "end": 5, "url": "c"}, {"start": 5, "end": 8, "url": "d"},
          {"start": 3, "end": 5, "url": "e"}]
    assert [e["url"] for e in find_chain(es, 8)] == ["a", "b"]
    assert find_chain(es[2:3], 8) == []
    assert [e["url"] for e in find_chain([es[2], es[3]], 8)] == ["c", "d"]


def test_registry_claims_are_exclusive_and_expire():
    reg = Registry(claim_ttl=0.2)
    assert reg.claim("m", 8, 3, "u1") == (0, 3)
    assert reg.claim("m", 8, 3, "u2") == (3, 6)          # pending claims count as served
    assert reg.claim("other", 8, 3, "u3") == (0, 3)      # per model
    reg.announce("m", "u1", 0, 3, 8, ttl=60)
    time.sleep(0.3)                                      # u2 never became ready: its claim lapses
    assert [(e["url"], e["ready"]) for e in reg.servers("m")] == [("u1", True)]
    assert reg.claim("m", 8, 3, "u4") == (3, 6)
    reg.withdraw("u1")
    assert [e["url"] for e in reg.servers("m")] == ["u4"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def swarm():
    env = dict(os.environ, OMP_NUM_THREADS="2")
    distribute = os.path.join(REPO, "distribute")
    rport = _port()
    reg_url = f"http://127.0.0.1:{rport}"
    procs = [subprocess.Popen([sys.executable, distribute, "registry", "--port", str(rport)],
                              env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)]
    from distributed_llm_inference.server.registry import RegistryClient
    client = RegistryClient(reg_url, timeout=5)
    deadline = time.time() + 120
    while True:
        try:
            client.servers()
            break
        except Exception:  # noqa: BLE001
            if procs[0].poll() is not None:
                raise RuntimeError(procs[0].stderr.read().decode()[-3000:])
            if time.time() > deadline:
                raise TimeoutError("registry did not come up")
            time.sleep(0.3)
    # three block servers, no --start/--end: each claims at most 3 of the 8 layers
    for _ in range(3):
        procs.append(subprocess.Popen(
            [sys.executable, distribute, "block-serve", "--model", "tiny-llama-8l",
             "--registry", reg_url, "--max-layers", "3", "--port", str(_port()), "--device", "cpu",
             "--seed", "3"], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
    deadline = time.time() + 240
    while len(client.servers("tiny-llama-8l")) < 3:
        for p in procs:
            if p.poll() is not None:
                raise RuntimeError(p.stderr.read().decode()[-3000:])
        if time.time() > deadline:
            raise TimeoutError(f"servers: {client.servers('tiny-llama-8l', ready_only=False)}")
        time.sleep(0.5)
    yield reg_url, client
    for p in procs[1:] + procs[:1]:
        p.terminate()
    for p in procs:
        p.wait(30)


def test_registry_servers_tile_the_model_and_chain_to_one_block(swarm):
    reg_url, client = swarm
    from distributed_llm_inference.config import resolve_model
    from distributed_llm_inference.models import LlamaBlock
    from distributed_llm_inference.server.block_server import RemoteSequential
    spec = resolve_model("tiny-llama-8l")
    ranges = sorted((e["start"], e["end"]) for e in client.servers(spec.name))
    assert ranges == [(0, 3), (3, 6), (6, 8)]
    chain = RemoteSequential.from_registry(reg_url, "tiny-llama-8l")
    assert (chain.start, chain.end) == (0, spec.num_layers) and len(chain.servers) == 3
    ref = LlamaBlock(spec, list(range(spec.num_layers))).init_random(3)
    cache = ref.new_cache(num_blocks=64)
    g = torch.Generator().manual_seed(1)
    with torch.inference_mode():
        for gid, T in (("a", 6), ("b", 2), ("a", 1), ("b", 1), ("a", 1)):
            x = (torch.randn(1, T, spec.hidden_size, generator=g) * 0.5).to(torch.bfloat16)
            y, r = chain.forward(gid, x), ref(gid, x, past_key_value=cache)[0]
            assert torch.allclose(y.float(), r.float(), atol=5e-2, rtol=5e-2), \
                (y.float() - r.float()).abs().max()
    chain.close_session("a")
    chain.close_session("b")
