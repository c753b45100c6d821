"""Remote hidden-state block forward (server/block_server.py), on the CPU.

A client process chains two block-server processes that hold disjoint layer ranges of one model
(the reference's swarm: a client sends hidden_states + generation_id to the server owning layers
[a, b), reference server/backend.py:31-42, server/worker.py:9-20).  The chain must match ONE
LlamaBlock over all layers: prefill, incremental decode keyed by generation_id with two
interleaved sessions, and close_session (a closed id starts from an empty cache again)."""
import os
import socket
import subprocess
import sys
import time

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def servers():
    procs, urls = [], []
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for (a, b) in ((0, 2), (2, 4)):
        port = _port()
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(REPO, "distribute"), "block-serve", "--model", "tiny-llama",
             "--start", str(a), "--end", str(b), "--port", str(port), "--device", "cpu",
             "--seed", "3"], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
        urls.append(f"http://127.0.0.1:{port}")
    from distributed_llm_inference.server.block_server import RemoteBlocks
    deadline = time.time() + 180
    for u, p in zip(urls, procs):
        c = RemoteBlocks(u)
        while not c.healthy():
            if p.poll() is not None:
                raise RuntimeError(p.stderr.read().decode()[-3000:])
            if time.time() > deadline:
                raise TimeoutError(u)
            time.sleep(0.5)
    yield urls
    for p in procs:
        p.terminate()
    for p in procs:
        p.wait(30)


def test_chained_block_servers_match_one_block(servers):
    from distributed_llm_inference.config import resolve_model
    from distributed_llm_inference.models import LlamaBlock
    from distributed_llm_inference.server.block_server import RemoteSequential
    spec = resolve_model("tiny-llama")
    chain = RemoteSequential(list(reversed(servers)))   # the client orders them by layer range
    assert (chain.start, chain.end) == (0, spec.num_layers)
    ref = LlamaBlock(spec, list(range(spec.num_layers))).init_random(3)
    cache = ref.new_cache(num_blocks=64)
    H = spec.hidden_size
    g = torch.Generator().manual_seed(0)

    def rnd(*shape):
        return (torch.randn(*shape, generator=g) * 0.5).to(torch.bfloat16)

    def close(a, b):
        assert a.shape == b.shape
        assert torch.allclose(a.float(), b.float(), atol=5e-2, rtol=5e-2), \
            (a.float() - b.float()).abs().max()

    with torch.inference_mode():
        # prefill two sessions, then interleaved decode steps
        prompts = {"s1": rnd(1, 7, H), "s2": rnd(1, 3, H)}
        for gid, x in prompts.items():
            close(chain.forward(gid, x), ref(gid, x, past_key_value=cache)[0])
        for _ in range(3):
            for gid in ("s2", "s1"):
                x = rnd(1, 1, H)
                close(chain.forward(gid, x), ref(gid, x, past_key_value=cache)[0])
        # closing a session frees it on every server: the same id starts from scratch
        chain.close_session("s1")
        cache.close_session("s1")
        x = rnd(1, 4, H)
        close(chain.forward("s1", x), ref("s1", x, past_key_value=cache)[0])
        # ... while the other session keeps its history
        x = rnd(1, 1, H)
        close(chain.forward("s2", x), ref("s2", x, past_key_value=cache)[0])


def test_block_server_rejects_bad_requests(servers):
    from distributed_llm_inference.server.block_server import RemoteBlocks
    c = RemoteBlocks(servers[0])
    with pytest.raises(RuntimeError, match="hidden must be"):
        c.forward("x", torch.zeros(1, 2, 7, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match="unknown block"):
        c.forward("x", torch.zeros(1, 2, 128, dtype=torch.bfloat16), block_id="nope")
    info = c.info()
    assert info["start"] == 0 and info["end"] == 2 and info["blocks"]
