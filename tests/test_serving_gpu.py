"""User-facing paths on the GPU: the `distribute generate` CLI on a sharded HF-format checkpoint
(safetensors loader -> stage -> HIP kernels -> hipGraph decode) and the HTTP server lifecycle
(`Server` -> `distribute worker --action serve` -> EngineService -> FastAPI)."""
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _spec():
    from distributed_llm_inference.config import PRESETS
    # head_dim 128 (the attention kernels' shape), N multiples of 256 (tile GEMM eligible)
    return PRESETS["tiny-llama"].replace(name="gpu-tiny-llama", vocab_size=1024, hidden_size=512,
                                         intermediate_size=1024, num_layers=3, num_heads=4,
                                         num_kv_heads=2, head_dim=128)


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    from distributed_llm_inference.utils.model import save_random_checkpoint
    path = str(tmp_path_factory.mktemp("ckpt"))
    save_random_checkpoint(_spec(), path, seed=3, shard_layers=2)
    return path


def _env():
    e = dict(os.environ)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    return e


def test_distribute_generate_cli_from_checkpoint(gpu, ckpt):
    cmd = [sys.executable, os.path.join(REPO, "distribute"), "generate", "--model", ckpt,
           "--checkpoint", ckpt, "--gpus", "1", "--prompt-ids", "1,5,9,13", "--prompt-ids", "7,8",
           "--max-tokens", "6", "--ignore-eos", "--max-seq-len", "128", "--max-batch", "4",
           "--max-batched-tokens", "64"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [x["prompt_ids"] for x in recs] == [[1, 5, 9, 13], [7, 8]]
    for x in recs:
        assert len(x["output_ids"]) == 6 and all(0 <= t < 1024 for t in x["output_ids"])
    # greedy decoding is deterministic: a second run (fresh process, fresh graphs) agrees
    r2 = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert [json.loads(l) for l in r2.stdout.splitlines() if l.startswith("{")] == recs


def _free_port():
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


def test_http_server_on_gpu(gpu, ckpt):
    from distributed_llm_inference.server.server import Server
    port = _free_port()
    srv = Server(ckpt, num_gpus=1, port=port, checkpoint=ckpt,
                 extra_args=["--max-seq-len", "128", "--max-batched-tokens", "64", "--max-batch", "4"],
                 health_interval=0.5, startup_timeout=180)
    try:
        srv.start()
        assert srv.is_healthy()
        outs = [_post(port, {"prompt_ids": [1, 2, 3 + i], "max_tokens": 5, "ignore_eos": True})
                for i in range(3)]
        for o in outs:
            assert len(o["output_ids"]) == 5
    finally:
        srv.stop()
