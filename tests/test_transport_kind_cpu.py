"""One definition of the default transport: the engine's head-rotation /
stage-plan decision and ``make_transport`` read the same kind list and default, so setting the
documented default explicitly changes nothing.

Reference: the health / restart intent at /root/reference/distributed_llm_inference/server/
server.py:19-23 (a stage plan must not depend on how the data plane was named)."""
import pytest
import torch

from distributed_llm_inference.config import plan_stages, resolve_model
from distributed_llm_inference.parallel.transport import (DEFAULT_GPU_TRANSPORT,
                                                          GPU_TRANSPORT_KINDS, transport_kind)
from distributed_llm_inference.runtime.engine import EngineConfig, head_rotation_wanted

GPU = torch.device("cuda", 0)   # only the device type is read: runs on the CPU
SPEC = resolve_model("llama-3-70b")
ROT = plan_stages(SPEC, 8, head_rotation=True)
NO_ROT = plan_stages(SPEC, 8, head_rotation=False)


@pytest.mark.parametrize("env,rotates", [(None, True), ("rccl", True), ("rccl-or-ipc", True),
                                         ("rccl-or-host", True), ("ipc", True), ("host", False)])
def test_rotation_and_stage_plan_per_kind(monkeypatch, env, rotates):
    monkeypatch.delenv("DLI_HEAD_ROTATION", raising=False)
    if env is None:
        monkeypatch.delenv("DLI_TRANSPORT", raising=False)
    else:
        monkeypatch.setenv("DLI_TRANSPORT", env)
    cfg = EngineConfig(model="llama-3-70b", pp=8)
    got = head_rotation_wanted(cfg, 8, GPU)
    assert got is rotates
    assert plan_stages(SPEC, 8, head_rotation=got) == (ROT if rotates else NO_ROT)
    assert transport_kind(GPU) == (env or DEFAULT_GPU_TRANSPORT)
    # the CPU always runs gloo, which rotates
    assert transport_kind(torch.device("cpu")) == "gloo"
    assert head_rotation_wanted(cfg, 8, torch.device("cpu"))


def test_unset_equals_explicit_default(monkeypatch):
    cfg = EngineConfig(model="llama-3-70b", pp=8)
    monkeypatch.delenv("DLI_TRANSPORT", raising=False)
    a = (head_rotation_wanted(cfg, 8, GPU), transport_kind(GPU))
    monkeypatch.setenv("DLI_TRANSPORT", DEFAULT_GPU_TRANSPORT)
    b = (head_rotation_wanted(cfg, 8, GPU), transport_kind(GPU))
    assert a == b == (True, "rccl-or-ipc")
    assert DEFAULT_GPU_TRANSPORT in GPU_TRANSPORT_KINDS


def test_unknown_kind_is_rejected(monkeypatch):
    monkeypatch.setenv("DLI_TRANSPORT", "nvlink")
    with pytest.raises(ValueError):
        transport_kind(GPU)
    with pytest.raises(ValueError):
        head_rotation_wanted(EngineConfig(model="llama-3-70b", pp=8), 8, GPU)


def test_rotation_overrides(monkeypatch):
    monkeypatch.delenv("DLI_TRANSPORT", raising=False)
    monkeypatch.setenv("DLI_HEAD_ROTATION", "0")
    assert not head_rotation_wanted(EngineConfig(model="llama-3-70b", pp=8), 8, GPU)
    monkeypatch.setenv("DLI_HEAD_ROTATION", "1")
    assert not head_rotation_wanted(EngineConfig(model="llama-3-70b", pp=1), 1, GPU)


def test_rccl_rank_hosts_sets_a_host_id_per_rank():
    """DLI_RCCL_RANK_HOSTS=1: each rank gets its own NCCL_HOSTID (what lets RCCL pair ranks that
    share a GPU), loopback sockets unless the user chose an interface; off by default."""
    from distributed_llm_inference.runtime.engine import rccl_rank_hosts
    env = {}
    assert not rccl_rank_hosts(3, env) and env == {}
    env = {"DLI_RCCL_RANK_HOSTS": "1", "NCCL_SOCKET_IFNAME": "eth0"}
    assert rccl_rank_hosts(3, env)
    assert env["NCCL_HOSTID"] == "dli-rehearsal-host-3"
    assert env["NCCL_SOCKET_IFNAME"] == "eth0" and env["NCCL_IB_DISABLE"] == "1"
    other = {"DLI_RCCL_RANK_HOSTS": "1"}
    rccl_rank_hosts(4, other)
    assert other["NCCL_HOSTID"] != env["NCCL_HOSTID"] and other["NCCL_SOCKET_IFNAME"] == "lo"
