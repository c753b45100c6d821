"""bench.py's driver contract on the multi-rank path (torchrun, one process per stage), exercised
on the CPU with a tiny Llama so it runs here: ONE JSON line from rank 0 with the required fields,
every in-flight sequence decoding one token per timed step, the max-over-ranks timing."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"]


def _no_nan(tok):
    raise AssertionError(f"bench line is not strict JSON: {tok}")

def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_multirank_json_contract(n):
    steps, warmup, bpm = 3, 1, 4
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", str(steps),
           "--warmup", str(warmup), "--model", "tiny-llama-8l", "--batch-per-mb", str(bpm),
           "--prompt-len", "16", "--max-batched-tokens", "64"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    if r.returncode != 0:   # the ranks' own errors first: torchrun's summary hides them
        keys = ("Error", "error", "Traceback", "terminate", "abort", "Abort", "watchdog", "File ")
        own = [l for l in r.stderr.splitlines() if any(k in l for k in keys)
               and "elastic" not in l and "ChildFailedError" not in l]
        pytest.fail("\n".join(own[-60:]) + "\n---- tail ----\n" + r.stderr[-2000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0], parse_constant=_no_nan)   # strict JSON: no NaN / Infinity
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["config"]["parallelism"] == f"pp{n}" and d["scaling"] == "weak"
    assert d["micro_batches"] == n + 1
    G = d["config"]["global_batch"]
    assert G == (n + 1) * bpm and d["tokens_timed"] == steps * G
    assert abs(d["value"] - d["tokens_timed"] / (d["ms_per_step"] * steps / 1e3)) < 0.02 * d["value"]
    # per-rank diagnostics of the multi-rank path (what the 8-GPU driver run is judged on)
    assert d["transport"] == "TorchDistTransport"   # gloo on the CPU; RCCL on GPUs
    ranges = d["stage_ranges"]
    assert len(ranges) == n and ranges[0][0] == 0 and all(
        ranges[i][1] == ranges[i + 1][0] for i in range(n - 1))
    pr = d["per_rank"]
    assert [r["rank"] for r in pr] == list(range(n))
    # every hop of prefill + warm-up was digested on both ends and matched (parallel/integrity.py)
    hi = d["hop_integrity"]
    assert hi["checked"] > 0 and hi["mismatch"] == 0 and hi["missing"] == 0, hi
    assert hi["checked"] == sum(r["hop_integrity"]["sent"] for r in pr), pr
    assert all(r["hop_integrity"]["checked"] > 0 for r in pr[1:]), pr
    for r in pr:
        assert r["transport"] == "TorchDistTransport"
        # every rank ran one compute step per micro-batch step of the timed window
        assert r["mb_steps"] == steps * (n + 1), r
        assert r["device_ms_per_mb_step"] > 0
        assert r["recv_wait_ms_per_mb_step"] >= 0
        # host time per micro-batch step, by phase (runtime/hostclock.py)
        ph = r["host_ms_per_mb_step"]
        assert "launch" in ph and "stage" in ph, r
        assert ("plan" in ph and "ctrl" in ph) if r["rank"] == 0 else ("ctrl_wait" in ph), r
        assert r["host_busy_ms_per_mb_step"] > 0
    dh = d["driver_host_phases"]
    assert dh["host_busy_ms_per_mb_step"] > 0 and "tokens" in dh["host_ms_per_mb_step"]
    H = 128  # tiny-llama-8l hidden size (bf16 activations)
    mb_bytes = bpm * H * 2
    T = steps * (n + 1)   # decode micro-batch steps in the window
    head = []             # rotating LM head (runtime/head.py): normed hidden states last -> r
    for i, r in enumerate(pr):
        stage_sent = T * mb_bytes if i < n - 1 else 0
        stage_recv = T * mb_bytes if i > 0 else 0
        if i < n - 1:
            assert r["bytes_sent"] == stage_sent, r
            extra = r["bytes_recv"] - stage_recv
            assert extra >= 0 and extra % mb_bytes == 0, r
            head.append(extra // mb_bytes)
        else:
            assert r["bytes_recv"] == stage_recv, r
            assert r["bytes_sent"] % mb_bytes == 0, r
            assert r["bytes_sent"] // mb_bytes == sum(head), (r, head)
            head.append(T - sum(head))   # steps whose head stayed on the last stage
    # every rank projected + sampled its 1/n share of the steps (step % n)
    assert all(T // n <= h <= -(-T // n) for h in head), head


@pytest.mark.parametrize("n,dp", [(4, 2), (2, 2)])
def test_bench_replicas_json_contract(n, dp):  # noqa: C901
    """``--dp``: dp independent pipeline replicas of n/dp stages (dp2 x pp2 over gloo, and two
    single-stage replicas); one JSON line whose tokens count every replica's sequences."""
    steps, warmup, bpm = 3, 1, 4
    pp = n // dp
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(n), "--dp", str(dp), "--steps", str(steps),
           "--warmup", str(warmup), "--model", "tiny-llama-8l", "--batch-per-mb", str(bpm),
           "--prompt-len", "16", "--max-batched-tokens", "64"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    if r.returncode != 0:   # the ranks' own errors first: torchrun's summary hides them
        keys = ("Error", "error", "Traceback", "terminate", "abort", "Abort", "watchdog", "File ")
        own = [l for l in r.stderr.splitlines() if any(k in l for k in keys)
               and "elastic" not in l and "ChildFailedError" not in l]
        pytest.fail("\n".join(own[-60:]) + "\n---- tail ----\n" + r.stderr[-2000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0], parse_constant=_no_nan)   # strict JSON: no NaN / Infinity
    for k in REQUIRED:
        assert k in d, k
    assert d["config"]["parallelism"] == f"dp{dp}xpp{pp}"
    assert d["replicas"] == dp and d["stages_per_replica"] == pp
    M = pp + 1 if pp > 1 else 1
    assert d["micro_batches"] == M
    G = d["config"]["global_batch"]
    assert G == dp * M * bpm and d["tokens_timed"] == steps * G
    assert abs(d["value"] - d["tokens_timed"] / (d["ms_per_step"] * steps / 1e3)) < 0.02 * d["value"]
    pr = d["per_rank"]
    assert [r["rank"] for r in pr] == list(range(n))
    assert [r["replica"] for r in pr] == [i // pp for i in range(n)]
    for rep in range(dp):
        rr = [r["stage"] for r in pr if r["replica"] == rep]
        assert rr[0][0] == 0 and rr[-1][1] == 8 and all(
            rr[i][1] == rr[i + 1][0] for i in range(len(rr) - 1))
