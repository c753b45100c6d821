#!/usr/bin/env python3
"""Headline benchmark: output tokens/s (whole node) + p50 per-token latency, Llama-3-70B, PP=N.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU; stage i of an N-stage pipeline (``plan_stages``) on GPU i; hidden states
move over RCCL P2P (xGMI), the control plane over shared memory.  Random-init weights of the real
Llama-3-70B architecture (bf16), synthetic random prompts.  Every stage always runs micro-batches of
``--batch-per-mb`` (512) sequences: N=1 runs ONE micro-batch (a single stage has nothing to overlap
with; 512-row GEMMs are 15-25 % cheaper per token than 256-row ones), N>1 keeps M = N+1 micro-batches
in flight so all N stages stay busy while tokens return to the driver.  Work per GPU per step is
fixed as N grows, so the scaling mode is "weak".  A "step" = every in-flight sequence decodes one token.  Timed region:
barrier + device sync -> exactly K decode steps -> barrier + device sync; the max over ranks is
reported.  Prefill and W warmup steps (incl. hipGraph capture) run before the timed region.

``--dp D`` (default 1) instead runs D independent pipeline replicas of N/D stages each (DP x PP:
e.g. dp8 = eight whole-model Llama-3-70B replicas, one per GPU; dp2 x pp4).  Every replica's
driver plans and times its own sequences; the replicas start and stop the timed window together
(barrier over the drivers) and ``value`` is the tokens of ALL replicas / the slowest replica's
window.  The BASELINE headline stays the default PP=N layout.
"""
from __future__ import annotations

import os

# Before torch / any HIP call: RCCL's cross-process buffer sharing on this ROCm needs the dmabuf
# IPC mode (the legacy mode fails with `hipIpcGetMemHandle: invalid argument`); the driver runs this
# file directly under torchrun, not through distributed_llm_inference.launcher.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# per-rank device time per micro-batch step and RCCL receive stalls (HIP events; cheap)
os.environ.setdefault("DLI_STAGE_TIMING", "1")
# every hop's payload digested on both ends during prefill + warm-up, checked at the barrier that
# opens the timed window (parallel/integrity.py): a corrupted or mis-routed pipeline fails the run
# instead of reporting tokens/s.  Off inside the timed window.
os.environ.setdefault("DLI_HOP_CHECK", "1")

import argparse  # noqa: E402
import json  # noqa: E402
import random  # noqa: E402
import statistics  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "output tokens/sec (whole node) + p50 token latency, Llama-3-70B PP=8"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--dp", type=int, default=1,
                    help="pipeline replicas (DP x PP, world = dp x pp); default 1 = one PP=N pipeline")
    ap.add_argument("--batch-per-mb", type=int, default=512)
    ap.add_argument("--micro-batches", type=int, default=0, help="0 = N+1 (N=1: 1)")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-batched-tokens", type=int, default=16384)
    ap.add_argument("--fp8", action="store_true", help="fp8-e4m3 weights (BASELINE config 5)")
    ap.add_argument("--int8", action="store_true",
                    help="LLM.int8 weights (the reference's 8-bit mode: int8 MFMA + bf16 outliers)")
    ap.add_argument("--kv-fp8", action="store_true", help="fp8-e4m3 KV cache")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kernels", default="",
                    help="kernel policy overrides (config.KernelPolicy), e.g. fp8_gemm4=gate_up")
    ap.add_argument("--num-layers", type=int, default=0,
                    help="REHEARSAL ONLY: the model's width with this many layers (e.g. 16 = 2 per "
                         "stage at PP=8, so 8 ranks x 9 micro-batches x 512 rows fit one GPU); the "
                         "result names the reduced model and is not a headline number")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


_T0 = time.perf_counter()
_PHASE = {"phase": "start"}


def _progress(msg: str) -> None:
    """Progress on stderr (a long multi-rank init / prefill must never look hung)."""
    _PHASE["phase"] = msg
    print(f"[bench rank {os.environ.get('RANK', '0')} +{time.perf_counter() - _T0:.0f}s] {msg}",
          file=sys.stderr, flush=True)


def _heartbeat(every_s: float = 30.0) -> None:
    import threading

    def run():
        while True:
            time.sleep(every_s)
            print(f"[bench rank {os.environ.get('RANK', '0')} +{time.perf_counter() - _T0:.0f}s] "
                  f"alive: {_PHASE['phase']}", file=sys.stderr, flush=True)
    threading.Thread(target=run, name="bench-heartbeat", daemon=True).start()


def _rank_record(node, rank: int, window_s: float) -> dict:
    """This rank's share of the timed window (between the last two barriers): stage range,
    data-plane transport, device compute per micro-batch step, receive stalls, traffic."""
    from distributed_llm_inference.runtime.faults import snapshot_delta
    rec = {"rank": rank, "replica": getattr(node, "replica", 0),
           "head_rotation": bool(getattr(node, "head_rotation", False))}
    ex = getattr(node, "ex", None)
    if ex is None:   # a single-stage replica (LocalPipeline): the whole model, no transport
        exs = node.executors
        rec.update({"stage": [exs[0].stage.start, exs[-1].stage.end], "device": str(exs[0].device),
                    "transport": "none"})
        return rec
    rec.update({"stage": [ex.stage.start, ex.stage.end], "device": str(ex.device)})
    rec.update(node.tr.describe())
    ig = getattr(node.tr, "integrity", None)
    if ig is not None:
        rec["hop_integrity"] = ig.summary()
    if len(node.snapshots) >= 2:
        from distributed_llm_inference.runtime.hostclock import per_step
        d = snapshot_delta(node.snapshots[-2], node.snapshots[-1])
        n = max(int(d.get("steps", 0)), 1)
        rec.update(per_step(d, n))
        rec.update({
            "mb_steps": int(d.get("steps", 0)),
            "device_ms_per_mb_step": round(d.get("device_ms", 0.0) / n, 3),
            "device_busy_frac": round(d.get("device_ms", 0.0) / 1e3 / window_s, 4) if window_s else None,
            "recv_wait_ms_per_mb_step": round(d.get("recv_wait_ms", 0.0) / n, 3),
            "bytes_sent": int(d.get("bytes_sent", 0)), "bytes_recv": int(d.get("bytes_recv", 0)),
        })
    return rec


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    from distributed_llm_inference import _build
    from distributed_llm_inference.config import (CacheConfig, KernelPolicy, ServeConfig,
                                                  resolve_model)
    from distributed_llm_inference.runtime.engine import EngineConfig, init_pipeline_rank
    from distributed_llm_inference.runtime.sequence import SamplingParams, Sequence

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run (one rank per GPU)")
        raise SystemExit(f"WORLD_SIZE={world} != --gpus={a.gpus}")
    if a.dp < 1 or a.gpus % a.dp:
        raise SystemExit(f"--dp {a.dp} must divide --gpus {a.gpus}")
    dp, pp = a.dp, a.gpus // a.dp
    os.environ.setdefault("DLI_PROGRESS", "1")   # init phases on stderr (runtime/engine.py)
    _heartbeat()
    if rank == 0:
        _build.build_all()
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    spec = resolve_model(a.model)
    model = a.model
    if a.num_layers:
        # host-path rehearsal at the real width / row count with fewer layers (never a headline)
        spec = spec.replace(num_layers=a.num_layers, name=f"{spec.name}-{a.num_layers}L")
        model = spec
    M = a.micro_batches or (pp + 1 if pp > 1 else 1)
    G = M * a.batch_per_mb
    # sequences prefilled in the first prefill round keep decoding through the remaining ones
    # (each round admits up to M x max_batched_tokens prompt tokens): none may reach max_tokens
    # before the end of the timed window
    prefill_rounds = -(-G * a.prompt_len // (M * a.max_batched_tokens))
    max_tokens = a.warmup + a.steps + 64 + prefill_rounds
    total_len = a.prompt_len + max_tokens + 8
    cfg = EngineConfig(
        model=model, random_init=True, seed=0, quantize="int8" if a.int8 else a.fp8, pp=pp, dp=dp,
        kernels=KernelPolicy().with_overrides(a.kernels),
        cache=CacheConfig(block_size=64, gpu_memory_utilization=0.92,
                          dtype="fp8" if a.kv_fp8 else "bf16"),
        serve=ServeConfig(max_batch_size=a.batch_per_mb, max_num_batched_tokens=a.max_batched_tokens,
                          num_micro_batches=M, max_seq_len=total_len, use_graphs=not a.no_graphs,
                          graph_batch_sizes=[a.batch_per_mb]))
    t_init = time.perf_counter()
    _progress("init")
    role, obj = init_pipeline_rank(cfg)
    _progress(f"init done ({role})")

    def world_reduce(elapsed: float, toks: int, rec: dict):
        """Same collectives on every rank, in the same order: max window, summed tokens, records."""
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n = torch.tensor([toks], dtype=torch.int64)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        recs = [None] * world
        dist.all_gather_object(recs, rec)
        dist.barrier()
        return float(t.item()), int(n.item()), recs

    if role == "follower":
        _progress("serving the driver's steps")
        obj.run()
        _progress("stopped")
        interval = obj.barrier_times[-1] - obj.barrier_times[-2] if len(obj.barrier_times) >= 2 else 0.0
        world_reduce(interval, 0, _rank_record(obj, rank, interval))
        obj.close()
        dist.destroy_process_group()
        return
    drv = obj
    dgroup = getattr(drv, "drivers_group", None)

    def sync_replicas():
        if dgroup is not None:
            dist.barrier(group=dgroup)

    init_s = time.perf_counter() - t_init
    rng = random.Random(1234 + 7919 * getattr(drv, "replica", 0))
    # generous max_tokens (above): none may finish inside the timed window (constant batch)
    params = SamplingParams(max_tokens=max_tokens, ignore_eos=True)
    seqs = [Sequence([rng.randrange(spec.vocab_size) for _ in range(a.prompt_len)], params)
            for _ in range(G)]
    for s in seqs:
        drv.sched.add(s)
    # prefill: run until every sequence produced its first token
    t_pf = time.perf_counter()
    _progress(f"prefill of {G} prompts x {a.prompt_len} tokens")
    n_rounds = 0
    while any(len(s.output) == 0 for s in seqs):
        drv.round()
        n_rounds += 1
        if n_rounds % 20 == 0:
            _progress(f"prefill: {sum(len(s.output) > 0 for s in seqs)}/{G} prompts done")
    prefill_s = time.perf_counter() - t_pf
    _progress(f"prefill done in {prefill_s:.1f}s; warmup")
    for _ in range(a.warmup):
        drv.round()
    drv.barrier()
    sync_replicas()
    n0 = sum(len(s.output) for s in seqs)
    for s in seqs:
        s.token_times.clear()
    _progress(f"timed: {a.steps} steps")
    from distributed_llm_inference.runtime.hostclock import HOST, per_step
    h0 = HOST.snapshot()
    t0 = time.perf_counter()
    w0 = drv.wait_s
    for _ in range(a.steps):
        drv.round()
    drv.barrier()
    t1 = time.perf_counter()
    h1 = HOST.snapshot()
    _progress(f"timed window {t1 - t0:.2f}s")
    sync_replicas()
    driver_busy = (t1 - t0) - (drv.wait_s - w0)
    n1 = sum(len(s.output) for s in seqs)
    elapsed = t1 - t0
    toks_mine = n1 - n0
    toks = toks_mine
    if world > 1:
        drv.stop()
        elapsed, toks, per_rank = world_reduce(elapsed, toks_mine, _rank_record(drv, rank, elapsed))
    if rank != 0:   # another replica's driver: rank 0 reports for the whole node
        drv.close()
        dist.destroy_process_group()
        return
    if toks_mine != a.steps * G or toks != a.steps * G * dp:
        print(f"WARNING: {toks} tokens in the timed window, expected {a.steps * G * dp} "
              "(KV cache too small to run every sequence at once?)", file=sys.stderr, flush=True)
    lat = []
    for s in seqs:
        tt = s.token_times
        lat += [(tt[i + 1] - tt[i]) * 1e3 for i in range(len(tt) - 1)]
    # None (JSON null, never NaN: the line must stay strict JSON) when too few intervals
    p50 = round(statistics.median(lat), 3) if lat else None
    p90 = round(statistics.quantiles(lat, n=10)[-1], 3) if len(lat) >= 10 else None
    value = toks / elapsed
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": a.gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("int8-weights/bf16-act" if a.int8 else "fp8-weights/bf16-act" if a.fp8 else "bf16")
                 + ("/fp8-kv" if a.kv_fp8 else ""),
        "data": f"synthetic (random-init {spec.name} weights, random prompt tokens)",
        "config": {"model": "Llama-3-70B" if (a.model == "llama-3-70b" and not a.num_layers)
                   else spec.name,
                   "global_batch": G * dp, "seq_len": total_len,
                   "parallelism": f"pp{pp}" if dp == 1 else f"dp{dp}xpp{pp}"},
        "p50_token_latency_ms": p50,
        "p90_token_latency_ms": p90,
        "transport": drv.tr.describe()["transport"] if (world > 1 and pp > 1) else "none",
        "kernel_policy": a.kernels or "default",
        "micro_batches": M,
        "batch_per_micro_batch": a.batch_per_mb,
        "prompt_len": a.prompt_len,
        "tokens_timed": toks,
        "prefill_s": round(prefill_s, 3),
        # host time of the driver rank per micro-batch step NOT spent waiting for results
        "driver_host_ms_per_mb_step": round(driver_busy / (a.steps * M) * 1e3, 3),
        # ... and by phase (runtime/hostclock.py; waits on the device / token channel apart)
        "driver_host_phases": per_step({k: h1[k] - h0.get(k, 0.0) for k in h1}, a.steps * M),
        "replicas": dp, "stages_per_replica": pp,
        "init_s": round(init_s, 1),
        "kv_blocks": int(drv.sched.total_blocks),
        "kv_blocks_needed": int(G * drv.sched.blocks_for(a.prompt_len + params.max_tokens)),
    }
    bad_hops = False
    if world > 1:
        igs = [r["hop_integrity"] for r in per_rank if "hop_integrity" in r]
        if igs:
            res["hop_integrity"] = {k: sum(int(g.get(k, 0)) for g in igs)
                                    for k in ("checked", "mismatch", "missing")}
            bad_hops = res["hop_integrity"]["mismatch"] > 0 or res["hop_integrity"]["missing"] > 0
        res["stage_ranges"] = [r["stage"] for r in per_rank]
        res["head_rotation"] = any(r.get("head_rotation") for r in per_rank)
        fb = sorted({r["fallback_from"] for r in per_rank if r.get("fallback_from")})
        if fb:   # the data plane is NOT RCCL: say so at the top level, not only per rank
            res["transport_fallback_from"] = fb
        res["per_rank"] = per_rank
    if a.num_layers:
        res["rehearsal"] = f"{a.num_layers} of {resolve_model(a.model).num_layers} layers"
        res["vs_baseline"] = None
    if a.model != "llama-3-70b" or a.num_layers:
        # the headline metric names its model; a run of another model says what it measured
        res["metric"] = (f"output tokens/sec (whole node) + p50 token latency, "
                         f"{res['config']['model']} PP={pp}")
    line = json.dumps(res)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    if world > 1:
        drv.close()
        dist.destroy_process_group()
    if bad_hops:
        print(f"ERROR: pipeline hop integrity failed: {res['hop_integrity']} (per rank: "
              f"{[r.get('hop_integrity') for r in per_rank]})", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(5)


if __name__ == "__main__":
    try:
        main()
    except SystemExit:   # argparse (--help, bad flags) and explicit exits: no abort broadcast
        raise
    except BaseException as e:
        # a failed rank ends every rank promptly, each printing its last pipeline op
        # (distributed_llm_inference/runtime/watchdog.py); no-op for a single process
        import traceback
        traceback.print_exc()
        from distributed_llm_inference.runtime.watchdog import abort_job
        abort_job(f"bench.py: {type(e).__name__}: {e}")
        raise
    # multi-rank runs, done (rank 0's JSON line is out): leave without interpreter finalisation —
    # daemon threads (watchdog, heartbeat, transport pollers) may still sit in C++ store / gloo
    # calls, and tearing their objects down under them ended a finished rank with SIGABRT
    # ("terminate called without an active exception") now and then on a loaded machine.  A
    # single process exits normally (a profiler's exit hooks write its trace then).
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        sys.exit(0)
    try:
        import torch
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:  # noqa: BLE001
        pass
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)
