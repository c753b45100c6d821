"""``distribute`` — command-line entry point (the reference's ``distribute`` file is empty).

    distribute plan     --model llama-3-70b --gpus 8 [--dp 2]
    distribute generate --model llama-3-8b --gpus 2 --prompt-ids 1,2,3 --max-tokens 32
    distribute serve    --model llama-3-70b --gpus 8 --port 8000 [--tokenizer DIR] [--dp 8]
    distribute bench    --gpus 8 --steps 20 --warmup 5 [--dp 2]  (bench.py under the launcher)
    distribute block-serve --model llama-3-8b --start 0 --end 16 --port 8100   (swarm block server)
    distribute registry --port 8099                                           (swarm block registry)
    distribute block-serve --model llama-3-8b --registry http://h:8099 --max-layers 16 --port 8100

One process per GPU (``launcher.launch``); each process owns one pipeline stage (``plan_stages``).
``--dp D`` splits the GPUs into D independent pipeline replicas of gpus/D stages (DP x PP,
``parallel/replicas.py``): ``generate`` deals the prompts over the replicas, ``serve`` puts one
HTTP front end (rank 0) over all of them.  The first rank of every replica is its driver
(scheduler + stage 0); the other ranks run the stage follower loop until their driver stops them.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
from typing import List, Optional

log = logging.getLogger("distribute")


def _common(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--model", default="llama-3-8b", help="preset name or HF config/checkpoint dir")
    ap.add_argument("--checkpoint", default=None, help="HF safetensors dir (default: random init)")
    ap.add_argument("--gpus", type=int, default=1, help="processes = GPUs (= dp x pipeline stages)")
    ap.add_argument("--dp", type=int, default=1,
                    help="pipeline replicas (data parallel); each gets gpus/dp stages")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fp8", action="store_true", help="fp8-e4m3 weights")
    ap.add_argument("--int8", action="store_true",
                    help="LLM.int8 weights (int8 MFMA + bf16 outlier columns), the reference's mode")
    ap.add_argument("--int8-threshold", type=float, default=6.0,
                    help="LLM.int8 outlier threshold (bitsandbytes / reference default 6.0 / 5.0)")
    ap.add_argument("--kv-dtype", choices=["bf16", "fp8"], default="bf16",
                    help="KV cache element type (fp8 = e4m3, half the bytes)")
    ap.add_argument("--window", type=int, default=0, help="attention-sink window length (0=full)")
    ap.add_argument("--sinks", type=int, default=0, help="attention-sink tokens")
    ap.add_argument("--block-size", type=int, default=64)
    ap.add_argument("--gpu-mem", type=float, default=0.90)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--max-seq-len", type=int, default=8192)
    ap.add_argument("--micro-batches", type=int, default=0)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kernels", default="",
                    help="kernel policy overrides, e.g. gemm4=0,fp8_gemm4=gate_up "
                         "(config.KernelPolicy fields)")
    ap.add_argument("--transport", default=None,
                    choices=["rccl-or-ipc", "rccl", "rccl-or-host", "ipc", "host"],
                    help="pipeline data plane (default rccl-or-ipc: RCCL on distinct GPUs, IPC "
                         "when stages share one)")
    ap.add_argument("--tokenizer", default=None, help="HF tokenizer dir (local files only)")
    ap.add_argument("-v", "--verbose", action="store_true")


def engine_config(a):
    from .config import CacheConfig, KernelPolicy, ServeConfig
    from .runtime.engine import EngineConfig
    if getattr(a, "transport", None):
        os.environ["DLI_TRANSPORT"] = a.transport   # read by every rank's make_transport
    return EngineConfig(
        kernels=KernelPolicy().with_overrides(getattr(a, "kernels", "")),
        model=a.model, checkpoint=a.checkpoint, random_init=a.checkpoint is None, seed=a.seed,
        quantize="fp8" if a.fp8 else ("int8" if a.int8 else False),
        int8_threshold=a.int8_threshold, pp=a.gpus // max(1, a.dp), dp=a.dp,
        cache=CacheConfig(block_size=a.block_size, gpu_memory_utilization=a.gpu_mem,
                          window_length=a.window, num_sink_tokens=a.sinks, dtype=a.kv_dtype),
        serve=ServeConfig(max_batch_size=a.max_batch, max_num_batched_tokens=a.max_batched_tokens,
                          num_micro_batches=a.micro_batches, max_seq_len=a.max_seq_len,
                          use_graphs=not a.no_graphs))


def load_tokenizer(path: Optional[str]):
    if not path:
        return None
    from transformers import AutoTokenizer
    return AutoTokenizer.from_pretrained(path, local_files_only=True)


# ------------------------------------------------------------------------------ actions
def cmd_plan(a) -> int:
    from .config import plan_stages, resolve_model
    from .models.llama.cache import KVPool
    from .runtime.engine import ReplicaLayout
    spec = resolve_model(a.checkpoint or a.model)
    layout = ReplicaLayout.for_world(a.gpus, a.dp)
    rotate = layout.pp > 1 and os.environ.get("DLI_HEAD_ROTATION", "1") == "1"
    ranges = plan_stages(spec, layout.pp, head_rotation=rotate)
    per_layer = spec.layer_param_count() * (1 if (a.fp8 or a.int8) else 2)
    emb = spec.vocab_size * spec.hidden_size * 2
    replicas = []
    for r in range(layout.dp):
        out = []
        for i, (s, e) in enumerate(ranges):
            # every rank holds the LM head when it rotates (runtime/head.py)
            w = (e - s) * per_layer + (emb if i == 0 else 0) + (
                emb if (i == len(ranges) - 1 or rotate) else 0)
            free = 288e9 * a.gpu_mem - w
            kv_tok = KVPool.bytes_per_block(spec, e - s, 1, 1 if a.kv_dtype == "fp8" else 2)
            out.append(dict(stage=i, rank=r * layout.pp + i, gpu=r * layout.pp + i, layers=[s, e],
                            weights_gb=round(w / 1e9, 2),
                            kv_capacity_tokens=int(max(0, free) // kv_tok)))
        replicas.append(dict(replica=r, driver_rank=r * layout.pp, stages=out))
    res = {"model": spec.name, "num_layers": spec.num_layers, "dp": layout.dp, "pp": layout.pp,
           "lm_head": "rotating over the pipeline ranks (decode)" if rotate else "last stage",
           "layout": f"dp{layout.dp}xpp{layout.pp}" if layout.dp > 1 else f"pp{layout.pp}",
           "stages": replicas[0]["stages"]}
    if layout.dp > 1:
        res["replicas"] = replicas
    print(json.dumps(res, indent=1))
    return 0


def cmd_block_serve(a) -> int:
    """One block server (reference server/worker.py intent): layers [start, end) behind HTTP.
    With ``--registry`` the range is claimed from the block registry (the least-served layers,
    reference server/server.py:7-8) instead of given."""
    from .server.block_server import serve_blocks
    from .server.worker import InferenceWorker
    logging.basicConfig(level=logging.WARNING)
    registry, url = None, None
    start, end = a.start, a.end
    if a.registry:
        from .config import resolve_model
        from .server.registry import RegistryClient
        spec = resolve_model(a.checkpoint or a.model)
        registry = RegistryClient(a.registry, token=a.registry_token)
        url = a.public_url or f"http://{a.host}:{a.port}"
        if start is None or end is None:
            start, end = registry.claim(spec.name, spec.num_layers,
                                        a.max_layers or spec.num_layers, url)
            print(f"block-serve: registry {a.registry} assigned layers [{start}, {end}) to {url}",
                  file=sys.stderr, flush=True)
    elif start is None or end is None:
        print("block-serve: give --start and --end, or --registry", file=sys.stderr)
        return 2
    worker = InferenceWorker(a.model, start, end, layers_per_block=a.layers_per_block,
                             device=a.device, random_init=a.checkpoint is None,
                             checkpoint=a.checkpoint, max_batch_size=a.max_batch_size,
                             window_length=a.window, num_sink_tokens=a.sinks, seed=a.seed)
    serve_blocks(worker, a.host, a.port, registry=registry, url=url,
                 rebalance_s=a.rebalance_s if registry is not None else 0.0,
                 max_layers=a.max_layers)
    return 0


def cmd_registry(a) -> int:
    """The block registry (server/registry.py): block servers claim layers, clients find chains."""
    from .server.registry import serve_registry
    logging.basicConfig(level=logging.WARNING)
    serve_registry(a.host, a.port, token=a.token)
    return 0


def _spawn_self(a, action: str, argv: List[str]) -> int:
    from .launcher import launch
    return launch(a.gpus, ["-m", "distributed_llm_inference.cli", "worker", "--action", action] + argv)


def cmd_worker(a) -> int:
    """Per-rank entry (started by the launcher)."""
    import torch.distributed as dist
    from .runtime.engine import init_pipeline_rank
    from .runtime.sequence import SamplingParams
    logging.basicConfig(level=logging.INFO if a.verbose else logging.WARNING,
                        format=f"[rank {os.environ.get('RANK', '0')}] %(levelname)s %(name)s: %(message)s")
    cfg = engine_config(a)
    role, obj = init_pipeline_rank(cfg)
    if role == "follower":
        obj.run()
        obj.close()
        if dist.is_initialized():
            dist.destroy_process_group()
        return 0
    drv = obj
    tok = load_tokenizer(a.tokenizer)
    layout = getattr(drv, "layout", None)
    dp = layout.dp if layout is not None else 1
    rep = getattr(drv, "replica", 0)
    try:
        if a.action == "generate":
            from .parallel.replicas import replica_generate
            prompts = []
            if a.prompt_ids:
                prompts = [[int(x) for x in p.split(",") if x] for p in a.prompt_ids]
            for p in a.prompt or []:
                if tok is None:
                    raise SystemExit("--prompt needs --tokenizer (or use --prompt-ids)")
                prompts.append(tok.encode(p))
            if not prompts:
                raise SystemExit("no prompts (use --prompt-ids 1,2,3 or --prompt TEXT)")
            params = SamplingParams(max_tokens=a.max_tokens, temperature=a.temperature,
                                    top_k=a.top_k, top_p=a.top_p, seed=a.sample_seed,
                                    ignore_eos=a.ignore_eos)
            outs = replica_generate(drv, prompts, params)
            for s in outs or []:
                rec = {"prompt_ids": s.prompt, "output_ids": s.output,
                       "finish_reason": s.finish_reason}
                if tok is not None:
                    rec["text"] = tok.decode(s.output, skip_special_tokens=True)
                print(json.dumps(rec), flush=True)
        elif a.action == "serve":
            from .server.http import serve
            from .server.service import EngineService
            svc = EngineService(drv, eos_token_id=getattr(drv.sched, "eos", None))
            try:
                if dp == 1:
                    serve(svc, a.host, a.port, tok, a.model, a.request_timeout)
                else:
                    _serve_replicas(a, svc, rep, dp, tok)
            finally:
                svc.shutdown(stop_driver=False)
        else:
            raise SystemExit(f"unknown action {a.action}")
    finally:
        drv.stop()
        drv.close()
        if dist.is_initialized():
            dist.destroy_process_group()
    return 0


def _serve_replicas(a, svc, rep: int, dp: int, tok) -> None:
    """DP serving: rank 0 hosts the HTTP front end over a :class:`ReplicaRouter`; every other
    replica driver serves rank 0's requests through a :class:`ReplicaServer`."""
    import torch.distributed as dist
    from .parallel.replicas import RemoteReplica, ReplicaRouter, ReplicaServer
    from .server.http import serve
    job = dist.distributed_c10d._get_default_store().get("dli_job").decode()
    if rep == 0:
        router = ReplicaRouter([svc] + [RemoteReplica(job, r) for r in range(1, dp)])
        try:
            serve(router, a.host, a.port, tok, a.model, a.request_timeout)
        finally:
            router.shutdown()
    else:
        rs = ReplicaServer(svc, job, rep)
        try:
            rs.serve_forever()
        finally:
            rs.close()


def _gen_args(ap):
    ap.add_argument("--prompt", action="append", help="text prompt (repeatable; needs --tokenizer)")
    ap.add_argument("--prompt-ids", action="append", help="comma-separated token ids (repeatable)")
    ap.add_argument("--max-tokens", type=int, default=32)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top-k", type=int, default=0)
    ap.add_argument("--top-p", type=float, default=1.0)
    ap.add_argument("--sample-seed", type=int, default=None)
    ap.add_argument("--ignore-eos", action="store_true")


def _serve_args(ap):
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--request-timeout", type=float, default=None,
                    help="abort (504) requests still running after this many seconds")


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="distribute", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("plan", help="print the stage placement and memory plan")
    _common(p)
    g = sub.add_parser("generate", help="offline generation")
    _common(g)
    _gen_args(g)
    s = sub.add_parser("serve", help="HTTP server (rank 0) over the pipeline")
    _common(s)
    _serve_args(s)
    b = sub.add_parser("bench", help="headline benchmark (bench.py) on N GPUs")
    b.add_argument("--gpus", type=int, default=1)
    b.add_argument("--dp", type=int, default=1, help="pipeline replicas (DP x PP)")
    b.add_argument("rest", nargs=argparse.REMAINDER)
    bs = sub.add_parser("block-serve",
                        help="serve a layer range's hidden-state forward over HTTP (swarm block server)")
    bs.add_argument("--model", default="llama-3-8b", help="preset name or HF config/checkpoint dir")
    bs.add_argument("--checkpoint", default=None, help="HF safetensors dir (default: random init)")
    bs.add_argument("--start", type=int, default=None, help="first layer (inclusive)")
    bs.add_argument("--end", type=int, default=None, help="last layer (exclusive)")
    bs.add_argument("--registry", default=None,
                    help="block registry URL: claim the least-served layers (or announce "
                         "--start/--end when given)")
    bs.add_argument("--max-layers", type=int, default=None,
                    help="with --registry: most layers this server holds (default: all)")
    bs.add_argument("--registry-token", default=None,
                    help="shared secret of a registry started with --token")
    bs.add_argument("--public-url", default=None,
                    help="with --registry: URL clients reach this server at (default http://host:port)")
    bs.add_argument("--rebalance-s", type=float, default=0.0,
                    help="with --registry: every this many seconds, move to less-served layers "
                         "when that raises the swarm's least-served coverage (0 = never)")
    bs.add_argument("--layers-per-block", type=int, default=None)
    bs.add_argument("--seed", type=int, default=0)
    bs.add_argument("--device", default=None, help="cuda:N / cpu (default: cuda:0 if present)")
    bs.add_argument("--max-batch-size", type=int, default=64)
    bs.add_argument("--window", type=int, default=0)
    bs.add_argument("--sinks", type=int, default=0)
    bs.add_argument("--host", default="127.0.0.1")
    bs.add_argument("--port", type=int, default=8100)
    rg = sub.add_parser("registry", help="block registry: servers claim layer ranges, clients find chains")
    rg.add_argument("--host", default="127.0.0.1")
    rg.add_argument("--port", type=int, default=8099)
    rg.add_argument("--token", default=None,
                    help="shared secret required by /claim, /announce and /withdraw (Bearer); "
                         "without it the registry must only be reachable from a trusted network")
    w = sub.add_parser("worker", help=argparse.SUPPRESS)
    _common(w)
    _gen_args(w)
    _serve_args(w)
    w.add_argument("--action", required=True)
    a = ap.parse_args(argv)
    if a.cmd == "plan":
        return cmd_plan(a)
    if a.cmd == "worker":
        return cmd_worker(a)
    if a.cmd == "registry":
        return cmd_registry(a)
    if a.cmd == "block-serve":
        return cmd_block_serve(a)
    if a.cmd == "bench":
        from .launcher import launch
        bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
        rest = [x for x in a.rest if x != "--"]
        return launch(a.gpus, [bench, "--gpus", str(a.gpus), "--dp", str(a.dp)] + rest)
    # generate / serve: re-run this CLI as `worker` in N processes
    idx = argv.index(a.cmd)
    return _spawn_self(a, a.cmd, argv[:idx] + argv[idx + 1:])


if __name__ == "__main__":
    sys.exit(main())
