"""Engine construction: stages -> executors -> pipeline driver.

* :func:`build_executor` — one stage on one device: weights (random-init or checkpoint, optional
  fp8), KV pool sized from free HBM (288 GB per MI355X), executor with graph buckets.  In a
  multi-process pipeline every rank agrees on the MIN block count (all-reduce over the gloo
  control group) so the driver's admission control is valid on every stage.
* :class:`LLMEngine` — in-process engine (PP=1, or PP>1 stages in one process).
* :func:`init_pipeline_rank` — per-rank bootstrap of the multi-process pipeline launched by
  ``distribute`` / torchrun: rank 0 gets a :class:`DistributedDriver`, other ranks a
  :class:`StageFollower` whose ``run()`` serves until the driver stops it.
"""
from __future__ import annotations

import logging
import os
import uuid
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..config import CacheConfig, KernelPolicy, ModelSpec, ServeConfig, plan_stages, resolve_model
from ..models.llama.cache import KVPool
from ..parallel.pipeline import (DistributedDriver, LocalPipeline, StageFollower, _Channels,
                                 make_transport)
from ..utils.model import build_stage
from .executor import StageExecutor
from .head import HeadJobs, HeadPolicy, HeadRunner
from .scheduler import Scheduler
from .sequence import SamplingParams, Sequence as Seq

log = logging.getLogger(__name__)


@dataclass
class EngineConfig:
    model: str = "llama-3-8b"
    checkpoint: Optional[str] = None
    random_init: bool = True
    seed: int = 0
    dtype: str = "bf16"
    quantize: object = False        # False | True / "fp8" (e4m3 weights) | "int8" (LLM.int8)
    int8_threshold: float = 6.0     # LLM.int8 outlier threshold (quantize="int8")
    pp: int = 1
    dp: int = 1                     # pipeline replicas (world = dp x pp in init_pipeline_rank)
    cache: CacheConfig = field(default_factory=CacheConfig)
    serve: ServeConfig = field(default_factory=ServeConfig)
    # hot-path kernel choices; None keeps the process's current policy (ops.policy())
    kernels: Optional[KernelPolicy] = None


def _activation_reserve(spec: ModelSpec, serve: ServeConfig) -> int:
    T = serve.max_num_batched_tokens
    per_tok = 2 * (spec.qkv_size + 3 * spec.intermediate_size + 4 * spec.hidden_size)
    logits = serve.max_batch_size * spec.vocab_size * 4
    return int(T * per_tok * 2 + logits + (2 << 30))


def build_executor(spec: ModelSpec, start: int, end: int, device: torch.device, cfg: EngineConfig,
                   group=None, num_blocks: Optional[int] = None,
                   kv_share: float = 1.0) -> StageExecutor:
    if cfg.kernels is not None:   # before any weight conversion reads it (int8_transposed)
        ops.set_policy(cfg.kernels)
    stage = build_stage(cfg.checkpoint or spec, start, end, device=device,
                        random_init=cfg.random_init and cfg.checkpoint is None, seed=cfg.seed,
                        quantize=cfg.quantize, checkpoint=cfg.checkpoint,
                        int8_threshold=cfg.int8_threshold)
    cc, sc = cfg.cache, cfg.serve
    nlayers = end - start
    if device.type == "cuda" and hasattr(stage.block, "set_fused_swiglu"):
        # gate|up weights in the tile GEMM's SwiGLU order (bf16, or fp8 on the fp8 tile path)
        stage.block.set_fused_swiglu(True)
    if device.type == "cuda" and sc.use_graphs:
        from .gemm_tuning import tune_decode_gemms
        buckets = [b for b in sc.graph_batch_sizes if 16 <= b <= sc.max_batch_size]
        tdir = os.environ.get("DLI_TUNING_DIR", os.path.join(os.path.dirname(os.path.dirname(
            os.path.dirname(os.path.abspath(__file__)))), "build", "tuning"))
        tune_decode_gemms(stage, buckets, os.path.join(tdir, "tunableop_results.csv"))
    if num_blocks is None:
        num_blocks = cc.num_blocks
    if num_blocks is None:
        if device.type == "cuda":
            # memory freed by load-time conversions (fp8 quantisation drops the bf16 weights) is
            # still held by this process's caching allocator and would not count as free
            torch.cuda.synchronize(device)
            torch.cuda.empty_cache()
            if group is not None:
                # ranks sharing a device (DLI_SHARE_GPU) must all hold their weights, and have
                # released their caches, before any of them measures what is left for KV
                dist.barrier(group=group)
            free, _ = torch.cuda.mem_get_info(device)
            num_blocks = KVPool.size_from_memory(spec, nlayers, cc.block_size, int(free * kv_share),
                                                 cc.gpu_memory_utilization,
                                                 _activation_reserve(spec, sc), cc.dtype_bytes)
        else:
            num_blocks = 1024
        if num_blocks < 2:
            raise RuntimeError(f"stage [{start},{end}) on {device}: no HBM left for the KV cache "
                               "(lower max_num_batched_tokens or use fp8 weights)")
    if group is not None:
        t = torch.tensor([num_blocks], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        num_blocks = int(t.item())
    if spec.rope_type == "dynamic" and sc.max_seq_len > spec.max_position_embeddings:
        # HF's dynamic NTK base depends on each forward's longest position, but the engine's
        # captured decode steps read ONE RoPE table: serve such lengths through the reference
        # API (LlamaBlock.forward rebuilds the table per call), or cap max_seq_len
        raise ValueError(f"rope_type 'dynamic' past max_position_embeddings "
                         f"({spec.max_position_embeddings}) is supported by LlamaBlock.forward "
                         f"only; the engine needs max_seq_len <= it (got {sc.max_seq_len})")
    win, sinks = cc.window_length, cc.num_sink_tokens
    if not win and spec.sliding_window and sc.max_seq_len > spec.sliding_window:
        # Mistral-style sliding-window attention IS the ring window with no sink tokens (each
        # query sees itself and the W-1 keys before it, at their true relative positions;
        # tests/test_model_parity_cpu.py::test_mistral_sliding_window_matches_hf_beyond_window)
        win, sinks = spec.sliding_window, 0
    pool = stage.make_pool(num_blocks, cc.block_size, win, sinks,
                           cc.max_chunk, cc.torch_dtype, cc.k_scale, cc.v_scale)
    log.info("stage [%d,%d) on %s: %d KV blocks x %d tokens", start, end, device, num_blocks,
             cc.block_size)
    return StageExecutor(stage, pool, max_num_seqs=sc.max_batch_size,
                         max_num_batched_tokens=sc.max_num_batched_tokens,
                         max_seq_len=sc.max_seq_len, use_graphs=sc.use_graphs,
                         graph_batch_sizes=sc.graph_batch_sizes)


def make_scheduler(spec: ModelSpec, ex: StageExecutor, cfg: EngineConfig, num_stages: int) -> Scheduler:
    sc = cfg.serve
    M = sc.num_micro_batches or (num_stages + 1 if num_stages > 1 else 1)
    m = ex.pool.manager
    return Scheduler(M, sc.max_batch_size, sc.max_num_batched_tokens, m.blocks_for, m.num_blocks,
                     eos_token_id=spec.eos_token_id, max_seq_len=sc.max_seq_len)


class LLMEngine:
    """In-process engine: ``LLMEngine("llama-3-8b").generate([[1, 2, 3]], SamplingParams(...))``."""

    def __init__(self, model="llama-3-8b", pp: int = 1, device=None, cfg: Optional[EngineConfig] = None,
                 **kw):
        cfg = cfg or EngineConfig(model=model if isinstance(model, str) else "custom", pp=pp, **kw)
        self.cfg = cfg
        spec = resolve_model(cfg.checkpoint or model)
        self.spec = spec
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        device = torch.device(device)
        ranges = plan_stages(spec, cfg.pp)
        self.executors: List[StageExecutor] = []
        total_layers = spec.num_layers
        for (s, e) in ranges:
            share = (e - s) / total_layers
            # later stages see less free memory: give each its layer share of what remains
            remaining_layers = sum(b - a for a, b in ranges[len(self.executors):])
            self.executors.append(build_executor(spec, s, e, device, cfg,
                                                 kv_share=(e - s) / remaining_layers))
        nb = min(ex.pool.num_blocks for ex in self.executors)
        self.scheduler = make_scheduler(spec, self.executors[0], cfg, len(ranges))
        self.scheduler.total_blocks = nb
        self.pipeline = LocalPipeline(self.executors, self.scheduler)

    def generate(self, prompts: Sequence[Sequence[int]],
                 params: Optional[SamplingParams] = None) -> List[Seq]:
        return self.pipeline.generate(prompts, params)


# =============================================================================================
@dataclass(frozen=True)
class ReplicaLayout:
    """DP x PP placement of one node's ranks: ``dp`` independent pipeline replicas of ``pp``
    stages each; replica r owns the consecutive ranks [r*pp, (r+1)*pp) (consecutive GPUs, so every
    stage hop stays on a direct xGMI link).  The reference's swarm hosts the same blocks on several
    servers (reference server/server.py:7-8,20; server/worker.py:9-20); on one MI355X node that is a
    replica of the whole layer range per pipeline."""
    dp: int
    pp: int

    @staticmethod
    def for_world(world: int, dp: int = 1) -> "ReplicaLayout":
        dp = max(1, int(dp))
        if world % dp:
            raise ValueError(f"world size {world} is not a multiple of dp={dp}")
        return ReplicaLayout(dp, world // dp)

    def replica(self, rank: int) -> int:
        return rank // self.pp

    def stage(self, rank: int) -> int:
        return rank % self.pp

    def ranks(self, replica: int) -> List[int]:
        return list(range(replica * self.pp, (replica + 1) * self.pp))

    def drivers(self) -> List[int]:
        return [r * self.pp for r in range(self.dp)]

    def describe(self, spec: ModelSpec, head_rotation: bool = True) -> dict:
        ranges = plan_stages(spec, self.pp, head_rotation=head_rotation)
        return {"dp": self.dp, "pp": self.pp,
                "replicas": [{"replica": r, "driver_rank": r * self.pp,
                              "stages": [{"rank": r * self.pp + i, "gpu": r * self.pp + i,
                                          "layers": list(rg)} for i, rg in enumerate(ranges)]}
                             for r in range(self.dp)]}


def _progress(msg: str) -> None:
    """``DLI_PROGRESS=1``: rank init phases on stderr (bench.py sets it; a multi-rank init of a
    70B stage takes minutes and must never look hung)."""
    if os.environ.get("DLI_PROGRESS") == "1":
        import sys
        import time
        print(f"[dli rank {os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}",
              file=sys.stderr, flush=True)


def _dp_from_env(cfg: EngineConfig) -> int:
    return int(os.environ.get("DLI_DP", cfg.dp or 1))


def rccl_rank_hosts(rank: int, env=os.environ) -> bool:
    """``DLI_RCCL_RANK_HOSTS=1`` (one-GPU RCCL rehearsals, with ``DLI_SHARE_GPU=1``): the rank
    claims an RCCL host of its own (``NCCL_HOSTID``), so RCCL's duplicate-device check, which
    compares (host, PCI bus id), passes for ranks sharing a GPU, and strict RCCL
    (``DLI_TRANSPORT=rccl``) connects them through its socket transport on loopback.  RCCL reads
    the host id once, so this must run before any RCCL call.  Returns whether it applied."""
    if env.get("DLI_RCCL_RANK_HOSTS") != "1":
        return False
    env["NCCL_HOSTID"] = f"dli-rehearsal-host-{rank}"
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")
    env.setdefault("NCCL_IB_DISABLE", "1")
    return True


def init_pipeline_rank(cfg: EngineConfig, backend: str = "gloo"):
    """Bootstrap this rank of a multi-process pipeline (env: RANK, WORLD_SIZE, LOCAL_RANK,
    MASTER_ADDR, MASTER_PORT; ``DLI_DP`` or ``cfg.dp`` = number of pipeline replicas).  Returns
    ``("driver", DistributedDriver | LocalPipeline)`` on the first rank of every replica and
    ``("follower", StageFollower)`` elsewhere.  Every returned object carries ``replica``,
    ``layout`` and ``drivers_group`` (a gloo group over the replica drivers, None for dp == 1)."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    spec = resolve_model(cfg.checkpoint or cfg.model)
    layout = ReplicaLayout.for_world(world, _dp_from_env(cfg))
    rep, srank, pp = layout.replica(rank), layout.stage(rank), layout.pp
    kv_share = 1.0
    if torch.cuda.is_available():
        # DLI_SHARE_GPU=1: several stage processes on the visible GPUs round-robin (tests on a
        # single-GPU box); otherwise one GPU per local rank
        if os.environ.get("DLI_SHARE_GPU") == "1":
            ndev = torch.cuda.device_count()
            kv_share = 1.0 / ((world + ndev - 1) // ndev)
            local = local % ndev
            rccl_rank_hosts(rank)
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")

    head_rotation = False

    def tag(obj):
        obj.replica, obj.layout, obj.drivers_group = rep, layout, drivers_group
        obj.head_rotation = head_rotation
        return obj

    drivers_group = None
    if world == 1:
        eng = LLMEngine(cfg.model, pp=1, device=device, cfg=cfg)
        return "driver", tag(eng.pipeline)
    if not dist.is_initialized():
        dist.init_process_group(backend)
    # every rank creates every group, in the same order (torch.distributed requirement)
    rep_groups = [dist.new_group(layout.ranks(r)) for r in range(layout.dp)] if layout.dp > 1 \
        else [dist.group.WORLD]
    if layout.dp > 1:
        drivers_group = dist.new_group(layout.drivers())
    group = rep_groups[rep]
    store = dist.distributed_c10d._get_default_store()
    if rank == 0:
        store.set("dli_job", uuid.uuid4().hex[:12])
    job = store.get("dli_job").decode()
    base_job = job
    if layout.dp > 1:
        job = f"{job}r{rep}"
    if pp == 1:
        # a single-stage replica: its own in-process pipeline on this GPU
        eng = LLMEngine(cfg.model, pp=1, device=device, cfg=cfg)
        dist.barrier()
        return "driver", tag(eng.pipeline)
    streams = None
    if device.type == "cuda":
        # every stream this rank will use, each on a hardware queue of its own, made current
        # before anything is allocated or launched (runtime/streams.py)
        from .streams import rank_streams, token_ring
        streams = rank_streams(device)
        streams.activate()
        # host-mapped allocations now, never in the step loop: allocating pinned / mapped host
        # memory may synchronise the device, i.e. wait for a stream parked in a peer wait
        # every decode step of every in-flight micro-batch (plus the rotating head's) may hold a
        # slot until its consumer reads it: size the ring from that, with headroom
        M = max(1, cfg.serve.num_micro_batches or pp)
        token_ring(device, max(4096, cfg.serve.max_batch_size), slots=max(64, 8 * (M + pp)))
    rotate = head_rotation_wanted(cfg, pp, device)
    ranges = plan_stages(spec, pp, head_rotation=rotate)
    if os.environ.get("DLI_STAGE_RANGES"):  # placement chosen by the server (rebalance)
        import json
        ranges = [tuple(r) for r in json.loads(os.environ["DLI_STAGE_RANGES"])]
        if len(ranges) != pp:
            raise ValueError("DLI_STAGE_RANGES must have one range per pipeline stage")
    start, end = ranges[srank]
    head = None
    if rotate and srank != pp - 1:
        # built before the KV pool is sized from the free HBM that is left
        from ..utils.model import build_head
        head = build_head(cfg.checkpoint or spec, device=device,
                          random_init=cfg.random_init and cfg.checkpoint is None, seed=cfg.seed,
                          checkpoint=cfg.checkpoint)
    _progress(f"building stage [{start},{end}) of {spec.name} on {device}")
    ex = build_executor(spec, start, end, device, cfg, group=group, kv_share=kv_share)
    _progress(f"stage built: {ex.pool.num_blocks} KV blocks; connecting the transport")
    if streams is not None:
        ex.capture_stream = streams.capture
    H = spec.hidden_size
    transport = make_transport(srank, pp, device, job=job, rank_offset=rep * pp, head_pairs=rotate,
                               streams=streams, max_bytes=ex.max_tokens * H * 2,
                               head_bytes=ex.max_num_seqs * H * 2)
    # a stalled wait or a failed rank ends the whole job with every rank's last op (watchdog.py)
    from .watchdog import TRACKER, start_watchdog
    start_watchdog(base_job, world, on_abort=getattr(transport, "abort", None))
    TRACKER.add_state("transport", transport.counters)
    if device.type == "cuda" and world > 1:
        TRACKER.enable_device_marks(device)
    # the fallback transport (agreed on by every rank) cannot carry the head: then nobody rotates
    rotate = rotate and transport.supports_head
    head_rotation = rotate   # recorded on the returned driver / follower (bench per-rank records)
    channels = _Channels(job, srank, pp, head_rotation=rotate)
    policy = HeadPolicy(pp, rotate, ex.max_num_seqs)
    dist.barrier()
    channels.unlink()  # every rank has attached: nothing may be left in /dev/shm after this
    heads_runner = None
    if rotate and head is not None:
        heads_runner = HeadRunner(head, device, ex.max_num_seqs, cfg.serve.use_graphs,
                                  ex.graph_sizes,
                                  capture_stream=streams.capture if streams is not None else None)
    if device.type == "cuda" and cfg.serve.use_graphs:
        # capture every decode graph NOW, before any transport traffic: no capture ever runs
        # next to in-flight receive kernels or the token publisher thread
        variants = (True, False) if (rotate and srank == pp - 1) else (True,)
        _progress(f"transport up ({type(transport).__name__}); capturing decode graphs")
        ex.warmup_graphs(variants=variants)
        if heads_runner is not None:
            heads_runner.warmup()
        dist.barrier(group=group)
        _progress("graphs captured")
    if srank == 0:
        sched = make_scheduler(spec, ex, cfg, pp)
        drv = DistributedDriver(ex, sched, transport, channels, pp, group, policy=policy)
        if heads_runner is not None:
            drv.heads = HeadJobs(heads_runner, transport, pp - 1, drv.publish_local, delay=pp,
                                 stream=streams.head if streams is not None else None)
            TRACKER.add_state("head_jobs", drv.heads.state)
        drv.streams = streams
        TRACKER.add_state("driver", lambda: {"inflight": [(p.step, p.mb) for p in drv.inflight]})
        return "driver", tag(drv)
    fol = StageFollower(ex, transport, channels, srank, pp, group, policy=policy)
    if heads_runner is not None:
        fol.heads = HeadJobs(heads_runner, transport, pp - 1, fol.publish, delay=pp - srank,
                             stream=streams.head if streams is not None else None)
        TRACKER.add_state("head_jobs", fol.heads.state)
        fol._start_publisher()
    fol.streams = streams
    return "follower", tag(fol)


def head_rotation_wanted(cfg: EngineConfig, pp: int, device: torch.device) -> bool:
    """Rotate the decode LM head over the pipeline ranks (runtime/head.py)?  On by default for
    PP > 1 over RCCL or IPC (GPUs) or gloo (CPU); the host-staged transport keeps it on the last
    stage.  ``DLI_HEAD_ROTATION=0/1`` overrides the config."""
    env = os.environ.get("DLI_HEAD_ROTATION")
    want = cfg.serve.head_rotation if env is None else env == "1"
    if not want or pp < 2:
        return False
    from ..parallel.transport import HEAD_ROTATING_KINDS, transport_kind
    return transport_kind(device) in HEAD_ROTATING_KINDS
