"""CPU tests of the host runtime: native block manager + shm channels, scheduler, in-process and
multi-process (gloo) pipelines, the reference-compatible session API and StreamingLLM semantics."""
import multiprocessing as mp
import os
import socket
import time

import pytest
import torch

from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig, plan_stages
from distributed_llm_inference.models import CausalLMStage, LlamaBlock, PartialLlamaSinkCache
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
from distributed_llm_inference.runtime.scheduler import Scheduler
from distributed_llm_inference.runtime.sequence import SamplingParams, Sequence, SeqStatus

SPEC = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=4,
                 num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                 max_position_embeddings=4096)


def _rt():
    from distributed_llm_inference import _runtime
    return _runtime


# ------------------------------------------------------------------------------ block manager
def test_block_manager_full_cache():
    bm = _rt().BlockManager(10, 32)
    assert bm.append(1, 40) and bm.append(2, 10)
    assert len(bm.block_table(1)) == 2 and len(bm.block_table(2)) == 1
    assert bm.num_free_blocks == 7
    assert not bm.can_append([3], [32 * 8])
    assert not bm.append(3, 32 * 8) and not bm.has_sequence(3) or bm.length(3) == 0
    t1 = bm.block_table(1)
    assert bm.slot_of(1, 33) == t1[1] * 32 + 1
    bm.free_sequence(1)
    assert bm.num_free_blocks == 9 - (1 if bm.has_sequence(3) and bm.block_table(3) else 0)


def test_block_manager_deterministic():
    ops = [(1, 70), (2, 5), (1, 1), (3, 100)]
    tabs = []
    for _ in range(2):
        bm = _rt().BlockManager(64, 32)
        for s, n in ops:
            bm.append(s, n)
        bm.free_sequence(2)
        bm.append(4, 33)
        tabs.append([bm.block_table(s) for s in (1, 3, 4)])
    assert tabs[0] == tabs[1]


def test_block_manager_window_slots():
    bm = _rt().BlockManager(64, 32, 100, 4, 16)  # window 100, 4 sinks, chunk 16
    assert bm.sink_pad == 32 and bm.ring % 32 == 0 and bm.ring >= 100 - 4 + 15
    bm.append(7, 1000)
    assert bm.slots_for(1000) == 32 + bm.ring
    assert len(bm.block_table(7)) == (32 + bm.ring + 31) // 32  # bounded, never grows past
    bt = bm.block_table(7)
    for a in (0, 3):
        assert bm.slot_of(7, a) == bt[0] * 32 + a
    a = 999
    logical = 32 + (a - 4) % bm.ring
    assert bm.slot_of(7, a) == bt[logical // 32] * 32 + logical % 32


def test_block_manager_prepare_buffers():
    bm = _rt().BlockManager(16, 32)
    bm.append(0, 5)
    bm.append(1, 40)
    slot = torch.empty(8, dtype=torch.int64)
    pos = torch.empty(8, dtype=torch.int32)
    bt = torch.full((4, 3), -7, dtype=torch.int32)
    sl = torch.empty(4, dtype=torch.int32)
    qs = torch.empty(5, dtype=torch.int32)
    T = bm.prepare([0, 1], [5, 3], slot.data_ptr(), pos.data_ptr(), bt.data_ptr(), 3,
                   sl.data_ptr(), qs.data_ptr(), 4, [])
    assert T == 8
    assert pos.tolist() == [0, 1, 2, 3, 4, 37, 38, 39]
    assert sl.tolist() == [5, 40, 0, 0] and qs.tolist() == [0, 5, 8, 8, 8]
    assert bt[2:].abs().sum() == 0
    assert slot[5] == bm.slot_of(1, 37)


# ------------------------------------------------------------------------------ shm channel
def _consumer(name, idx, nreaders, n, q):
    ch = _rt().ShmChannel(name, idx, 8, 256, nreaders, False, 10.0)
    got = [ch.recv(10.0) for _ in range(n)]
    q.put((idx, got))


def test_shm_channel_broadcast_multiprocess():
    R = _rt()
    name = f"/dli_test_{os.getpid()}"
    prod = R.ShmChannel(name, -1, 8, 256, 2, True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_consumer, args=(name, i, 2, 50, q)) for i in range(2)]
    for p in ps:
        p.start()
    msgs = [f"m{i}".encode() * (i % 5 + 1) for i in range(50)]
    # more messages than slots: exercises back-pressure.  Generous timeouts: the spawned
    # consumers import this module (and torch) before they attach, slow on a loaded machine
    for m in msgs:
        prod.send(m, 180.0)
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(10)
    assert res[0] == msgs and res[1] == msgs


def test_shm_channel_timeout_and_close():
    R = _rt()
    name = f"/dli_test2_{os.getpid()}"
    prod = R.ShmChannel(name, -1, 4, 64, 1, True)
    cons = R.ShmChannel(name, 0, 4, 64, 1, False, 5.0)
    with pytest.raises(TimeoutError):
        cons.recv(0.05)
    for i in range(4):
        prod.send(b"x", 1.0)
    with pytest.raises(TimeoutError):  # ring full, consumer not reading
        prod.send(b"y", 0.05)
    assert cons.recv(1.0) == b"x"
    prod.close()
    with pytest.raises(EOFError):
        for _ in range(10):
            cons.recv(1.0)
    assert cons.idle_seconds(-1) >= 0.0


# ------------------------------------------------------------------------------ scheduler
def test_scheduler_chunked_prefill_and_finish():
    bm = _rt().BlockManager(64, 32)
    sch = Scheduler(1, 4, 16, bm.blocks_for, 64, eos_token_id=9)
    a = Sequence(list(range(1, 30)), SamplingParams(max_tokens=3, ignore_eos=True))
    b = Sequence([5, 6], SamplingParams(max_tokens=5))
    sch.add(a)
    sch.add(b)
    p = sch.plan(0)
    assert p.q_lens == [16] and p.sample_rows == []  # a's prompt chunked, b waits for budget
    sch.on_tokens(0, [])
    p = sch.plan(0)
    assert p.q_lens == [13, 2] and p.sample_rows == [0, 1]
    sch.on_tokens(0, [100, 9])  # b hits EOS -> finished
    assert b.status == SeqStatus.FINISHED and b.finish_reason == "stop"
    p = sch.plan(0)
    assert p.free_ids == [b.seq_id] and p.q_lens == [1] and p.tokens == [100]
    sch.on_tokens(0, [101])
    p = sch.plan(0)
    sch.on_tokens(0, [102])
    assert a.output == [100, 101, 102] and a.status == SeqStatus.FINISHED


def test_scheduler_respects_kv_capacity():
    bm = _rt().BlockManager(4, 32)
    sch = Scheduler(1, 8, 1024, bm.blocks_for, 4)
    seqs = [Sequence([1] * 40, SamplingParams(max_tokens=20)) for _ in range(3)]
    for s in seqs:
        sch.add(s)
    p = sch.plan(0)
    assert len(p.seq_ids) == 2  # 60 tokens = 2 blocks each; third must wait
    with pytest.raises(ValueError):
        sch.add(Sequence([1] * 200, SamplingParams(max_tokens=1)))
    # aborting the request that waits for KV retires it at once (admission is still blocked)
    sch.abort(seqs[2].seq_id)
    assert not sch.waiting and seqs[2].finish_reason == "abort"
    assert seqs[2] in sch.pop_finished()


# ------------------------------------------------------------------------------ engines
def _cfg(pp=1, mbs=0, window=0, sinks=0):
    return EngineConfig(model="t", pp=pp, seed=3,
                        cache=CacheConfig(num_blocks=256, block_size=32, window_length=window,
                                          num_sink_tokens=sinks, max_chunk=64),
                        serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=64,
                                          num_micro_batches=mbs, max_seq_len=512, use_graphs=False))


PROMPTS = [list(range(3, 40)), [7, 8, 9], list(range(100, 190)), [11]]


@pytest.mark.parametrize("pp,mbs", [(2, 0), (3, 1), (4, 6)])
def test_local_pipeline_equals_single_stage(pp, mbs):
    p = SamplingParams(max_tokens=6, ignore_eos=True)
    a = [s.output for s in LLMEngine(SPEC, cfg=_cfg()).generate(PROMPTS, p)]
    b = [s.output for s in LLMEngine(SPEC, cfg=_cfg(pp, mbs)).generate(PROMPTS, p)]
    assert a == b


def test_lookahead_matches_plain_decode():
    """One-step lookahead (single micro-batch: step t+1 issued before step t's tokens reach the
    host, its input tokens taken from the device sampler output) changes nothing observable:
    same tokens, same finish reasons, including sequences that stop on EOS inside the lookahead
    window and sequences with different max_tokens."""
    from distributed_llm_inference.runtime.sequence import Sequence
    ref_eng = LLMEngine(SPEC, cfg=_cfg(mbs=1))
    ref_eng.pipeline.lookahead = False
    p0 = SamplingParams(max_tokens=12, ignore_eos=True)
    base = [s.output for s in ref_eng.generate(PROMPTS, p0)]
    # an EOS id that some sequences emit mid-generation
    eos = base[0][4]

    def run(lookahead):
        eng = LLMEngine(SPEC, cfg=_cfg(mbs=1))
        eng.pipeline.lookahead = lookahead
        eng.pipeline.sched.eos = eos
        seqs = [Sequence(list(pr), SamplingParams(max_tokens=mt, temperature=t, seed=7))
                for pr, mt, t in zip(PROMPTS, (12, 3, 9, 12), (0.0, 0.0, 0.9, 0.0))]
        for s_ in seqs:
            eng.pipeline.sched.add(s_)
        eng.pipeline.run_until_done()
        return [(s_.output, s_.finish_reason) for s_ in seqs], eng

    off, _ = run(False)
    on, eng = run(True)
    assert on == off
    assert any(r == "stop" for _, r in on) and any(r == "length" for _, r in on)
    assert eng.pipeline.lookahead


def test_sampling_reproducible_and_max_tokens():
    p = SamplingParams(max_tokens=7, temperature=1.0, top_k=20, ignore_eos=True, seed=4)
    g = torch.Generator().manual_seed(0)
    e = LLMEngine(SPEC, cfg=_cfg())
    out = e.generate(PROMPTS, p)
    assert all(len(s.output) == 7 and s.finish_reason == "length" for s in out)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _mp_worker(rank, world, port, q, params=None, rotation="1"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLI_HEAD_ROTATION=rotation)
    import torch.distributed as dist
    from distributed_llm_inference.runtime.engine import init_pipeline_rank
    cfg = _cfg(pp=world)
    cfg.model = SPEC  # type: ignore[assignment]
    role, obj = init_pipeline_rank(cfg)
    if role == "driver":
        out = obj.generate(PROMPTS, params or SamplingParams(max_tokens=6, ignore_eos=True))
        obj.stop()
        obj.close()
        q.put([s.output for s in out])
    else:
        obj.run()
        obj.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rotation", [(3, "0"), (4, "1")])
def test_multiprocess_rotating_head_sampling(world, rotation):
    """Seeded top-k / temperature sampling through the multi-process pipeline with the LM head
    rotating over the ranks (and, for contrast, pinned to the last rank): identical tokens to the
    single-stage engine (the sampler's RNG is keyed by seed and step, not by rank)."""
    p = SamplingParams(max_tokens=7, temperature=0.9, top_k=40, top_p=0.95, seed=3,
                       ignore_eos=True)
    ref = [s.output for s in LLMEngine(SPEC, cfg=_cfg()).generate(PROMPTS, p)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_mp_worker, args=(r, world, port, q, p, rotation))
          for r in range(world)]
    for pr in ps:
        pr.start()
    got = q.get(timeout=240)
    for pr in ps:
        pr.join(60)
        assert pr.exitcode == 0
    assert got == ref


@pytest.mark.parametrize("world", [2, 3, 4])
def test_multiprocess_pipeline_gloo(world):
    ref = [s.output for s in LLMEngine(SPEC, cfg=_cfg()).generate(
        PROMPTS, SamplingParams(max_tokens=6, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_mp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=240)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert got == ref


# ------------------------------------------------------------------------------ reference API
def test_llama_block_session_api_incremental_equals_full():
    blk = LlamaBlock(SPEC, [0, 1, 2]).init_random(1)
    x = torch.randn(2, 12, 128, dtype=torch.bfloat16)
    (full,) = blk("g-full", x)  # stateless, causal within the chunk
    cache = PartialLlamaSinkCache(0, 0, num_blocks=32, block_size=32)
    (a,) = blk("g1", x[:, :8], past_key_value=cache)
    (b,) = blk("g1", x[:, 8:10], past_key_value=cache)
    (c,) = blk("g1", x[:, 10:], past_key_value=cache)
    inc = torch.cat([a, b, c], 1)
    assert torch.allclose(inc.float(), full.float(), atol=3e-2, rtol=3e-2)
    assert cache.get_seq_length(0, "g1") == 12
    with pytest.raises(ValueError):
        cache.get_seq_length(0)
    out = blk("g2", x[:, :4], past_key_value=cache, output_hidden_states=True)
    assert len(out) == 2 and len(out[1]) == 4  # input + one per layer
    cache.close_session("g1")
    assert cache.get_seq_length(0, "g1") == 0


def test_llama_block_padding_mask():
    blk = LlamaBlock(SPEC, [0, 1]).init_random(2)
    x = torch.randn(1, 6, 128, dtype=torch.bfloat16)
    xp = torch.cat([torch.zeros(1, 3, 128, dtype=torch.bfloat16), x], 1)  # left padding
    mask = torch.tensor([[0, 0, 0, 1, 1, 1, 1, 1, 1]])
    (ref,) = blk("a", x)
    (out,) = blk("b", xp, attention_mask=mask)
    assert torch.allclose(out[:, 3:].float(), ref.float(), atol=2e-2, rtol=2e-2)
    assert out[:, :3].abs().sum() == 0


def test_cache_update_protocol():
    cache = PartialLlamaSinkCache(0, 0, num_blocks=16, block_size=32).bind(SPEC, [0, 1])
    k = torch.randn(2, 2, 5, 32, dtype=torch.bfloat16)
    v = torch.randn(2, 2, 5, 32, dtype=torch.bfloat16)
    K, V = cache.update(k, v, 0, {"generation_id": "s"})
    assert K.shape == (2, 2, 5, 32) and torch.equal(K, k) and torch.equal(V, v)
    K1, _ = cache.update(k, v, 1, {"generation_id": "s"})
    assert torch.equal(K1, k)
    k2 = torch.randn(2, 2, 1, 32, dtype=torch.bfloat16)
    K, _ = cache.update(k2, k2, 0, {"generation_id": "s"})
    assert K.shape[2] == 6 and torch.equal(K[:, :, 5:], k2)


# ------------------------------------------------------------------------------ StreamingLLM
def test_sink_window_matches_streamingllm_definition():
    """1-layer model (cached K/V depend only on token + position): decoding a long sequence
    through the sink/window cache must equal a fresh full-cache forward of the StreamingLLM view
    [sink tokens] + [last W - n_sink tokens] at contiguous positions 0..W-1."""
    spec = SPEC.replace(num_layers=1)
    stage = CausalLMStage(spec, 0, 1).init_random(11)
    W, S = 48, 4
    toks = torch.randint(0, spec.vocab_size, (130,)).tolist()
    pool = stage.make_pool(64, 32, window_length=W, num_sink_tokens=S, max_chunk=8)
    pool.manager.append(0, 8)
    meta = pool.build_metadata([0], [8])
    meta.logits_rows = torch.tensor([7])
    stage(torch.tensor(toks[:8], dtype=torch.int32), meta, pool)
    for t in range(8, len(toks)):
        pool.manager.append(0, 1)
        meta = pool.build_metadata([0], [1])
        logits = stage(torch.tensor([toks[t]], dtype=torch.int32), meta, pool)
    view = toks[:S] + toks[len(toks) - (W - S):]
    ref_pool = stage.make_pool(64, 32)
    ref_pool.manager.append(0, len(view))
    m = ref_pool.build_metadata([0], [len(view)])
    m.logits_rows = torch.tensor([len(view) - 1])
    ref = stage(torch.tensor(view, dtype=torch.int32), m, ref_pool)
    assert torch.allclose(logits.float(), ref.float(), atol=3e-2, rtol=3e-2)


def test_plan_stages_balanced():
    from distributed_llm_inference.config import PRESETS
    r = plan_stages(PRESETS["llama-3-70b"], 8)
    assert r[0][0] == 0 and r[-1][1] == 80 and all(b > a for a, b in r)
    assert all(r[i][1] == r[i + 1][0] for i in range(7))
    assert r[-1][1] - r[-1][0] <= r[0][1] - r[0][0]  # last stage also runs the LM head


def test_plan_stages_minimises_slowest_stage():
    """The planner's slowest stage (layers + LM-head equivalent on the last stage, divided by the
    stage's speed) equals the brute-force optimum over all contiguous splits."""
    import itertools
    import math
    from distributed_llm_inference.config import PRESETS
    assert [b - a for a, b in plan_stages(PRESETS["llama-3-70b"], 8)] == [10] * 8
    for name in ("llama-3-8b", "llama-3-70b", "tiny-llama"):
        spec = PRESETS[name]
        head = 0.6 * spec.vocab_size * spec.hidden_size / spec.layer_param_count()
        L = spec.num_layers
        for n in (2, 3, 4):
            if n > L:
                continue
            for w in ([1.0] * n, [1.0] * (n - 1) + [0.5], [0.5] + [1.0] * (n - 1)):
                def cost(counts):
                    return max((c + (head if i == n - 1 else 0.0)) / w[i]
                               for i, c in enumerate(counts))
                got = cost([b - a for a, b in plan_stages(spec, n, weights=w)])
                best = math.inf
                for cuts in itertools.combinations(range(1, L), n - 1):
                    edges = (0,) + cuts + (L,)
                    best = min(best, cost([edges[i + 1] - edges[i] for i in range(n)]))
                assert got <= best + 1e-9, (name, n, w, got, best)


def test_fp8_kv_cache_close_to_bf16_cpu():
    """fp8 (e4m3) KV cache through the CPU reference path: same greedy tokens in the first steps
    and logits close to the bf16 cache."""
    from distributed_llm_inference.models import CausalLMStage
    st = CausalLMStage(SPEC, 0, 4).init_random(5)
    prompts = [[1, 2, 3, 4, 5, 6, 7, 8], [9, 8, 7]]

    def logits(kv_dtype):
        pool = st.make_pool(64, 32, kv_dtype=kv_dtype)
        sids = [0, 1]
        for s_, p_ in zip(sids, prompts):
            pool.manager.append(s_, len(p_))
        meta = pool.build_metadata(sids, [len(p_) for p_ in prompts],
                                   logits_rows=torch.tensor([7, 10]))
        ids = torch.tensor([t for p_ in prompts for t in p_])
        out = [st(ids, meta, pool).float()]
        for tok in ([3, 4], [5, 6]):
            for s_ in sids:
                pool.manager.append(s_, 1)
            out.append(st(torch.tensor(tok), pool.build_metadata(sids, [1, 1]), pool).float())
        return out

    a, b = logits(torch.bfloat16), logits(torch.float8_e4m3fn)
    for x, y in zip(a, b):
        assert ((x - y).norm() / x.norm()).item() < 0.08


def test_swiglu_interleave_roundtrip_and_tile_splits():
    import torch
    from distributed_llm_inference import ops
    w = torch.randn(1024, 8)
    wi = ops.swiglu_interleave(w)
    assert torch.equal(ops.swiglu_deinterleave(wi), w)
    # interleaved GEMM output -> silu(gate) * up in natural column order
    x = torch.randn(5, 8)
    ref = ops.silu_mul((x @ w.t()).bfloat16()).float()
    got = ops.swiglu_interleaved((x @ wi.t()).bfloat16()).float()
    assert (ref - got).abs().max() < 2e-2 * ref.abs().max()
    # split-K choice fills whole waves of 256 CUs (70B decode shapes at M = 512)
    assert ops.tile_gemm_splits(512, 10240, 8192) == 3
    assert ops.tile_gemm_splits(512, 8192, 8192) == 4
    assert ops.tile_gemm_splits(512, 8192, 28672) == 4
    assert ops.tile_gemm_splits(512, 57344, 8192) == 1
    assert ops.tile_gemm_splits(64, 8192, 8192) == 0      # too few rows
    assert ops.tile_gemm_splits(512, 100, 8192) == 0      # N not a multiple of 256
    assert ops.tile_gemm_splits(512, 128256, 8192) == 0   # LM head stays on hipBLASLt


@pytest.mark.parametrize("head", [False, True])
def test_rccl_connect_plan_resolves_without_a_cycle(head):
    """RcclTransport brings every P2P link up at init with blocking, matched send/recv pairs
    (parallel/transport.py connect_plan).  Simulate all ranks for every world size up to 16: each
    op completes only when the peer's current op is its match; every rank must finish, and every
    link the runtime uses (stage i -> i+1, head last -> r) must be connected exactly once."""
    from distributed_llm_inference.parallel.transport import connect_plan
    for world in range(1, 17):
        plans = [connect_plan(r, world, head) for r in range(world)]
        pos = [0] * world
        links = []
        progress = True
        while progress:
            progress = False
            for r in range(world):
                if pos[r] >= len(plans[r]):
                    continue
                op, kind, peer = plans[r][pos[r]]
                if pos[peer] >= len(plans[peer]):
                    continue
                pop, pkind, ppeer = plans[peer][pos[peer]]
                if ppeer == r and pkind == kind and {op, pop} == {"send", "recv"}:
                    src, dst = (r, peer) if op == "send" else (peer, r)
                    links.append((kind, src, dst))
                    pos[r] += 1
                    pos[peer] += 1
                    progress = True
        assert all(pos[r] == len(plans[r]) for r in range(world)), (world, head, pos)
        want = [("stage", i, i + 1) for i in range(world - 1)]
        if head and world > 1:
            want += [("head", world - 1, r) for r in range(world - 1)]
        assert sorted(links) == sorted(want), (world, head)
