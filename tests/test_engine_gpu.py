"""End-to-end runtime on one MI355X: stage numerics vs the CPU reference path, hipGraph decode vs
eager, in-process PP=2/4 vs PP=1, attention-sink window mode, fp8 weights."""
import pytest
import torch

from distributed_llm_inference import ops
from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig
from distributed_llm_inference.models import CausalLMStage
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
from distributed_llm_inference.runtime.sequence import SamplingParams

pytestmark = pytest.mark.gpu

SPEC = ModelSpec(name="t", vocab_size=1000, hidden_size=256, intermediate_size=512, num_layers=4,
                 num_heads=8, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                 max_position_embeddings=4096)


def _stage_logits(stage, prompts, steps):
    pool = stage.make_pool(128, block_size=64)
    sids = list(range(len(prompts)))
    for s, p in zip(sids, prompts):
        pool.manager.append(s, len(p))
    meta = pool.build_metadata(sids, [len(p) for p in prompts])
    meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(stage.device)
    ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=stage.device)
    outs = [stage(ids, meta, pool).float().cpu()]
    for _ in range(steps):
        toks = outs[-1].argmax(-1)
        for s in sids:
            pool.manager.append(s, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        outs.append(stage(toks.to(torch.int32).to(stage.device), meta, pool).float().cpu())
    return outs


def test_stage_gpu_matches_cpu(gpu):
    prompts = [list(range(1, 70)), [5, 6, 7], list(range(100, 300))]
    cpu = CausalLMStage(SPEC, 0, 4).init_random(3)
    g = CausalLMStage(SPEC, 0, 4, device=gpu).init_random(3)
    # same weights on both sides (init is device-dependent RNG): copy CPU -> GPU
    g.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})
    a = _stage_logits(cpu, prompts, 0)  # prefill only: decode tokens could diverge on near-ties
    b = _stage_logits(g, prompts, 0)
    for x, y in zip(a, b):
        err = (x - y).abs().max().item()
        assert err < 0.03 * max(1.0, x.abs().max().item()), err


SPEC128 = ModelSpec(name="t128", vocab_size=1000, hidden_size=512, intermediate_size=768,
                    num_layers=3, num_heads=8, num_kv_heads=1, head_dim=128, rope_theta=10000.0,
                    max_position_embeddings=4096)


@pytest.mark.parametrize("window,sinks", [(0, 0), (128, 0), (128, 4)])
def test_stage_head128_prefill32_matches_cpu(gpu, window, sinks):
    """head_dim 128 runs prefill on attn_prefill32.hip (the 32-dim SPEC above never reaches it):
    prefill of prompts up to 300 tokens and forced decode steps on the GPU stage against the CPU
    reference stage - full cache, Mistral-style sliding window, StreamingLLM sinks - the windowed
    ones past the window (ring wrapped)."""
    prompts = [list(range(1, 301)), list(range(500, 537)), [5, 6, 7, 8, 9], list(range(40, 170))]
    forced = [[17, 23, 5, 9], [5, 900, 1, 2], [44, 1, 3, 7]]
    cpu = CausalLMStage(SPEC128, 0, 3).init_random(3)
    g = CausalLMStage(SPEC128, 0, 3, device=gpu).init_random(3)
    g.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})

    def run(stage):
        pool = stage.make_pool(64, 64, window_length=window, num_sink_tokens=sinks, max_chunk=512)
        sids = list(range(len(prompts)))
        for s_, p_ in zip(sids, prompts):
            pool.manager.append(s_, len(p_))
        meta = pool.build_metadata(sids, [len(p_) for p_ in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p_) for p_ in prompts]), 0) - 1).to(
            stage.device)
        ids = torch.tensor([t for p_ in prompts for t in p_], dtype=torch.int32, device=stage.device)
        outs = [stage(ids, meta, pool).float().cpu()]
        for step in forced:
            for s_ in sids:
                pool.manager.append(s_, 1)
            meta = pool.build_metadata(sids, [1] * len(sids))
            outs.append(stage(torch.tensor(step, dtype=torch.int32, device=stage.device), meta,
                              pool).float().cpu())
        return outs

    for x, y in zip(run(cpu), run(g)):
        err = (x - y).abs().max().item()
        assert err < 0.03 * max(1.0, x.abs().max().item()), err


def _engine(pp=1, graphs=True, window=0, sinks=0, quantize=False, mbs=0):
    cfg = EngineConfig(model="t", pp=pp, seed=5, quantize=quantize,
                       cache=CacheConfig(num_blocks=256, block_size=64, window_length=window,
                                         num_sink_tokens=sinks, max_chunk=256),
                       serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=512,
                                         max_seq_len=1024, use_graphs=graphs, num_micro_batches=mbs,
                                         graph_batch_sizes=[1, 2, 4, 8]))
    return LLMEngine(SPEC, device="cuda:0", cfg=cfg)


PROMPTS = [list(range(3, 40)), [7, 8, 9], list(range(200, 330)), [11]]


def test_graph_decode_equals_eager(gpu):
    p = SamplingParams(max_tokens=12, ignore_eos=True)
    a = [s.output for s in _engine(graphs=False).generate(PROMPTS, p)]
    b = [s.output for s in _engine(graphs=True).generate(PROMPTS, p)]
    assert a == b


@pytest.mark.parametrize("pp,mbs", [(2, 1), (4, 1), (4, 3)])
def test_pipeline_loopback_equals_single_stage(gpu, pp, mbs):
    # same micro-batch count on both sides: identical GEMM shapes -> bitwise-equal decisions
    # (a different micro-batch split changes hipBLASLt's M and therefore bf16 rounding)
    p = SamplingParams(max_tokens=8, ignore_eos=True)
    a = [s.output for s in _engine(pp=1, mbs=mbs).generate(PROMPTS, p)]
    b = [s.output for s in _engine(pp=pp, mbs=mbs).generate(PROMPTS, p)]
    assert a == b


def _forced_logits(stage, prompts, forced, window=0, sinks=0):
    pool = stage.make_pool(128, 64, window_length=window, num_sink_tokens=sinks, max_chunk=256)
    sids = list(range(len(prompts)))
    for s, p in zip(sids, prompts):
        pool.manager.append(s, len(p))
    meta = pool.build_metadata(sids, [len(p) for p in prompts])
    meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(stage.device)
    ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=stage.device)
    outs = [stage(ids, meta, pool).float().cpu()]
    for step in forced:
        for s in sids:
            pool.manager.append(s, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        outs.append(stage(torch.tensor(step, dtype=torch.int32, device=stage.device), meta,
                          pool).float().cpu())
    return outs


def test_window_mode_runs_and_matches_full_cache_before_eviction(gpu):
    # while the sequences are shorter than the window the sink cache equals a full cache
    stage = CausalLMStage(SPEC, 0, 4, device=gpu).init_random(3)
    prompts = PROMPTS[:2]
    forced = [[17, 23], [5, 900], [44, 1], [2, 3]]
    a = _forced_logits(stage, prompts, forced)
    b = _forced_logits(stage, prompts, forced, window=512, sinks=4)
    for x, y in zip(a, b):
        assert (x - y).abs().max() < 0.03 * max(1.0, x.abs().max().item())
    # and it keeps generating past the window (ring eviction) without error
    long = [list(range(1, 600))]
    out = _engine(window=256, sinks=4).generate(long, SamplingParams(max_tokens=20, ignore_eos=True))
    assert len(out[0].output) == 20


def test_fp8_weights_close_to_bf16(gpu):
    stage = CausalLMStage(SPEC, 0, 4, device=gpu).init_random(9)
    prompts = [list(range(1, 50))]
    a = _stage_logits(stage, prompts, 0)[0]
    stage.quantize_fp8()
    b = _stage_logits(stage, prompts, 0)[0]
    rel = (a - b).norm() / a.norm()
    assert rel < 0.1, rel


def test_fp8_stage_gpu_matches_cpu(gpu):
    """The fused fp8 path (norm->quant, silu->quant, hipBLASLt row-wise scaled GEMM) against the
    CPU dequantised reference with identical fp8 weights."""
    prompts = [list(range(1, 70)), [5, 6, 7]]
    cpu = CausalLMStage(SPEC, 0, 4).init_random(3)
    g = CausalLMStage(SPEC, 0, 4, device=gpu).init_random(3)
    g.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})
    cpu.quantize_fp8()
    g.quantize_fp8()
    a = _stage_logits(cpu, prompts, 0)[0]
    b = _stage_logits(g, prompts, 0)[0]
    rel = ((a - b).norm() / a.norm()).item()
    assert rel < 0.05, rel


def test_fp8_tile_path_fused_swiglu_matches_cpu(gpu):
    """fp8 weights on the hand-written tile GEMMs: QKV partials into the RoPE kernel, O partials
    into the fused norm + quantiser, gate|up with the SwiGLU epilogue on pairwise-interleaved fp8
    rows + scales, down partials into the next layer's quantiser — against the CPU dequantised
    reference with identical fp8 weights (prefill of 384 tokens), and (+ a 128-sequence decode
    step) against the unfused order (reduce passes, SwiGLU as a separate pass)."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=1024, num_heads=8, num_kv_heads=2,
                        head_dim=64)
    prompts = [[(7 * i + j) % 997 + 1 for j in range(3)] for i in range(128)]
    cpu = CausalLMStage(spec, 0, 3).init_random(4)
    g = CausalLMStage(spec, 0, 3, device=gpu).init_random(4)
    g.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})
    cpu.quantize_fp8()
    g.quantize_fp8()
    wq0 = g.block.layers[0].mlp.gate_up_proj.weight_fp8.clone()
    g.block.set_fused_swiglu(True)
    assert all(l.mlp.fused_swiglu for l in g.block.layers)
    assert not torch.equal(g.block.layers[0].mlp.gate_up_proj.weight_fp8.view(torch.uint8),
                           wq0.view(torch.uint8))
    a = _stage_logits(cpu, prompts, 0)[0]

    def prefill_then_decode(stage):
        pool = stage.make_pool(256, block_size=64)
        sids = list(range(len(prompts)))
        for sid, p in zip(sids, prompts):
            pool.manager.append(sid, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(gpu)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=gpu)
        pre = stage(ids, meta, pool).float().cpu()
        for sid in sids:
            pool.manager.append(sid, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        toks = torch.tensor([(13 * i) % 997 + 1 for i in sids], dtype=torch.int32, device=gpu)
        return pre, stage(toks, meta, pool).float().cpu()

    b = prefill_then_decode(g)
    rel = ((a - b[0]).norm() / a.norm()).item()
    # two fp8 pipelines that round anything differently (here: bf16 split-K partials, MX block
    # scales) land ~5 % apart on this random-init stack, while a layout bug lands near 100 %
    # (test_fp8_bf16_splitk_partials_close_to_fp32_partials measures both at the same 10 % from
    # the bf16-weight model)
    assert rel < 0.08, rel
    # the decode step against the unfused order (SwiGLU pass, reduce passes)
    g.block.set_fused_swiglu(False)
    with ops.kernel_policy(defer_splitk=False, fp8_mx=False):
        c = prefill_then_decode(g)
    for x, y in zip(c, b):
        rel = ((x - y).norm() / x.norm()).item()
        assert rel < 0.08, rel
    g.block.set_fused_swiglu(True)
    g.block.set_fused_swiglu(False)   # round trip restores the quantised rows exactly
    assert torch.equal(g.block.layers[0].mlp.gate_up_proj.weight_fp8.view(torch.uint8),
                       wq0.view(torch.uint8))


def test_fp8_mx_down_projection_engages_and_matches_per_row_path(gpu, monkeypatch):
    """fp8 decode with the SwiGLU output handed to the down projection as MX (e8m0 per row and
    128-column block, quantised in the gate|up epilogue) vs the bf16 h + per-row quantiser path
    (KernelPolicy.fp8_mx=False): the MX kernels run for every layer, and against the bf16-weight
    logits the MX path is no less accurate than the per-row one."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=1024, num_heads=8, num_kv_heads=2,
                        head_dim=64)
    prompts = [[(5 * i + j) % 991 + 1 for j in range(4)] for i in range(256)]
    g = CausalLMStage(spec, 0, 3, device=gpu).init_random(6)
    calls = []
    real = ops.gemm_tile_fp8_mx

    def counted(*a, **k):
        calls.append(1)
        return real(*a, **k)
    monkeypatch.setattr(ops, "gemm_tile_fp8_mx", counted)

    def decode(stage):
        pool = stage.make_pool(256, block_size=64)
        sids = list(range(len(prompts)))
        for sid, p in zip(sids, prompts):
            pool.manager.append(sid, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(gpu)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=gpu)
        stage(ids, meta, pool)
        for sid in sids:
            pool.manager.append(sid, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        toks = torch.tensor([(11 * i) % 991 + 1 for i in sids], dtype=torch.int32, device=gpu)
        return stage(toks, meta, pool).float().cpu()

    ref = decode(g)   # bf16 weights
    g.quantize_fp8()
    g.block.set_fused_swiglu(True)
    a = decode(g)
    n = len(calls)
    assert n >= 3, calls   # at least one MX down projection per layer (the decode step)
    with ops.kernel_policy(fp8_mx=False):
        b = decode(g)
    assert len(calls) == n
    # two fp8 quantisations of h differ by ~fp8 resolution; against the bf16 model the MX path
    # (finer, per-block scales) is no worse than the per-row one
    rel_mx = ((a - ref).norm() / ref.norm()).item()
    rel_row = ((b - ref).norm() / ref.norm()).item()
    assert rel_mx < 0.1 and rel_mx < 1.1 * rel_row + 0.005, (rel_mx, rel_row)


def test_sampling_params_in_engine(gpu):
    p = SamplingParams(max_tokens=10, temperature=0.8, top_k=50, top_p=0.9, seed=1, ignore_eos=True)
    a = [s.output for s in _engine().generate(PROMPTS, p)]
    b = [s.output for s in _engine().generate(PROMPTS, p)]
    assert a == b  # seeded sampling is reproducible
    assert all(len(x) == 10 for x in a)


def test_sink_window_matches_streamingllm_definition_gpu(gpu):
    """GPU version of the CPU test: 1-layer model, long decode through the ring with sinks equals
    a fresh full-cache forward of [sinks] + [last W - n_sink tokens] at positions 0..W-1."""
    spec = SPEC.replace(num_layers=1)
    stage = CausalLMStage(spec, 0, 1, device=gpu).init_random(11)
    W, S = 96, 4
    g = torch.Generator().manual_seed(0)
    toks = torch.randint(0, spec.vocab_size, (300,), generator=g).tolist()
    outs = _forced_logits(stage, [toks[:16]], [[t] for t in toks[16:]], window=W, sinks=S)
    view = toks[:S] + toks[len(toks) - (W - S):]
    ref = _forced_logits(stage, [view], [])[0]
    assert (outs[-1] - ref).abs().max() < 0.03 * max(1.0, ref.abs().max().item())


def test_lookahead_equals_plain_decode_gpu(gpu):
    """Single micro-batch lookahead on the GPU (hipGraph decode, sampled tokens fed back on the
    device) gives exactly the tokens of the plain loop, greedy and seeded-temperature."""
    for p in (SamplingParams(max_tokens=10, ignore_eos=True),
              SamplingParams(max_tokens=10, temperature=0.9, top_k=40, seed=3, ignore_eos=True)):
        outs = []
        for la in (False, True):
            eng = _engine(mbs=1)
            eng.pipeline.lookahead = la
            outs.append([s.output for s in eng.generate(PROMPTS, p)])
        assert outs[0] == outs[1]


def test_fp8_kv_cache_engine_close_to_bf16(gpu):
    stage = CausalLMStage(SPEC, 0, 4, device=gpu).init_random(21)
    prompts = [list(range(1, 90)), [5, 6, 7]]

    def run(kv_dtype):
        pool = stage.make_pool(128, 64, kv_dtype=kv_dtype)
        sids = [0, 1]
        for s, p in zip(sids, prompts):
            pool.manager.append(s, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = torch.tensor([88, 91], device=gpu)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=gpu)
        outs = [stage(ids, meta, pool).float().cpu()]
        for toks in ([3, 4], [9, 10], [11, 12]):
            for s in sids:
                pool.manager.append(s, 1)
            meta = pool.build_metadata(sids, [1, 1])
            outs.append(stage(torch.tensor(toks, dtype=torch.int32, device=gpu), meta,
                              pool).float().cpu())
        return outs

    a, b = run(torch.bfloat16), run(torch.float8_e4m3fn)
    for x, y in zip(a, b):
        assert ((x - y).norm() / x.norm()).item() < 0.08


def test_int8_weights_close_to_bf16(gpu):
    """LLM.int8 mode (reference convert_to_optimized_block(quantize=True, threshold)): int8 MFMA
    tile GEMM + bf16 outlier columns, end to end through the stage."""
    stage = CausalLMStage(SPEC, 0, 4, device=gpu).init_random(9)
    prompts = [list(range(1, 50))]
    a = _stage_logits(stage, prompts, 0)[0]
    stage.quantize("int8", threshold=5.0)
    assert stage.block.layers[0].self_attn.qkv_proj.is_int8
    b = _stage_logits(stage, prompts, 0)[0]
    rel = (a - b).norm() / a.norm()
    assert rel < 0.1, rel


def test_int8_fused_path_matches_unfused(gpu, monkeypatch):
    """LLM.int8 stage on the fused path (outlier product in the tile epilogue, SwiGLU on
    interleaved int8 rows, QKV / O / down partials into their consumers) vs the unfused path
    (separate reduce passes, silu_mul), at a 128-sequence decode batch and a 384-token prefill."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=1024, num_heads=8, num_kv_heads=2,
                        head_dim=64)
    g = CausalLMStage(spec, 0, 3, device=gpu).init_random(12)
    g.quantize("int8", threshold=3.0)
    prompts = [[(5 * i + j) % 997 + 1 for j in range(3)] for i in range(128)]

    def run():
        pool = g.make_pool(256, block_size=64)
        sids = list(range(len(prompts)))
        for sid, p in zip(sids, prompts):
            pool.manager.append(sid, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(gpu)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=gpu)
        pre = g(ids, meta, pool).float().cpu()
        for sid in sids:
            pool.manager.append(sid, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        toks = torch.tensor([(11 * i) % 997 + 1 for i in sids], dtype=torch.int32, device=gpu)
        return pre, g(toks, meta, pool).float().cpu()

    # fp32 partials on both sides: this compares the fused epilogue with the unfused path (bf16
    # partials are checked against the bf16 model in test_8bit_bf16_splitk_partials_*)
    with ops.kernel_policy(bf16_partials=False, defer_splitk=False):
        a = run()
    wq0 = g.block.layers[0].mlp.gate_up_proj.weight_int8.clone()
    g.block.set_fused_swiglu(True)
    assert g.block.layers[0].mlp.fused_swiglu
    with ops.kernel_policy(bf16_partials=False):
        b = run()
    for x, y in zip(a, b):
        rel = ((x - y).norm() / x.norm()).item()
        assert rel < 0.02, rel
    g.block.set_fused_swiglu(False)
    assert torch.equal(g.block.layers[0].mlp.gate_up_proj.weight_int8, wq0)


def test_deferred_splitk_reduce_is_bit_identical(gpu):
    """Split-K partials reduced inside the next RMSNorm (default) vs the separate reduce pass
    (KernelPolicy.defer_splitk=False): same bf16 rounding points, so the stage output is
    bit-identical."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=1024, num_heads=4, num_kv_heads=2,
                        head_dim=128)
    g = CausalLMStage(spec, 0, 4, device=gpu).init_random(5)
    prompts = [list(range(1, 200)), list(range(3, 150))]   # 347 rows: tile GEMMs with split-K
    with ops.kernel_policy(bf16_partials=False):   # fp32 partials: the bit-identity claim
        a = _stage_logits(g, prompts, 0)[0]
        with ops.kernel_policy(bf16_partials=False, defer_splitk=False):
            b = _stage_logits(g, prompts, 0)[0]
    assert torch.equal(a, b)
    # default bf16 partials (one extra bf16 rounding per partial): close, not identical
    c = _stage_logits(g, prompts, 0)[0]
    rel = ((c.float() - b.float()).norm() / b.float().norm()).item()
    assert rel < 1e-2, rel


def test_deferred_splitk_reduce_is_bit_identical_fp8(gpu):
    """fp8 weights: the long-K down projection (fp8 tile GEMM, split-K) hands its partials to the
    next layer's fused RMSNorm + fp8 quantiser; bit-identical to the separate reduce pass."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=16384, num_heads=4, num_kv_heads=2,
                        head_dim=128)
    g = CausalLMStage(spec, 0, 3, device=gpu).init_random(6)
    g.quantize_fp8()
    prompts = [list(range(1, 200)), list(range(3, 150))]
    with ops.kernel_policy(bf16_partials=False):   # fp32 partials: the bit-identity claim
        a = _stage_logits(g, prompts, 0)[0]
    with ops.kernel_policy(bf16_partials=False, defer_splitk=False):
        b = _stage_logits(g, prompts, 0)[0]
    assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["fp8", "int8"])
def test_8bit_bf16_splitk_partials_as_accurate_as_fp32(gpu, monkeypatch, mode):
    """8-bit weights with bf16 split-K partials (gemm_tile epilogue 4, summed in fp32 by the RoPE
    kernel and the fused norm (+ quantiser) consumers) vs fp32 partials, a 256-sequence decode step
    through QKV / O / down split-K: both equally far from the bf16-weight model."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=2048, num_heads=8, num_kv_heads=2,
                        head_dim=64)
    g = CausalLMStage(spec, 0, 3, device=gpu).init_random(8)
    prompts = [[(3 * i + j) % 983 + 1 for j in range(5)] for i in range(256)]
    calls = []
    mod = ops.native()

    def spy(out, a, b, splits=1, epilogue=0, *args, **kw):
        calls.append(epilogue)
        return mod.gemm_tile(out, a, b, splits, epilogue, *args, **kw)

    class _N:
        def __getattr__(self, k):
            return spy if k == "gemm_tile" else getattr(mod, k)
    nat = _N()

    def decode(parts):
        with ops.kernel_policy(bf16_partials=parts == "1"):
            return _decode()

    def _decode():
        pool = g.make_pool(256, block_size=64)
        sids = list(range(len(prompts)))
        for sid, p in zip(sids, prompts):
            pool.manager.append(sid, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(gpu)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=gpu)
        g(ids, meta, pool)
        for sid in sids:
            pool.manager.append(sid, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        toks = torch.tensor([(7 * i) % 983 + 1 for i in sids], dtype=torch.int32, device=gpu)
        calls.clear()
        with monkeypatch.context() as m:
            m.setattr(ops, "native", lambda: nat)
            y = g(toks, meta, pool).float().cpu()
        return y, list(calls)

    ref, _ = decode("1")   # bf16 weights: fp32 partials throughout
    if mode == "fp8":
        g.quantize_fp8()
    else:
        g.quantize("int8", threshold=3.0)
    g.block.set_fused_swiglu(True)
    a, ca = decode("1")
    b, cb = decode("0")
    assert 4 in ca and 4 not in cb and 1 in cb   # the decode step's split-K GEMMs took each path
    # against the bf16-weight model, bf16 partials are as accurate as fp32 ones (their difference
    # to each other is of the same order as each one's fp8 error: a random-init stack amplifies
    # any perturbation, so the two are compared through the reference, not to each other)
    rel_b = ((a - ref).norm() / ref.norm()).item()
    rel_f = ((b - ref).norm() / ref.norm()).item()
    print(mode, "logits vs bf16 model: bf16 partials", rel_b, "fp32 partials", rel_f)
    assert rel_b < 1.15 * rel_f + 0.005, (rel_b, rel_f)


@pytest.mark.parametrize("preset", ["qwen2-7b", "mistral-7b"])
def test_llama_family_variants_gpu_match_cpu(gpu, preset):
    """Qwen2 (q/k/v bias, GQA group 7, hidden 3584) and Mistral (sliding window) shapes on the
    HIP kernels vs the CPU reference path, 2 real-size layers, prefill + sliding-window decode."""
    from distributed_llm_inference.config import PRESETS
    spec = PRESETS[preset].replace(num_layers=2, vocab_size=4096)
    if spec.sliding_window:
        spec = spec.replace(sliding_window=64)
    cpu = CausalLMStage(spec, 0, 2).init_random(7)
    with torch.no_grad():
        for n, p in cpu.named_parameters():
            if n.endswith(".bias"):
                p.normal_(0, 0.5)
    g = CausalLMStage(spec, 0, 2, device=gpu)
    g.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})
    prompts = [list(range(1, 90)), [5, 6, 7]]

    def run(stage):
        pool = stage.make_pool(64, block_size=64, window_length=spec.sliding_window or 0)
        sids = [0, 1]
        for s, p in zip(sids, prompts):
            pool.manager.append(s, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(stage.device)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=stage.device)
        return stage(ids, meta, pool).float().cpu()

    a, b = run(cpu), run(g)
    rel = ((a - b).norm() / a.norm()).item()
    assert rel < 0.03, rel


def test_reference_llama_block_api_on_gpu(gpu):
    """The reference's stage API (LlamaBlock(config, layer_ids)(generation_id, hidden_states,
    past_key_value=PartialLlamaSinkCache)) on the HIP kernels: incremental session decoding
    equals the full causal pass, sessions are isolated, close_session frees them, and the GPU
    agrees with the CPU reference path."""
    from distributed_llm_inference.models import LlamaBlock, PartialLlamaSinkCache
    spec = SPEC.replace(hidden_size=512, intermediate_size=1024, num_heads=4, num_kv_heads=2,
                        head_dim=128)
    cpu = LlamaBlock(spec, [0, 1, 2]).init_random(4)
    blk = LlamaBlock(spec, [0, 1, 2], device=gpu)
    blk.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})
    torch.manual_seed(3)
    x = torch.randn(2, 40, 512, dtype=torch.bfloat16)
    (full_cpu,) = cpu("g", x)
    xg = x.to(gpu)
    (full,) = blk("g-full", xg)
    rel = ((full.float().cpu() - full_cpu.float()).norm() / full_cpu.float().norm()).item()
    assert rel < 0.02, rel
    cache = PartialLlamaSinkCache(0, 0, num_blocks=64, block_size=64)
    parts = [blk("g1", xg[:, a:b], past_key_value=cache)[0] for a, b in ((0, 30), (30, 31), (31, 40))]
    (other,) = blk("g2", xg[:, :5].flip(0), past_key_value=cache)   # another session in between
    inc = torch.cat(parts, 1)
    rel = ((inc.float() - full.float()).norm() / full.float().norm()).item()
    assert rel < 0.02, rel
    assert cache.get_seq_length(0, "g1") == 40 and cache.get_seq_length(0, "g2") == 5
    cache.close_session("g1")
    assert cache.get_seq_length(0, "g1") == 0


@pytest.mark.parametrize("temperature", [0.0, 0.8])
def test_rotating_head_split_matches_local_head(gpu, temperature):
    """The rotating LM head's two halves on the GPU (runtime/head.py): the last stage's decode
    graph that ends at the final norm, then HeadRunner's projection + sampling graph replayed on a
    side stream, produce exactly the tokens of the fused last-stage head (greedy and seeded
    top-k sampling)."""
    from distributed_llm_inference.parallel.pipeline import _sample_tokens_to_host
    from distributed_llm_inference.runtime.head import HeadRunner
    p = SamplingParams(max_tokens=8, temperature=temperature, top_k=30, seed=11, ignore_eos=True)
    ref = [s.output for s in _engine(pp=2, mbs=3).generate(PROMPTS, p)]
    eng = _engine(pp=2, mbs=3)
    pipe = eng.pipeline
    last = pipe.executors[-1]
    runner = HeadRunner(last.stage.head, last.device, last.max_num_seqs, True, last.graph_sizes)
    side = torch.cuda.Stream()
    orig, split = pipe._issue, []

    def issue(plan):
        if not (plan.seq_ids and plan.is_decode and len(plan.sample_rows) == len(plan.seq_ids)):
            return orig(plan)
        x = None
        for ex in pipe.executors[:-1]:
            x = ex.execute(plan, x)
        h = last.execute(plan, x, project=False)
        assert h.shape == (len(plan.seq_ids), SPEC.hidden_size)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            tok = runner.run(plan, h).clone()
        torch.cuda.current_stream().wait_stream(side)
        pipe._last_tokens = tok
        pipe._results[plan.step] = _sample_tokens_to_host(tok)
        split.append(plan.step)

    pipe._issue = issue
    got = [s.output for s in eng.generate(PROMPTS, p)]
    assert len(split) >= 6 and runner._graphs   # decode steps took the split path, graphed
    assert got == ref


def test_bf16_splitk_partials_end_to_end_vs_cpu_reference(gpu, monkeypatch):
    """Default bf16 path: QKV / O / down split-K partials stored as bf16 (gemm_tile / gemm4
    epilogue 4) vs fp32 partials, a 256-sequence decode step, each against the fp32 CPU
    reference of the same weights (the extra rounding is bounded end to end)."""
    spec = SPEC.replace(hidden_size=1024, intermediate_size=2048, num_heads=16, num_kv_heads=4,
                        head_dim=64)
    cpu = CausalLMStage(spec, 0, 3).init_random(9)
    g = CausalLMStage(spec, 0, 3, device=gpu).init_random(9)
    g.load_state_dict({k: v.to(gpu) for k, v in cpu.state_dict().items()})
    prompts = [[(5 * i + j) % 983 + 1 for j in range(4)] for i in range(256)]
    mod = ops.native()
    calls = []

    class _N:
        def __getattr__(self, k):
            if k not in ("gemm_tile", "gemm4"):   # the tile GEMMs (gemm4: the bf16 default)
                return getattr(mod, k)
            fn = getattr(mod, k)

            def spy(out, a, b, splits=1, epilogue=0, *args, **kw):
                calls.append(epilogue)
                return fn(out, a, b, splits, epilogue, *args, **kw)
            return spy

    def decode(stage, parts=None):
        with ops.kernel_policy(bf16_partials=parts != "0"):
            return _decode(stage)

    def _decode(stage):
        dev = stage.device
        pool = stage.make_pool(256, block_size=64)
        sids = list(range(len(prompts)))
        for sid, p in zip(sids, prompts):
            pool.manager.append(sid, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(dev)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=dev)
        stage(ids, meta, pool)
        for sid in sids:
            pool.manager.append(sid, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        toks = torch.tensor([(11 * i) % 983 + 1 for i in sids], dtype=torch.int32, device=dev)
        calls.clear()
        with monkeypatch.context() as m:
            if dev.type == "cuda":
                m.setattr(ops, "native", lambda: _N())
            y = stage(toks, meta, pool).float().cpu()
        return y, list(calls)

    ref, _ = decode(cpu)
    a, ca = decode(g, "1")
    b, cb = decode(g, "0")
    assert 4 in ca and 4 not in cb and 1 in cb, (ca, cb)   # both partial paths really ran
    rel_b = ((a - ref).norm() / ref.norm()).item()
    rel_f = ((b - ref).norm() / ref.norm()).item()
    print("bf16 logits vs CPU reference: bf16 partials", rel_b, "fp32 partials", rel_f)
    assert rel_b < 0.03 and rel_b < 1.15 * rel_f + 0.005, (rel_b, rel_f)


@pytest.mark.parametrize("mode", ["fp8", "int8"])
def test_8bit_gemv_vs_quantised_path_bounded(gpu, monkeypatch, mode):
    """1-2 decode rows take the weight-streaming GEMV on bf16 activations; >= 3 rows (or
    KernelPolicy.gemv=False) quantise the activations (fp8 rows / LLM.int8 with outlier split).  Both stay
    close to the fp32 product of the same 8-bit weights, and the GEMV is the closer of the two, so
    the batch-size dependence of a row's output is bounded (docs/parity.md C11)."""
    from distributed_llm_inference.models.common import Linear
    torch.manual_seed(0)
    lin = Linear(8192, 1024, device=gpu)
    lin.weight.data.normal_(0, 0.02)
    x = torch.randn(2, 8192, device=gpu).to(torch.bfloat16)
    x[:, 17] *= 12.0    # one outlier feature, as real activations have
    if mode == "fp8":
        lin.quantize_fp8()
        wdq = lin.weight_fp8.float() * lin.weight_scale.float().view(-1, 1)
    else:
        lin.quantize_int8(threshold=6.0)
        wdq = lin.weight_int8.float() * lin.weight_scale.float().view(-1, 1)
    ref = x.float() @ wdq.t()
    a = lin(x).float()
    with ops.kernel_policy(gemv=False):
        b = lin(x).float()
    ea = ((a - ref).norm() / ref.norm()).item()
    eb = ((b - ref).norm() / ref.norm()).item()
    eab = ((a - b).norm() / ref.norm()).item()
    print(mode, "GEMV", ea, "quantised path", eb, "difference", eab)
    assert ea < 0.01 and eb < 0.06 and ea <= eb + 1e-3 and eab < 0.06, (ea, eb, eab)


@pytest.mark.parametrize("quantize", [False, "fp8", "int8"])
def test_gemv_fused_norm_path_matches_unfused_decode(gpu, monkeypatch, quantize):
    """1-2 row decode with the RMSNorms fused into the QKV / gate|up GEMVs (KernelPolicy.gemv_norm,
    default) against the unfused order: bf16 weights give identical greedy tokens; 8-bit
    weights (the fused path feeds bf16 rows instead of quantised ones) stay close."""
    prompts = [list(range(3, 40))]

    def run(flag):
        with ops.kernel_policy(gemv_norm=flag == "1"):
            eng = _engine(graphs=False, quantize=quantize)
            outs = eng.generate(prompts, SamplingParams(max_tokens=12, temperature=0.0))
        return [o.output for o in outs]

    a, b = run("1"), run("0")
    if not quantize:
        assert a == b
    else:
        agree = sum(x == y for x, y in zip(a[0], b[0])) / len(a[0])
        assert agree >= 0.5, (a, b)


def test_gemm4_dispatch_bit_identical_in_a_decode_step(gpu, monkeypatch):
    """KernelPolicy.gemm4 routes the bf16 decode projections to gemm4.hip (same epilogues: split-K
    partials into the norms / RoPE, fused SwiGLU): a 256-sequence decode step's logits are
    bit-identical to the gemm_tile ones."""
    spec = SPEC.replace(hidden_size=512, intermediate_size=1024, num_heads=8, num_kv_heads=4,
                        head_dim=64)
    g = CausalLMStage(spec, 0, 2, device=gpu).init_random(4)
    g.block.set_fused_swiglu(True)
    prompts = [[(3 * i + j) % 977 + 1 for j in range(3)] for i in range(256)]

    def step(flag):
        with ops.kernel_policy(gemm4=flag == "1"):
            return _step()

    def _step():
        pool = g.make_pool(320, block_size=64)   # one block per sequence
        sids = list(range(len(prompts)))
        for sid, p in zip(sids, prompts):
            pool.manager.append(sid, len(p))
        meta = pool.build_metadata(sids, [len(p) for p in prompts])
        meta.logits_rows = (torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1).to(gpu)
        ids = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device=gpu)
        g(ids, meta, pool)
        for sid in sids:
            pool.manager.append(sid, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        toks = torch.tensor([(5 * i) % 977 + 1 for i in sids], dtype=torch.int32, device=gpu)
        return g(toks, meta, pool).float().cpu()

    a, b = step("0"), step("1")
    assert torch.equal(a, b), (a - b).abs().max().item()
