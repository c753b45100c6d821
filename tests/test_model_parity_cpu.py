"""Numerics of the model stages on CPU against the installed HF transformers implementations.

These run the same code path as the GPU runtime (packed varlen tokens, paged KV pool, native
block manager) with the torch reference ops, so they pin the *model* semantics (RoPE incl. llama3
scaling, GQA, causal masking, residual stream, RMSNorm eps, GPT-2 Conv1D layout) independently of
the kernels, whose numerics are pinned by tests/test_kernels_gpu.py.
"""
import math

import pytest
import torch

from distributed_llm_inference import ops
from distributed_llm_inference.config import ModelSpec
from distributed_llm_inference.models import CausalLMStage
from distributed_llm_inference.ops.reference import build_cos_sin
from distributed_llm_inference.utils.model import stage_from_hf_model

transformers = pytest.importorskip("transformers")


def _hf_llama(layers=3, rope_scaling=None, seed=0):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(seed)
    kw = dict(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=layers,
              num_attention_heads=4, num_key_value_heads=2, rms_norm_eps=1e-5,
              max_position_embeddings=16384, tie_word_embeddings=False)
    if rope_scaling:
        kw["rope_parameters"] = dict(rope_scaling, rope_theta=500000.0)
    else:
        kw["rope_parameters"] = {"rope_type": "default", "rope_theta": 10000.0}
    cfg = LlamaConfig(**kw)
    m = LlamaForCausalLM(cfg).eval()
    with torch.no_grad():  # round weights to bf16 so both sides see identical parameters
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    return m


def _run_stage(stage, prompts, decode_steps=0, hf=None):
    """Prefill all prompts as one varlen batch, then greedy-decode; returns list of logits rows."""
    pool = stage.make_pool(64, block_size=32)
    m = pool.manager
    sids = list(range(len(prompts)))
    for s, p in zip(sids, prompts):
        m.append(s, len(p))
    meta = pool.build_metadata(sids, [len(p) for p in prompts])
    ends = torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1
    meta.logits_rows = ends
    ids = torch.tensor([t for p in prompts for t in p])
    logits = [stage(ids, meta, pool).float()]
    toks = logits[-1].argmax(-1)
    for _ in range(decode_steps):
        for s in sids:
            m.append(s, 1)
        meta = pool.build_metadata(sids, [1] * len(sids))
        logits.append(stage(toks.to(torch.int32), meta, pool).float())
        toks = logits[-1].argmax(-1)
    return logits


@pytest.mark.parametrize("rope_scaling", [None, {"rope_type": "llama3", "factor": 8.0,
                                                  "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                  "original_max_position_embeddings": 64}])
def test_llama_prefill_and_decode_match_hf(rope_scaling):
    hf = _hf_llama(rope_scaling=rope_scaling)
    stage = stage_from_hf_model(hf, 0, hf.config.num_hidden_layers)
    prompts = [[5, 17, 99, 3, 250, 7, 7, 1, 42, 11, 19], [8, 2, 64]]
    steps = 4
    ours = _run_stage(stage, prompts, decode_steps=steps)
    # HF reference: run each full sequence (prompt + our generated tokens) without cache
    gen = torch.stack([o.argmax(-1) for o in ours], 1)  # [B, steps+1]
    for b, p in enumerate(prompts):
        seq = torch.tensor(p + gen[b, :steps].tolist())[None]
        with torch.no_grad():
            ref_logits = hf(seq).logits[0].float()
        for s in range(steps + 1):
            pos = len(p) - 1 + s
            a, r = ours[s][b], ref_logits[pos]
            err = (a - r).abs().max().item()
            assert err < 0.05 * max(1.0, r.abs().max().item()), f"b={b} step={s} err={err}"


def test_rope_table_matches_hf_llama3():
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding
    from transformers import LlamaConfig
    rs = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
          "original_max_position_embeddings": 8192, "rope_theta": 500000.0}
    cfg = LlamaConfig(hidden_size=4096, num_attention_heads=32, rope_parameters=rs,
                      max_position_embeddings=131072)
    rot = LlamaRotaryEmbedding(cfg)
    pos = torch.tensor([[0, 1, 100, 5000, 20000, 100000]])
    cos, sin = rot(torch.zeros(1, dtype=torch.float32), pos)
    table = build_cos_sin(128, 100001, 500000.0, {k: v for k, v in rs.items() if k != "rope_theta"})
    ours = table[pos[0]]
    # HF forms position*inv_freq in fp32 (error grows ~linearly with position); ours is fp64-exact
    tol = (2e-4 + 1e-7 * pos[0].float())[:, None]
    assert ((ours[:, :64] - cos[0, :, :64]).abs() <= tol).all()
    assert ((ours[:, 64:] - sin[0, :, :64]).abs() <= tol).all()


def test_pipeline_split_equals_single_stage():
    spec = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=4,
                     num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                     max_position_embeddings=2048)
    full = CausalLMStage(spec, 0, 4).init_random(7)
    s0 = CausalLMStage(spec, 0, 2).init_random(7)
    s1 = CausalLMStage(spec, 2, 4).init_random(7)
    prompts = [[1, 2, 3, 4, 5], [9, 8]]
    ref = _run_stage(full, prompts, decode_steps=2)
    # run the two stages by hand with their own pools
    p0, p1 = s0.make_pool(64, 32), s1.make_pool(64, 32)
    sids = [0, 1]
    for pool in (p0, p1):
        for s, p in zip(sids, prompts):
            pool.manager.append(s, len(p))
    ids = torch.tensor([t for p in prompts for t in p])
    m0 = p0.build_metadata(sids, [5, 2])
    m1 = p1.build_metadata(sids, [5, 2], logits_rows=torch.tensor([4, 6]))
    h = s0(ids, m0, p0)
    out = s1(h, m1, p1).float()
    assert torch.allclose(out, ref[0], atol=1e-2, rtol=1e-2)


def test_fp8_stage_close_to_bf16_cpu():
    """fp8-weight path (fused norm->quant and silu->quant producers) on the CPU reference ops."""
    spec = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=2,
                     num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                     max_position_embeddings=2048)
    st = CausalLMStage(spec, 0, 2).init_random(11)
    prompts = [[1, 2, 3, 4, 5], [9, 8]]
    a = _run_stage(st, prompts, decode_steps=1)
    st.quantize_fp8()
    b = _run_stage(st, prompts, decode_steps=1)
    for x, y in zip(a, b):
        assert ((x - y).norm() / x.norm()).item() < 0.1


def test_fp8_stage_head_dim_128_uses_mx_attention_handoff_cpu(monkeypatch):
    """head_dim 128 fp8 stages hand the single-split decode attention output to the O projection
    as MX fp8 (the GPU attention epilogue's format; CPU: ops.mx_quantize of the bf16 output).
    The MX and per-row paths agree closely, and both stay close to bf16."""
    spec = ModelSpec(name="t128", vocab_size=300, hidden_size=256, intermediate_size=512,
                     num_layers=2, num_heads=2, num_kv_heads=1, head_dim=128, rope_theta=10000.0,
                     max_position_embeddings=2048)
    assert ops.attn_decode_mx_ok(128, 1) and not ops.attn_decode_mx_ok(64, 1)
    assert not ops.attn_decode_mx_ok(128, 4)
    st = CausalLMStage(spec, 0, 2).init_random(5)
    prompts = [[1, 2, 3, 4, 5, 6], [9, 8, 7]]
    a = _run_stage(st, prompts, decode_steps=1)
    st.quantize_fp8()
    calls = []
    real = ops.attn_decode

    def spy(*args, **kw):
        calls.append(kw.get("mx_out", False))
        return real(*args, **kw)
    monkeypatch.setattr(ops, "attn_decode", spy)
    b = _run_stage(st, prompts, decode_steps=1)
    assert calls and all(calls), calls           # every decode step took the MX hand-off
    calls.clear()
    with ops.kernel_policy(fp8_mx=False):
        c = _run_stage(st, prompts, decode_steps=1)
    assert calls and not any(calls)
    for x, y, z in zip(a, b, c):   # (one decode step: later ones may sample different tokens)
        assert ((x - y).norm() / x.norm()).item() < 0.15
        assert ((y - z).norm() / z.norm()).item() < 0.1


def test_mx_fp8_quantiser_layout_and_linear_cpu():
    """MX activations (fp8 + e8m0 per (row, 128-column block)): exponent layout, dequantisation
    error, and the Linear path that consumes them (CPU reference of gemm_tile.hip kFp8Mx)."""
    from distributed_llm_inference.models.common import Linear
    torch.manual_seed(3)
    M, K = 70, 384
    mag = torch.exp2(torch.randint(-8, 9, (M, K // 128)).float()).repeat_interleave(128, 1)
    h = (torch.randn(M, K) * mag).to(torch.bfloat16)
    a = ops.mx_quantize(h)
    nb = (M + 63) // 64
    assert a.sc.numel() == (K // 128) * nb * 64 and a.q.dtype == torch.float8_e4m3fn
    e = a.exponents()
    am = h.float().abs().view(M, K // 128, 128).amax(-1)
    # smallest power of two that brings every block under 448
    assert ((am / torch.exp2(e.float())) <= 448).all()
    assert ((am / torch.exp2(e.float() - 1)) > 448).all()
    # byte of (row r, block kt) sits at (kt * nb + r // 64) * 64 + (r % 16) * 4 + (r % 64) // 16
    r, kt = 37, 2
    assert int(a.sc[(kt * nb + r // 64) * 64 + (r % 16) * 4 + (r % 64) // 16]) == int(e[r, kt]) + 127
    err = (a.dequantize() - h.float()).abs()
    assert (err <= h.float().abs() / 16 + am.repeat_interleave(128, 1) * 2 ** -17).all()
    lin = Linear(K, 256)
    torch.nn.init.normal_(lin.weight, std=0.05)
    lin.quantize_fp8()
    y = lin(None, x_q=a).float()
    ref = a.dequantize() @ (lin.weight_fp8.float() * lin.weight_scale.reshape(-1, 1)).t()
    assert (y - ref).abs().max().item() < 1e-2 * ref.abs().max().item()


def test_gpt2_matches_hf():
    from transformers import GPT2Config, GPT2LMHeadModel
    torch.manual_seed(0)
    cfg = GPT2Config(vocab_size=256, n_embd=128, n_layer=2, n_head=4, n_positions=128)
    hf = GPT2LMHeadModel(cfg).eval()
    with torch.no_grad():
        for p in hf.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    stage = stage_from_hf_model(hf, 0, 2)
    prompts = [[3, 1, 4, 1, 5, 9, 2, 6], [2, 7, 1]]
    ours = _run_stage(stage, prompts, decode_steps=2)
    gen = torch.stack([o.argmax(-1) for o in ours], 1)
    for b, p in enumerate(prompts):
        seq = torch.tensor(p + gen[b, :2].tolist())[None]
        with torch.no_grad():
            ref_logits = hf(seq).logits[0].float()
        for s in range(3):
            a, r = ours[s][b], ref_logits[len(p) - 1 + s]
            assert (a - r).abs().max() < 0.05 * max(1.0, r.abs().max().item())


# ------------------------------------------------------------------ LLM.int8 (reference Linear8bitLt)
def test_llm_int8_outlier_decomposition_cpu():
    """Activation columns above the threshold are multiplied in bf16: with a few large-magnitude
    feature columns (the LLM.int8 outlier pattern) the decomposed product stays accurate, while
    plain row-wise int8 of the same input loses the small features."""
    import torch
    from distributed_llm_inference import ops
    torch.manual_seed(0)
    M, K, N = 16, 512, 256
    x = torch.randn(M, K)
    x[:, [7, 100, 301]] *= 60.0                      # systematic outlier features
    w = torch.randn(N, K) / K ** 0.5
    xb = x.to(torch.bfloat16)
    ref = xb.float() @ w.to(torch.bfloat16).float().t()
    wq, ws = ops.quantize_weight_int8(w.to(torch.bfloat16))
    y_dec = ops.llm_int8_linear(xb, wq, ws, threshold=6.0).float()
    y_all = ops.llm_int8_linear(xb, wq, ws, threshold=0.0).float()
    e_dec = ((y_dec - ref).norm() / ref.norm()).item()
    e_all = ((y_all - ref).norm() / ref.norm()).item()
    assert e_dec < 0.02, e_dec
    assert e_all > 2 * e_dec, (e_all, e_dec)
    # the quantiser zeroes flagged columns and scales the rest by their own row absmax
    flags = torch.zeros(K, dtype=torch.uint8)
    flags[[7, 100, 301]] = 1
    q, s = ops.quant_rowwise_int8(xb, flags)
    assert int(q[:, [7, 100, 301]].abs().sum()) == 0
    assert torch.allclose(s, xb.float().masked_fill(flags.bool(), 0).abs().amax(-1) / 127)


def test_int8_stage_close_to_bf16_cpu():
    import torch
    from distributed_llm_inference.config import PRESETS
    from distributed_llm_inference.models.stage import CausalLMStage
    from distributed_llm_inference.utils import convert_to_optimized_block
    spec = PRESETS["llama-3-8b"].replace(hidden_size=256, intermediate_size=512, num_layers=2,
                                         num_heads=4, num_kv_heads=2, head_dim=64, vocab_size=1000)
    st = CausalLMStage(spec, 0, 2).init_random(5)
    torch.manual_seed(1)
    h = torch.randn(1, 29, 256).to(torch.bfloat16)
    a = st.block("g", h.clone())[0].float()
    convert_to_optimized_block(st.block, quantize="int8", threshold=5.0, device=torch.device("cpu"))
    assert st.block.layers[0].mlp.gate_up_proj.is_int8
    b = st.block("g2", h.clone())[0].float()
    assert ((a - b).norm() / a.norm()).item() < 0.05


def test_apply_rotary_pos_emb_matches_hf_with_batch():
    """Reference helper name, B2 fixed: batch > 1 broadcasts over heads and equals HF's."""
    import torch
    from transformers.models.llama.modeling_llama import apply_rotary_pos_emb as hf_apply
    from distributed_llm_inference.models.llama import apply_rotary_pos_emb
    torch.manual_seed(0)
    B, H, KVH, T, D = 3, 4, 2, 5, 16
    q, k = torch.randn(B, H, T, D), torch.randn(B, KVH, T, D)
    ang = torch.randn(B, T, D // 2)
    cos, sin = torch.cat([ang.cos()] * 2, -1), torch.cat([ang.sin()] * 2, -1)
    a = apply_rotary_pos_emb(q, k, cos, sin)
    b = hf_apply(q, k, cos, sin)
    assert torch.allclose(a[0], b[0], atol=1e-6) and torch.allclose(a[1], b[1], atol=1e-6)


# ------------------------------------------------------------ Llama-family variants (Qwen2, Mistral)
def _hf_variant(kind, layers=2, seed=1, sliding_window=None):
    torch.manual_seed(seed)
    kw = dict(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=layers,
              num_attention_heads=4, num_key_value_heads=2, rms_norm_eps=1e-6,
              max_position_embeddings=4096, tie_word_embeddings=False)
    if kind == "qwen2":
        from transformers import Qwen2Config as C, Qwen2ForCausalLM as M
        kw["rope_parameters"] = {"rope_type": "default", "rope_theta": 1000000.0}
    else:
        from transformers import MistralConfig as C, MistralForCausalLM as M
        kw["rope_parameters"] = {"rope_type": "default", "rope_theta": 10000.0}
        kw["sliding_window"] = sliding_window
    m = M(C(**kw)).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith(".bias"):   # HF zero-inits biases: make them matter
                p.normal_(0, 0.5)
            p.copy_(p.to(torch.bfloat16).float())
    return m


def _check_against_hf(hf, stage_logits, prompts, steps):
    gen = torch.stack([o.argmax(-1) for o in stage_logits], 1)
    for b, p in enumerate(prompts):
        seq = torch.tensor(p + gen[b, :steps].tolist())[None]
        with torch.no_grad():
            ref_logits = hf(seq).logits[0].float()
        for s in range(steps + 1):
            a, r = stage_logits[s][b], ref_logits[len(p) - 1 + s]
            err = (a - r).abs().max().item()
            assert err < 0.05 * max(1.0, r.abs().max().item()), f"b={b} step={s} err={err}"


def test_qwen2_matches_hf():
    """Qwen2 = Llama with q/k/v bias only (no o_proj bias), parsed from model_type."""
    hf = _hf_variant("qwen2")
    stage = stage_from_hf_model(hf, 0, hf.config.num_hidden_layers)
    spec = stage.spec
    assert spec.model_type == "qwen2" and spec.attention_bias and not spec.has_o_proj_bias
    assert stage.block.layers[0].self_attn.o_proj.bias is None
    prompts = [[5, 17, 99, 3, 250, 7, 7, 1], [8, 2, 64]]
    _check_against_hf(hf, _run_stage(stage, prompts, decode_steps=3), prompts, 3)
    # round trip through the HF config / state-dict writers
    assert ModelSpec.from_hf_config(spec.to_hf_dict()).replace(name=spec.name) == spec
    sd = stage.block.layers[0].hf_state_dict()
    assert "self_attn.q_proj.bias" in sd and "self_attn.o_proj.bias" not in sd


def test_mistral_matches_hf_within_window():
    hf = _hf_variant("mistral", sliding_window=4096)
    stage = stage_from_hf_model(hf, 0, hf.config.num_hidden_layers)
    assert stage.spec.model_type == "mistral" and stage.spec.sliding_window == 4096
    prompts = [[5, 17, 99, 3, 250, 7, 7, 1, 42], [8, 2, 64]]
    _check_against_hf(hf, _run_stage(stage, prompts, decode_steps=3), prompts, 3)


def test_mistral_sliding_window_matches_hf_beyond_window():
    """Sliding-window attention (W = 8) past the window, in prefill (13-token prompt) and decode:
    the ring window with no sink tokens reproduces HF Mistral exactly."""
    W = 8
    hf = _hf_variant("mistral", sliding_window=W)
    stage = stage_from_hf_model(hf, 0, hf.config.num_hidden_layers)
    prompts = [list(range(3, 16)), [8, 2, 64, 9, 10, 11]]
    steps = 10
    pool = stage.make_pool(64, block_size=32, window_length=W, num_sink_tokens=0)
    m = pool.manager
    sids = [0, 1]
    for s, p in zip(sids, prompts):
        m.append(s, len(p))
    meta = pool.build_metadata(sids, [len(p) for p in prompts])
    meta.logits_rows = torch.cumsum(torch.tensor([len(p) for p in prompts]), 0) - 1
    outs = [stage(torch.tensor([t for p in prompts for t in p]), meta, pool).float()]
    for _ in range(steps):
        toks = outs[-1].argmax(-1)
        for s in sids:
            m.append(s, 1)
        meta = pool.build_metadata(sids, [1, 1])
        outs.append(stage(toks.to(torch.int32), meta, pool).float())
    _check_against_hf(hf, outs, prompts, steps)


def test_engine_uses_sliding_window_from_config():
    from distributed_llm_inference.config import CacheConfig, ServeConfig
    from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    hf = _hf_variant("mistral", sliding_window=8)
    spec = ModelSpec.from_hf_config(hf.config)
    cfg = EngineConfig(model="m", cache=CacheConfig(num_blocks=64, block_size=32),
                       serve=ServeConfig(max_batch_size=4, max_num_batched_tokens=64,
                                         max_seq_len=64, use_graphs=False))
    eng = LLMEngine(spec, device="cpu", cfg=cfg)
    assert eng.executors[0].pool.manager.window_length == 8
    out = eng.generate([list(range(3, 16))], SamplingParams(max_tokens=4, ignore_eos=True))
    assert len(out[0].output) == 4


def test_llama_block_4d_custom_mask_matches_hf():
    """Reference model.py:115-119: a pre-inverted 4-D mask replaces the causal mask.  A prefix-LM
    mask (first 4 tokens attend bidirectionally) through LlamaBlock.forward equals HF's eager
    decoder layers under the same additive mask; a 4-D causal mask equals the default path."""
    from distributed_llm_inference.models.llama import LlamaBlock  # noqa: F401
    hf = _hf_llama(layers=2, seed=5)
    hf.config._attn_implementation = "eager"
    stage = stage_from_hf_model(hf, 0, 2)
    blk = stage.block
    torch.manual_seed(0)
    B, T, P = 2, 9, 4
    ids = torch.randint(0, 256, (B, T))
    with torch.no_grad():
        emb = hf.model.embed_tokens(ids).to(torch.bfloat16).float()
        neg = torch.finfo(torch.float32).min
        allowed = torch.tril(torch.ones(T, T, dtype=torch.bool))
        allowed[:P, :P] = True                                  # prefix-LM block
        mask = torch.zeros(B, 1, T, T).masked_fill(~allowed, neg)
        pos = torch.arange(T)[None].expand(B, -1)
        cos, sin = hf.model.rotary_emb(emb, pos)
        h = emb
        for layer in hf.model.layers:
            h = layer(h, attention_mask=mask, position_ids=pos, position_embeddings=(cos, sin))
            h = h[0] if isinstance(h, tuple) else h
        (ours,) = blk("s", emb.to(torch.bfloat16), attention_mask=mask)
        err = (ours.float() - h).norm() / h.norm()
        assert err.item() < 2e-2, err.item()
        # the prefix-LM mask really differs from causal on the prefix rows
        (causal,) = blk("c", emb.to(torch.bfloat16))
        assert (causal[:, :P - 1].float() - ours[:, :P - 1].float()).abs().max() > 1e-2
        # a 4-D causal mask is the default path; T = 1 decode with a 4-D all-zero mask too
        cm = torch.zeros(B, 1, T, T).masked_fill(~torch.tril(torch.ones(T, T, dtype=torch.bool)), neg)
        (c4,) = blk("c4", emb.to(torch.bfloat16), attention_mask=cm)
        assert torch.allclose(c4.float(), causal.float(), atol=2e-2, rtol=2e-2)
        x1 = torch.randn(B, 1, 128, dtype=torch.bfloat16)
        (d_plain,) = blk("c", x1)
        (d_4d,) = blk("c4", x1, attention_mask=torch.zeros(B, 1, 1, T + 1))
        assert torch.allclose(d_plain.float(), d_4d.float(), atol=2e-2, rtol=2e-2)
        with pytest.raises(ValueError):
            blk("bad", emb.to(torch.bfloat16), attention_mask=mask + 1.0)   # not inverted
