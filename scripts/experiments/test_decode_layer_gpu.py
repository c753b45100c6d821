"""The persistent batch-1 decode-layer kernel (csrc/kernels/decode_layer.hip) against the
six-kernel fused-norm GEMV path it replaces: every phase reuses that path's arithmetic, so the
logits of every decode step must be bit-identical, for bf16 / fp8 / int8 weights and bf16 / fp8
KV caches, across split-count changes as the context grows; and no grid barrier may time out."""
import pytest
import torch

from distributed_llm_inference import ops
from distributed_llm_inference.config import PRESETS
from distributed_llm_inference.models import CausalLMStage

pytestmark = pytest.mark.gpu

SPEC = PRESETS["llama-3-8b"].replace(hidden_size=1024, intermediate_size=2048, num_heads=8,
                                     num_kv_heads=2, head_dim=128, vocab_size=512)


def _decode(stage, flag, monkeypatch, kv_dtype, steps, prompt_len):
    monkeypatch.setenv("DLI_DECODE_LAYER", flag)
    dev = stage.device
    pool = stage.make_pool(64, block_size=64, kv_dtype=kv_dtype)
    prompt = [(7 * j) % 500 + 1 for j in range(prompt_len)]
    pool.manager.append(0, len(prompt))
    meta = pool.build_metadata([0], [len(prompt)])
    meta.logits_rows = torch.tensor([len(prompt) - 1], device=dev)
    stage(torch.tensor(prompt, dtype=torch.int32, device=dev), meta, pool)
    outs = []
    for s in range(steps):
        pool.manager.append(0, 1)
        meta = pool.build_metadata([0], [1])
        tok = torch.tensor([(13 * s) % 500 + 1], dtype=torch.int32, device=dev)
        outs.append(stage(tok, meta, pool).float().cpu())
    return torch.stack(outs)


@pytest.mark.parametrize("quant", [None, "fp8", "int8"])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_decode_layer_kernel_bit_identical(gpu, monkeypatch, quant, kv):
    kv_dtype = torch.float8_e4m3fn if kv == "fp8" else torch.bfloat16
    stage = CausalLMStage(SPEC, 0, 3, device=gpu).init_random(11)
    if quant == "fp8":
        stage.block.quantize_fp8()
    elif quant == "int8":
        stage.block.quantize_int8()
    stage.block.set_fused_swiglu(True)   # after quantising, as the engine does
    # 40-token prompt + 60 steps: crosses 32-key steps, cache blocks and split-count changes
    ref = _decode(stage, "0", monkeypatch, kv_dtype, 60, 40)
    got = _decode(stage, "1", monkeypatch, kv_dtype, 60, 40)
    assert torch.equal(ref, got), (ref - got).abs().max().item()
    errs = sum(l.decode_layer_errors() for l in stage.block.layers)
    assert errs == 0
    assert any(getattr(l, "_dl_bar", None) is not None for l in stage.block.layers), \
        "the decode-layer kernel did not run"


def test_decode_layer_kernel_long_context_many_splits(gpu, monkeypatch):
    """1.5k-token context: the attention phase runs 4-wave groups over many splits plus the
    partial merge phase."""
    stage = CausalLMStage(SPEC, 0, 2, device=gpu).init_random(5)
    stage.block.set_fused_swiglu(True)
    ref = _decode(stage, "0", monkeypatch, torch.bfloat16, 4, 1500)
    got = _decode(stage, "1", monkeypatch, torch.bfloat16, 4, 1500)
    assert torch.equal(ref, got), (ref - got).abs().max().item()
    assert sum(l.decode_layer_errors() for l in stage.block.layers) == 0


@pytest.mark.parametrize("quant", [None, "fp8"])
def test_decode_layer_kernel_merge_fast_path(gpu, monkeypatch, quant):
    """560-600 token contexts: 8-16 splits merged 4 at a time in the attention groups, so the
    O phase's staging merges 2-4 partials per head (its single-round path)."""
    stage = CausalLMStage(SPEC, 0, 2, device=gpu).init_random(7)
    if quant == "fp8":
        stage.block.quantize_fp8()
    stage.block.set_fused_swiglu(True)
    ref = _decode(stage, "0", monkeypatch, torch.bfloat16, 40, 560)
    got = _decode(stage, "1", monkeypatch, torch.bfloat16, 40, 560)
    assert torch.equal(ref, got), (ref - got).abs().max().item()
    assert sum(l.decode_layer_errors() for l in stage.block.layers) == 0
