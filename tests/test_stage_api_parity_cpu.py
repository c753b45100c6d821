"""Stage-API parity nits against the reference LlamaBlock contract
(/root/reference/distributed_llm_inference/models/llama/model.py:23, 35-37, 57-76), on CPU:

* ``output_hidden_states=None`` falls back to the config's ``output_hidden_states``;
* an all-padding call still returns L + 1 (zero) hidden states;
* ``rope_type: "dynamic"`` rotates positions past ``max_position_embeddings`` with HF's
  NTK-rescaled base (``_compute_dynamic_ntk_parameters`` / ``dynamic_rope_update``).
"""
import pytest
import torch

from distributed_llm_inference.config import ModelSpec
from distributed_llm_inference.models import LlamaBlock
from distributed_llm_inference.ops.reference import build_cos_sin
from distributed_llm_inference.utils.model import stage_from_hf_model

transformers = pytest.importorskip("transformers")

TINY = dict(vocab_size=256, hidden_size=128, intermediate_size=256, num_layers=3, num_heads=4,
            num_kv_heads=2, head_dim=32, rope_theta=10000.0, max_position_embeddings=4096)


def test_output_hidden_states_defaults_to_the_config():
    cfg = {"model_type": "llama", "vocab_size": 256, "hidden_size": 128,
           "intermediate_size": 256, "num_hidden_layers": 3, "num_attention_heads": 4,
           "num_key_value_heads": 2, "output_hidden_states": True}
    spec = ModelSpec.from_hf_config(cfg)
    assert spec.output_hidden_states is True
    assert ModelSpec.from_hf_config(dict(cfg, output_hidden_states=False)).output_hidden_states \
        is False
    assert spec.to_hf_dict()["output_hidden_states"] is True
    x = torch.randn(2, 5, 128, dtype=torch.bfloat16)
    on = LlamaBlock(spec, [0, 1, 2]).init_random(1)
    out = on("s", x)                                  # None -> config: True
    assert len(out) == 2 and len(out[1]) == 4
    assert len(on("t", x, output_hidden_states=False)) == 1   # an explicit False wins
    off = LlamaBlock(spec.replace(output_hidden_states=False), [0, 1, 2]).init_random(1)
    (y,) = off("s", x)
    assert torch.equal(y, out[0])
    torch.testing.assert_close(out[1][0], x)          # the first state is the block's input


def test_all_padding_call_returns_l_plus_1_zero_states():
    spec = ModelSpec(**TINY)
    blk = LlamaBlock(spec, [0, 1, 2]).init_random(2)
    cache = blk.new_cache(num_blocks=16)
    x = torch.randn(2, 4, 128, dtype=torch.bfloat16)
    out, hs = blk("p", x, attention_mask=torch.zeros(2, 4, dtype=torch.long),
                  past_key_value=cache, output_hidden_states=True)
    assert torch.count_nonzero(out) == 0
    assert len(hs) == 3 + 1 and all(h.shape == x.shape and torch.count_nonzero(h) == 0 for h in hs)
    # nothing was cached: a real call afterwards starts at position 0, like a fresh session
    (a,) = blk("p", x, past_key_value=cache)
    (b,) = blk("q", x, past_key_value=cache)
    assert torch.equal(a, b)


def _hf_dynamic(layers=2, factor=2.0, mpe=32, seed=3):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(seed)
    cfg = LlamaConfig(vocab_size=256, hidden_size=128, intermediate_size=256,
                      num_hidden_layers=layers, num_attention_heads=4, num_key_value_heads=2,
                      rms_norm_eps=1e-5, max_position_embeddings=mpe, tie_word_embeddings=False,
                      rope_parameters={"rope_type": "dynamic", "factor": factor,
                                       "rope_theta": 10000.0})
    m = LlamaForCausalLM(cfg).eval()
    m.config._attn_implementation = "eager"
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith(("q_proj.weight", "k_proj.weight")):
                p.mul_(6.0)   # sharp attention, so the rotation (positions) shows in the output
            p.copy_(p.to(torch.bfloat16).float())
    return m


def test_dynamic_rope_table_matches_hf():
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding
    hf = _hf_dynamic()
    rot = LlamaRotaryEmbedding(hf.config)
    for T in (20, 32, 50, 300):   # at / below max_position_embeddings: the base table
        pos = torch.arange(T)[None]
        cos, sin = rot(torch.zeros(1), pos)
        ours = build_cos_sin(32, T, 10000.0, {"rope_type": "dynamic", "factor": 2.0},
                             max_position_embeddings=32, seq_len=T)
        assert torch.allclose(ours[:, :16], cos[0, :, :16], atol=2e-5), T
        assert torch.allclose(ours[:, 16:], sin[0, :, :16], atol=2e-5), T
    plain = build_cos_sin(32, 300, 10000.0, None)
    assert not torch.allclose(ours, plain, atol=1e-3)   # past 32 the base really moved


def test_llama_block_dynamic_rope_matches_hf_past_max_positions():
    """A 48-token prefill (max_position_embeddings 32, factor 2) and one decode step through
    LlamaBlock.forward equal HF's decoder layers with its dynamic rotary embedding."""
    hf = _hf_dynamic()
    stage = stage_from_hf_model(hf, 0, 2)
    blk = stage.block
    assert blk.config.rope_type == "dynamic"
    cache = blk.new_cache(num_blocks=16)
    torch.manual_seed(0)
    B, T = 1, 48
    ids = torch.randint(0, 256, (B, T + 1))
    neg = torch.finfo(torch.float32).min
    with torch.no_grad():
        emb = hf.model.embed_tokens(ids).to(torch.bfloat16).float()

        def hf_layers(h, pos, kv_len):
            q = pos.shape[1]
            allowed = torch.ones(q, kv_len, dtype=torch.bool).tril(kv_len - q)
            mask = torch.zeros(B, 1, q, kv_len).masked_fill(~allowed, neg)
            cos, sin = hf.model.rotary_emb(h, pos)
            for layer in hf.model.layers:
                h = layer(h, attention_mask=mask, position_ids=pos, position_embeddings=(cos, sin))
                h = h[0] if isinstance(h, tuple) else h
            return h

        # HF over the whole 49 tokens, no cache (its base depends on max(position) + 1 = 49)
        ref = hf_layers(emb, torch.arange(T + 1)[None], T + 1)
        x48 = emb[:, :T]
        (ours,) = blk("d", x48.to(torch.bfloat16), past_key_value=cache)
        ref48 = hf_layers(x48, torch.arange(T)[None], T)

        def rel(a):   # error of the block's contribution (the residual stream dominates)
            return ((a.float() - ref48).norm() / (ref48 - x48).norm()).item()
        err = rel(ours)
        assert err < 5e-2, err
        # with the base table (no rescale) the past-32 positions come out clearly different
        plain = LlamaBlock(blk.config.replace(rope_scaling=None), blk.layer_ids)
        plain.load_state_dict(blk.state_dict())
        (p48,) = plain("d", x48.to(torch.bfloat16))
        assert rel(p48) > 2 * err, (rel(p48), err)
        # decode step at position 48: the last row of the 49-token HF run (HF's cache would hold
        # keys rotated with the 48-token base; HF recomputes the whole sequence here, our cache
        # keeps the prefill's keys - the same approximation as HF's own cached generation)
        (d,) = blk("d", emb[:, T:].to(torch.bfloat16), past_key_value=cache)
        err_d = (d[:, 0].float() - ref[:, T]).norm() / (ref[:, T] - emb[:, T]).norm()
        assert err_d.item() < 1e-1, err_d.item()


def test_engine_refuses_dynamic_rope_past_max_positions():
    from distributed_llm_inference.config import CacheConfig, ServeConfig
    from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
    spec = ModelSpec(**dict(TINY, max_position_embeddings=64),
                     rope_scaling=(("factor", 2.0), ("rope_type", "dynamic")), name="dyn")
    cfg = EngineConfig(model="dyn", cache=CacheConfig(num_blocks=32, block_size=32),
                       serve=ServeConfig(max_batch_size=2, max_num_batched_tokens=64,
                                         max_seq_len=128, use_graphs=False))
    with pytest.raises(ValueError, match="dynamic"):
        LLMEngine(spec, device="cpu", cfg=cfg)
