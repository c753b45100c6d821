"""KV reservations are atomic: a call that is rejected -- pool exhausted, bad
4-D mask, failing forward -- leaves every session exactly as it was, and one oversized request in
a server batch fails alone instead of poisoning the other sessions of that batch.

Reference: per-session state in /root/reference/distributed_llm_inference/models/llama/
cache.py:78-109 (there a failure inside ``update`` also leaves the dicts half-grown)."""
import pytest
import torch

from distributed_llm_inference.config import ModelSpec
from distributed_llm_inference.models import LlamaBlock
from distributed_llm_inference.server.backend import BatchTensorDescriptor, InferenceBackend

SPEC = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=4,
                 num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                 max_position_embeddings=4096)


def _close(a, b):
    return torch.allclose(a.float(), b.float(), atol=3e-2, rtol=3e-2)


def test_block_manager_rollback_restores_allocation_order():
    from distributed_llm_inference import _runtime  # built by the conftest fixture
    m = _runtime.BlockManager(8, 32)
    assert m.append_batch([0, 1], [40, 10])
    tables = (m.block_table(0), m.block_table(1))
    free = m.num_free_blocks
    assert m.append_batch([0, 1], [70, 1])       # grows 0 by 3 blocks
    m.rollback_batch([0, 1], [70, 1])
    assert (m.block_table(0), m.block_table(1)) == tables and m.num_free_blocks == free
    assert m.length(0) == 40 and m.length(1) == 10
    # re-appending hands out the same physical blocks as the undone reservation did
    assert m.append(0, 70)
    t0 = m.block_table(0)
    m.rollback(0, 70)
    assert m.append(0, 70) and m.block_table(0) == t0
    # a sequence rolled back to zero tokens is gone
    assert m.append(5, 3)
    m.rollback(5, 3)
    assert not m.has_sequence(5)
    with pytest.raises(ValueError):
        m.rollback(1, 11)
    # append_batch that does not fit changes nothing
    before = m.num_free_blocks
    assert not m.append_batch([0, 7], [1, 10_000])
    assert m.num_free_blocks == before and not m.has_sequence(7)


def test_block_forward_rejections_leave_session_unchanged():
    blk = LlamaBlock(SPEC, [0, 1]).init_random(3)
    cache = blk.new_cache(num_blocks=4, block_size=64)
    x = torch.randn(1, 10, 128, dtype=torch.bfloat16)
    blk("s", x, past_key_value=cache)
    assert cache.get_seq_length(0, "s") == 10 and cache.get_seen_tokens("s") == 10
    free = cache.pool.manager.num_free_blocks
    # a 4-D mask whose key length is short of cached + new tokens
    bad = torch.zeros(1, 1, 2, 11)
    with pytest.raises(ValueError):
        blk("s", torch.randn(1, 2, 128, dtype=torch.bfloat16), attention_mask=bad,
            past_key_value=cache)
    assert cache.get_seq_length(0, "s") == 10 and cache.get_seen_tokens("s") == 10
    assert cache.pool.manager.num_free_blocks == free
    # malformed position ids
    with pytest.raises(ValueError):
        blk("s", torch.randn(1, 2, 128, dtype=torch.bfloat16), position_ids=torch.arange(1)[None],
            past_key_value=cache)
    assert cache.get_seq_length(0, "s") == 10
    # pool exhaustion: nothing reserved, and a session created by the call disappears again
    with pytest.raises(MemoryError):
        blk("s", torch.randn(1, 300, 128, dtype=torch.bfloat16), past_key_value=cache)
    with pytest.raises(MemoryError):
        blk("new", torch.randn(1, 300, 128, dtype=torch.bfloat16), past_key_value=cache)
    assert cache.get_seq_length(0, "s") == 10 and not cache.has_session("new")
    assert cache.pool.manager.num_free_blocks == free
    # the session continues exactly like an untouched one
    ref = LlamaBlock(SPEC, [0, 1]).init_random(3)
    rc = ref.new_cache(num_blocks=4, block_size=64)
    ref("s", x, past_key_value=rc)
    d = torch.randn(1, 1, 128, dtype=torch.bfloat16)
    assert _close(blk("s", d, past_key_value=cache)[0], ref("s", d, past_key_value=rc)[0])


def test_block_forward_failure_inside_layers_rolls_back(monkeypatch):
    blk = LlamaBlock(SPEC, [0, 1]).init_random(3)
    cache = blk.new_cache(num_blocks=4, block_size=64)
    blk("s", torch.randn(1, 7, 128, dtype=torch.bfloat16), past_key_value=cache)
    free = cache.pool.manager.num_free_blocks

    def boom(*a, **k):
        raise RuntimeError("kernel failed")
    monkeypatch.setattr(blk, "forward_tokens", boom)
    with pytest.raises(RuntimeError):
        blk("s", torch.randn(1, 70, 128, dtype=torch.bfloat16), past_key_value=cache)
    assert cache.get_seq_length(0, "s") == 7 and cache.get_seen_tokens("s") == 7
    assert cache.pool.manager.num_free_blocks == free


def test_backend_overflowing_session_fails_alone():
    # 3 blocks of 64 tokens: the __schema__ probe runs and is closed at construction
    blk = LlamaBlock(SPEC, [0, 1]).init_random(4)
    be = InferenceBackend("blk", blk, args_schema=(BatchTensorDescriptor((1, 128)),),
                          max_batch_size=1024, pool_timeout=0.1, num_blocks=3)
    ref = LlamaBlock(SPEC, [0, 1]).init_random(4)
    rc = ref.new_cache(num_blocks=8)
    xa = torch.randn(1, 20, 128, dtype=torch.bfloat16)
    xb = torch.randn(1, 150, 128, dtype=torch.bfloat16)     # needs 3 blocks: only 2 left
    fa = be.submit(xa, generation_id="a")
    fb = be.submit(xb, generation_id="b")
    assert _close(fa.result(20)[0], ref("a", xa, past_key_value=rc)[0])
    with pytest.raises(MemoryError):
        fb.result(20)
    assert not be.cache.has_session("b")
    assert be.cache.get_seq_length(0, "a") == 20
    # session a keeps decoding exactly like an untouched session
    for _ in range(3):
        d = torch.randn(1, 1, 128, dtype=torch.bfloat16)
        assert _close(be.submit(d, generation_id="a").result(20)[0],
                      ref("a", d, past_key_value=rc)[0])
    assert be.cache.get_seq_length(0, "a") == 23
    # freeing a makes room, and b's rejected request now succeeds unchanged
    be.close_session("a")
    (yb,) = be.submit(xb, generation_id="b").result(20)
    rc2 = ref.new_cache(num_blocks=8)
    assert _close(yb, ref("b", xb, past_key_value=rc2)[0])
    be.shutdown()


def test_backend_two_steps_of_one_session_in_one_batch_run_in_order():
    blk = LlamaBlock(SPEC, [0, 1]).init_random(5)
    be = InferenceBackend("blk", blk, args_schema=(BatchTensorDescriptor((1, 128)),),
                          max_batch_size=64, pool_timeout=0.2, num_blocks=16)
    ref = LlamaBlock(SPEC, [0, 1]).init_random(5)
    rc = ref.new_cache(num_blocks=16)
    steps = [torch.randn(1, n, 128, dtype=torch.bfloat16) for n in (6, 1, 1)]
    futs = [be.submit(x, generation_id="a") for x in steps]
    other = torch.randn(1, 4, 128, dtype=torch.bfloat16)
    fo = be.submit(other, generation_id="o")
    for x, f in zip(steps, futs):
        assert _close(f.result(20)[0], ref("a", x, past_key_value=rc)[0])
    assert _close(fo.result(20)[0], ref("o", other, past_key_value=rc)[0])
    assert be.cache.get_seq_length(0, "a") == 8
    be.shutdown()
