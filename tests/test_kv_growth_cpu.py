"""On-demand KV growth with preemption, on CPU.

The reference's per-session cache grows with every ``update`` and never commits capacity up
front (/root/reference/distributed_llm_inference/models/llama/cache.py:103-109).  The scheduler
admits a sequence with its prompt (+ the first sampled token), takes another block when a token
crosses a block boundary, and when the pool runs dry preempts the youngest running sequence
(blocks freed on every stage in the same order, recomputed later).  A pool sized for N worst-case
reservations then runs 2N sequences at once, and every token equals an unconstrained run."""
import pytest

from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
from distributed_llm_inference.runtime.scheduler import Scheduler
from distributed_llm_inference.runtime.sequence import SamplingParams, Sequence, SeqStatus

SPEC = ModelSpec(name="t", vocab_size=300, hidden_size=128, intermediate_size=256, num_layers=4,
                 num_heads=4, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                 max_position_embeddings=4096)
BS = 32
PROMPTS = [list(range(3 + i, 23 + i + (i % 3) * 4)) for i in range(8)]   # 20-28 tokens each
MAX_TOKENS = 40                                                           # worst case <= 68 -> 3 blocks


def _engine(num_blocks, pp=1, mbs=0, seqs=8):
    cfg = EngineConfig(model="t", pp=pp, seed=3,
                       cache=CacheConfig(num_blocks=num_blocks, block_size=BS, max_chunk=64),
                       serve=ServeConfig(max_batch_size=seqs, max_num_batched_tokens=256,
                                         num_micro_batches=mbs, max_seq_len=256,
                                         use_graphs=False))
    return LLMEngine(SPEC, cfg=cfg)


def _scheduler(eng):
    return eng.pipeline.sched


@pytest.mark.parametrize("pp,mbs", [(1, 0), (2, 3)])
def test_pool_for_n_worst_cases_runs_2n_sequences(pp, mbs):
    params = SamplingParams(max_tokens=MAX_TOKENS, ignore_eos=True)
    worst = -(-(max(len(p) for p in PROMPTS) + MAX_TOKENS) // BS)   # blocks per sequence
    N = len(PROMPTS) // 2
    ref = [s.output for s in _engine(256, pp, mbs).generate(PROMPTS, params)]
    eng = _engine(N * worst, pp, mbs)
    out = eng.generate(PROMPTS, params)
    sched = _scheduler(eng)
    assert sched.max_running >= 2 * N, sched.max_running     # all 2N admitted at once
    assert sched.preemptions > 0                             # ... and the pool ran dry
    assert [s.output for s in out] == ref
    assert all(len(s.output) == MAX_TOKENS and s.finish_reason == "length" for s in out)
    assert sched.reserved_blocks == 0 and not sched._reserve


def test_sampled_sequences_survive_preemption():
    """Temperature / top-k sampling is keyed by (seed, position): a preempted sequence that is
    recomputed samples the same tokens it would have without the preemption."""
    params = [SamplingParams(max_tokens=MAX_TOKENS, temperature=0.9, top_k=40, seed=100 + i,
                             ignore_eos=True) for i in range(len(PROMPTS))]
    def run(nb):
        eng = _engine(nb)
        seqs = [Sequence(list(p), sp) for p, sp in zip(PROMPTS, params)]
        for s in seqs:
            eng.pipeline.sched.add(s)
        done = {s.seq_id: s for s in eng.pipeline.run_until_done()}
        return [done[s.seq_id].output for s in seqs], eng.pipeline.sched.preemptions
    ref, p0 = run(256)
    out, p1 = run(10)
    assert p0 == 0 and p1 > 0
    assert out == ref


def test_scheduler_grows_by_blocks_and_preempts_the_youngest():
    """Bookkeeping on the scheduler alone: admission takes prompt + 1 token, a decode step that
    crosses a block boundary takes one block, and a dry pool preempts the most recently admitted
    sequence, whose free rides in the next plan and which is requeued first."""
    bs = 4
    sch = Scheduler(1, 8, 64, lambda n: -(-n // bs), total_blocks=5, watermark=0)
    a = Sequence([1, 2, 3], SamplingParams(max_tokens=8, ignore_eos=True))
    b = Sequence([4, 5, 6], SamplingParams(max_tokens=8, ignore_eos=True))
    sch.add(a)
    sch.add(b)
    p = sch.plan(0)
    assert p.seq_ids == [a.seq_id, b.seq_id] and sch._reserve == {a.seq_id: 1, b.seq_id: 1}
    sch.on_tokens(0, [10, 20])
    # next tokens (position 3) fit the first block; the step after crosses into a second block
    p = sch.plan(0)
    assert sch.reserved_blocks == 2
    sch.on_tokens(0, [11, 21])
    p = sch.plan(0)   # position 4 -> second block each
    assert sch._reserve == {a.seq_id: 2, b.seq_id: 2} and sch.reserved_blocks == 4
    sch.on_tokens(0, [12, 22])
    for _ in range(3):   # positions 5-7 stay in the second block
        sch.plan(0)
        sch.on_tokens(0, [13, 23])
    # position 8 -> third block each: 6 > 5 blocks; b (the younger) is preempted
    p = sch.plan(0)
    assert p.seq_ids == [a.seq_id] and p.free_ids == [b.seq_id]
    assert b.status is SeqStatus.WAITING and b.num_computed == 0 and sch.waiting[0] is b
    assert sch._reserve == {a.seq_id: 3} and sch.preemptions == 1
    sch.on_tokens(0, [14])
    # b comes back as soon as it fits: it recomputes its prompt and its 6 outputs in one chunk
    while b.status is not SeqStatus.RUNNING:
        p = sch.plan(0)
        if b.status is SeqStatus.RUNNING:   # the plan that re-admitted b
            row = p.seq_ids.index(b.seq_id)
            assert p.q_lens[row] == len(b.prompt) + 6 == b.num_computed
            assert row in p.sample_rows
        sch.on_tokens(0, [15] * len(p.sample_rows))
    assert b.output[:6] == [20, 21, 22, 23, 23, 23] and len(b.output) == 7
