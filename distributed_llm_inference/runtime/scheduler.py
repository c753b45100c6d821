"""Continuous-batching scheduler for a pipeline of stages (runs on the driver, stage 0).

The reference batches independent requests with hivemind's TaskPool (server/backend.py:42;
SURVEY §3.4) and keys sessions by generation_id.  Here the driver keeps M micro-batches in flight
through the N-stage pipeline (M >= N keeps every stage busy; a micro-batch's next step can only be
planned once its sampled tokens came back from the last stage — the loop-carried dependency of
SURVEY §7.4 item 2).  Per micro-batch step it packs:
  * one decode token for every running sequence of the micro-batch,
  * prefill chunks of newly admitted sequences (chunked to ``max_num_batched_tokens``),
and frees the KV blocks of sequences that finished in the previous step.

KV capacity grows on demand, like the reference's per-session cache that grows with every
``update`` (/root/reference/distributed_llm_inference/models/llama/cache.py:103-109): admission
reserves the prompt plus the first sampled token (keeping ``watermark`` blocks free for the
running sequences to grow into), and a sequence takes one more block whenever its next token
crosses a block boundary.  When the pool runs dry the youngest running sequence is preempted:
its blocks are freed (the free rides in the plan being built, so every stage applies it after
every step that used the blocks, in the same order) and it goes back to the front of the queue
for recompute - its prompt and the tokens it already generated are prefilled again, and
sampling (keyed by seed and position) continues exactly where it stopped.  Every stage runs the
identical block-manager call sequence, so stage-local block tables agree without being
communicated.
"""
from __future__ import annotations

import collections
from typing import Callable, Deque, Dict, List, Optional

from .executor import StepPlan
from .sequence import Sequence, SeqStatus


class Scheduler:
    def __init__(self, num_micro_batches: int, max_seqs_per_mb: int, max_tokens_per_step: int,
                 blocks_for: Callable[[int], int], total_blocks: int,
                 eos_token_id: Optional[int] = None, max_seq_len: int = 8192,
                 watermark: Optional[int] = None):
        self.M = max(1, num_micro_batches)
        self.max_seqs = max_seqs_per_mb
        self.max_tokens = max_tokens_per_step
        self.blocks_for = blocks_for
        self.total_blocks = total_blocks
        self.eos = eos_token_id
        self.max_seq_len = max_seq_len
        self.waiting: Deque[Sequence] = collections.deque()
        self.mbs: List[List[Sequence]] = [[] for _ in range(self.M)]
        self.pending_free: List[List[int]] = [[] for _ in range(self.M)]
        self.inflight: List[Optional[StepPlan]] = [None] * self.M
        self.reserved_blocks = 0
        self._reserve: Dict[int, int] = {}
        # tokens per KV block (blocks_for is a ceil-division by it)
        self.block_size = next(n for n in range(1, 1 << 20) if blocks_for(n + 1) > blocks_for(n))
        # blocks admission leaves free for the running sequences' growth
        self.watermark = total_blocks // 100 if watermark is None else int(watermark)
        self._order: Dict[int, int] = {}       # seq_id -> admission counter (youngest = largest)
        self._n_admitted = 0
        # per micro-batch: decode steps every member can take before one needs another block
        self._headroom: List[int] = [0] * self.M
        # per micro-batch: ids preempted while a plan holding them was in flight (their tokens
        # from that plan are stale, even if they were re-admitted meanwhile)
        self._stale: List[set] = [set() for _ in range(self.M)]
        self.preemptions = 0
        self.max_running = 0
        self.step = 0
        self.finished: List[Sequence] = []
        # steady-state decode fast path: while a micro-batch's membership is unchanged and every
        # member is decoding, the next plan differs from the last one only in its tokens
        self._dirty: List[bool] = [True] * self.M
        self._decode_cache: List[Optional[dict]] = [None] * self.M
        self._rows: List[List[Sequence]] = [[] for _ in range(self.M)]  # plan row -> sequence
        # one-step lookahead (single micro-batch pipelines): the next decode step of a clean
        # micro-batch, issued before the in-flight step's tokens reached the host
        self.lookahead: List[Optional[StepPlan]] = [None] * self.M

    # ------------------------------------------------------------------ requests
    def add(self, seq: Sequence) -> None:
        total = len(seq.prompt) + seq.params.max_tokens
        if total > self.max_seq_len:
            raise ValueError(f"prompt + max_tokens = {total} exceeds max_seq_len {self.max_seq_len}")
        if self.blocks_for(total) > self.total_blocks:
            raise ValueError("request can never fit in the KV cache")
        self.waiting.append(seq)

    def abort(self, seq_id: int) -> None:
        # a request still waiting holds no KV and is in no plan: retire it right away, so its
        # future resolves at the next publish even while admission is blocked on KV capacity
        for s in list(self.waiting):
            if s.seq_id == seq_id:
                self.waiting.remove(s)
                s.status = SeqStatus.ABORTED
                s.finish_reason = "abort"
                self.finished.append(s)
        for q in self.mbs:
            for s in list(q):
                if s.seq_id == seq_id:
                    s.status = SeqStatus.ABORTED
                    s.finish_reason = "abort"
                    if s.micro_batch >= 0:
                        self._dirty[s.micro_batch] = True

    def has_work(self) -> bool:
        return (bool(self.waiting) or any(self.mbs) or any(p is not None for p in self.inflight)
                or any(p is not None for p in self.lookahead))

    def num_running(self) -> int:
        return sum(len(m) for m in self.mbs)

    # ------------------------------------------------------------------ planning
    def _admit(self, mb: int, budget: int) -> List[Sequence]:
        admitted = []
        m = self.mbs[mb]
        # balance: fill this micro-batch up to its fair share of (running + waiting)
        share = -(-(self.num_running() + len(self.waiting)) // self.M)
        target = min(self.max_seqs, max(1, share))
        while self.waiting and len(m) < target and budget > 0:
            s = self.waiting[0]
            if s.status == SeqStatus.ABORTED:
                self.waiting.popleft()
                self.finished.append(s)
                continue
            # the tokens to (re)compute and the first sampled one; a preempted sequence recomputes
            # its prompt and everything it generated
            need = self.blocks_for(s.total_len + 1)
            room = self.total_blocks - (self.watermark if self.num_running() else 0)
            if self.reserved_blocks + need > room:
                break
            self.waiting.popleft()
            self.reserved_blocks += need
            self._reserve[s.seq_id] = need
            self._n_admitted += 1
            self._order[s.seq_id] = self._n_admitted
            s.status = SeqStatus.RUNNING
            s.micro_batch = mb
            m.append(s)
            admitted.append(s)
            self._dirty[mb] = True
            budget -= min(s.total_len - s.num_computed, budget)
        self.max_running = max(self.max_running, self.num_running())
        return admitted

    # ------------------------------------------------------------------ KV growth / preemption
    def _preempt(self, mb: int, v: Sequence) -> None:
        """Free ``v``'s blocks (in the plan being built for ``mb``) and queue it for recompute."""
        mv = v.micro_batch
        self.mbs[mv].remove(v)
        self._dirty[mv] = True
        if self.inflight[mv] is not None or self.lookahead[mv] is not None:
            self._stale[mv].add(v.seq_id)
        self.reserved_blocks -= self._reserve.pop(v.seq_id, 0)
        self._order.pop(v.seq_id, None)
        self.pending_free[mb].append(v.seq_id)
        v.status = SeqStatus.WAITING
        v.num_computed = 0
        v.micro_batch = -1
        self.waiting.appendleft(v)
        self.preemptions += 1

    def _grow(self, mb: int, rows: List[tuple]) -> None:
        """Reserve the blocks ``rows`` ((sequence, tokens this step)) need; when the pool is
        short, preempt the youngest running sequence (possibly the one asking) until it fits."""
        for s, take in rows:
            if s.status is not SeqStatus.RUNNING:
                continue   # preempted by an earlier row of this pass
            need = self.blocks_for(s.num_computed + take) - self._reserve[s.seq_id]
            while need > 0:
                if self.reserved_blocks + need <= self.total_blocks:
                    self._reserve[s.seq_id] += need
                    self.reserved_blocks += need
                    break
                victim = max((x for q in self.mbs for x in q), key=lambda x: self._order[x.seq_id])
                self._preempt(mb, victim)
                if victim is s:
                    break

    @staticmethod
    def _decoding(s: Sequence) -> bool:
        """Only the last sampled token is pending (a preempted sequence recomputing its outputs,
        like one prefilling its prompt, is not)."""
        return s.num_computed >= max(len(s.prompt), s.total_len - 1)

    def _set_headroom(self, mb: int) -> None:
        bs = self.block_size
        self._headroom[mb] = min((self._reserve[s.seq_id] * bs - s.num_computed
                                  for s in self.mbs[mb]), default=0)

    def plan(self, mb: int) -> Optional[StepPlan]:
        """Next step for micro-batch ``mb`` (None if it has nothing to do)."""
        assert self.inflight[mb] is None, "micro-batch still in flight"
        m = self.mbs[mb]
        # drop aborted sequences
        for s in [s for s in m if s.status == SeqStatus.ABORTED]:
            self._retire(mb, s)
        if not self._dirty[mb] and m and self._headroom[mb] < 1:
            # a clean micro-batch whose next token crosses a block boundary for some member
            self._grow(mb, [(s, 1) for s in m])
            if not self._dirty[mb]:
                self._set_headroom(mb)
        if self._dirty[mb]:
            decode_n = sum(1 for s in m if self._decoding(s))
        else:
            decode_n = len(m)  # a clean micro-batch is all-decode (see _decode_plan)
        self._admit(mb, self.max_tokens - decode_n)
        if not self._dirty[mb] and m:
            return self._decode_plan(mb)
        budget = self.max_tokens - decode_n
        work = []
        for s in m:
            pend = s.pending_tokens()
            if self._decoding(s):
                take = 1  # decode: the last sampled token
                pend = pend[-1:]
            else:       # prefill chunk (a prompt, or a preempted sequence's recompute)
                take = min(len(pend), budget)
                if take <= 0:
                    continue
                budget -= take
                pend = pend[:take]
            work.append((s, take, pend))
        self._grow(mb, [(s, take) for s, take, _ in work])
        seq_ids, q_lens, tokens, sample_rows = [], [], [], []
        temps, topk, topp, seeds, spos = [], [], [], [], []
        for s, take, pend in work:
            if s.status is not SeqStatus.RUNNING:
                continue   # preempted to make room
            row = len(seq_ids)
            seq_ids.append(s.seq_id)
            q_lens.append(take)
            tokens.extend(pend)
            if s.num_computed + take >= s.total_len:  # reaches the end of known tokens: sample
                sample_rows.append(row)
                temps.append(float(s.params.temperature))
                topk.append(int(s.params.top_k))
                topp.append(float(s.params.top_p))
                seeds.append(int(s.seed))
                spos.append(s.num_computed + take)   # the sampled token's position
        free_ids = self.pending_free[mb]
        self.pending_free[mb] = []
        if not seq_ids and not free_ids:
            return None
        plan = StepPlan(step=self.step, mb=mb, seq_ids=seq_ids, q_lens=q_lens, free_ids=free_ids,
                        sample_rows=sample_rows, temperature=temps, top_k=topk, top_p=topp,
                        seeds=seeds, sample_pos=spos, tokens=tokens)
        self.step += 1
        # the tokens are (about to be) in the cache on every stage
        byid = {s.seq_id: s for s in m}
        rows = [byid[sid] for sid in seq_ids]
        for s, q in zip(rows, q_lens):
            s.num_computed += q
        self._rows[mb] = rows
        self.inflight[mb] = plan if seq_ids else None
        self._set_headroom(mb)
        # cache the all-decode layout; it stays valid until the membership changes
        if seq_ids and len(rows) == len(m) and all(q == 1 for q in q_lens) \
                and len(sample_rows) == len(rows):
            self._decode_cache[mb] = dict(seq_ids=seq_ids, q_lens=q_lens, sample_rows=sample_rows,
                                          temperature=temps, top_k=topk, top_p=topp, seeds=seeds)
            self._dirty[mb] = False
        else:
            self._decode_cache[mb] = None
            self._dirty[mb] = True
        return plan

    def plan_lookahead(self, mb: int) -> Optional[StepPlan]:
        """The step after the in-flight one, planned BEFORE its tokens are known (their values
        stay on the device: stage 0 reads them from the sampler output).  Only for a clean,
        all-decode micro-batch with nobody waiting for admission and no sequence that could
        reach max_tokens within the two steps; an EOS inside the window costs one wasted token.
        Returns None when any condition fails (the caller then plans normally)."""
        if (self.inflight[mb] is None or self.lookahead[mb] is not None or self._dirty[mb]
                or self.waiting or self.pending_free[mb] or not self.mbs[mb]):
            return None
        rows = self._rows[mb]
        if len(rows) != len(self.mbs[mb]) or self._headroom[mb] < 1:
            return None   # (a member needs another KV block first: plan it normally)
        for s in rows:
            if s.status is not SeqStatus.RUNNING or len(s.output) + 2 > s.params.max_tokens:
                return None
        c = self._decode_cache[mb]
        for s in rows:
            s.num_computed += 1
        plan = StepPlan(step=self.step, mb=mb, seq_ids=c["seq_ids"], q_lens=c["q_lens"],
                        free_ids=[], sample_rows=c["sample_rows"], temperature=c["temperature"],
                        top_k=c["top_k"], top_p=c["top_p"], seeds=c["seeds"],
                        sample_pos=[s.num_computed for s in rows], tokens=None)
        self.step += 1
        self.lookahead[mb] = plan
        self._headroom[mb] -= 1
        return plan

    def _decode_plan(self, mb: int) -> StepPlan:
        """Plan of a clean micro-batch: same rows as last step, one new token each."""
        c = self._decode_cache[mb]
        rows = self._rows[mb]
        tokens = [s.output[-1] for s in rows]
        for s in rows:
            s.num_computed += 1
        free_ids = self.pending_free[mb]
        self.pending_free[mb] = []
        plan = StepPlan(step=self.step, mb=mb, seq_ids=c["seq_ids"], q_lens=c["q_lens"],
                        free_ids=free_ids, sample_rows=c["sample_rows"],
                        temperature=c["temperature"], top_k=c["top_k"], top_p=c["top_p"],
                        seeds=c["seeds"], sample_pos=[s.num_computed for s in rows],
                        tokens=tokens)
        self.step += 1
        self.inflight[mb] = plan
        self._headroom[mb] -= 1
        return plan

    # ------------------------------------------------------------------ results
    def _retire(self, mb: int, s: Sequence) -> None:
        self.mbs[mb].remove(s)
        self._dirty[mb] = True
        self.pending_free[mb].append(s.seq_id)
        self.reserved_blocks -= self._reserve.pop(s.seq_id, 0)
        self._order.pop(s.seq_id, None)
        self.finished.append(s)

    def on_tokens(self, mb: int, tokens: List[int], now: Optional[float] = None) -> List[Sequence]:
        """Sampled tokens for the in-flight step of ``mb`` (one per sample row, in order)."""
        plan = self.inflight[mb]
        self.inflight[mb] = self.lookahead[mb]  # the lookahead step (if any) is now the oldest
        self.lookahead[mb] = None
        if plan is None:
            return []
        rows = self._rows[mb]
        stale = self._stale[mb]
        done = []
        for row, tok in zip(plan.sample_rows, tokens):
            s = rows[row]
            if s.status is not SeqStatus.RUNNING:  # finished / aborted / preempted meanwhile
                continue
            if s.seq_id in stale:   # preempted (and re-admitted) since this plan was issued
                continue
            if s.append_token(tok, self.eos, now):
                done.append(s)
        for s in done:
            self._retire(mb, s)
        if self.inflight[mb] is None:
            stale.clear()
        return done

    def pop_finished(self) -> List[Sequence]:
        out, self.finished = self.finished, []
        return out
