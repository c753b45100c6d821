"""Request / sequence state and sampling parameters."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence as Seq


@dataclass
class SamplingParams:
    """Per-request decoding parameters (temperature 0 = greedy)."""

    max_tokens: int = 16
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    seed: Optional[int] = None
    stop_token_ids: Optional[List[int]] = None
    ignore_eos: bool = False
    min_tokens: int = 0

    def __post_init__(self):
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not (0 < self.top_p <= 1.0):
            raise ValueError("top_p must be in (0, 1]")


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2
    ABORTED = 3


_ids = itertools.count()


@dataclass
class Sequence:
    prompt: List[int]
    params: SamplingParams
    seq_id: int = field(default_factory=lambda: next(_ids))
    request_id: Optional[str] = None
    output: List[int] = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    num_computed: int = 0        # tokens whose KV is in the cache (prompt + fed-back outputs)
    micro_batch: int = -1
    finish_reason: Optional[str] = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    token_times: List[float] = field(default_factory=list)
    seed: int = 0

    def __post_init__(self):
        if not self.prompt:
            raise ValueError("empty prompt")
        self.seed = self.params.seed if self.params.seed is not None else (self.seq_id * 7919 + 17)

    @property
    def all_tokens(self) -> List[int]:
        return self.prompt + self.output

    @property
    def total_len(self) -> int:
        return len(self.prompt) + len(self.output)

    def pending_tokens(self) -> List[int]:
        """Tokens not yet in the KV cache (prompt remainder, or the last sampled token)."""
        return self.all_tokens[self.num_computed:]

    def is_finished(self) -> bool:
        return self.status in (SeqStatus.FINISHED, SeqStatus.ABORTED)

    def append_token(self, tok: int, eos_token_id: Optional[int], now: Optional[float] = None) -> bool:
        """Record a sampled token; returns True if the sequence is now finished."""
        now = time.perf_counter() if now is None else now
        if self.first_token_time is None:
            self.first_token_time = now
        self.token_times.append(now)
        self.output.append(int(tok))
        p = self.params
        n = len(self.output)
        if n >= p.max_tokens:
            self.status, self.finish_reason = SeqStatus.FINISHED, "length"
        elif n >= p.min_tokens and not p.ignore_eos and (
                (eos_token_id is not None and tok == eos_token_id)
                or (p.stop_token_ids and tok in p.stop_token_ids)):
            self.status, self.finish_reason = SeqStatus.FINISHED, "stop"
        return self.is_finished()
