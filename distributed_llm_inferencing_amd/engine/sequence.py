"""Requests, sequences and sampling parameters.

Defaults reproduce the reference worker's ``generate`` call exactly
(``worker/app.py:297-305``): do_sample with temperature 0.8, top_k 50, top_p 0.95, one
return sequence, ``max_length`` = 100 tokens *including* the prompt
(``master/dashboard/views.py:351``).
"""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class SamplingParams:
    max_length: Optional[int] = 100        # prompt + generated (HF semantics)
    max_new_tokens: Optional[int] = None   # overrides max_length when set
    temperature: float = 0.8
    top_k: int = 50
    top_p: float = 0.95
    do_sample: bool = True
    seed: Optional[int] = None
    ignore_eos: bool = False
    stop_token_ids: List[int] = field(default_factory=list)
    timeout_s: Optional[float] = None      # per-request deadline (reference 'timeout', 60 s)

    def effective_temperature(self) -> float:
        return self.temperature if self.do_sample else 0.0

    def budget(self, prompt_len: int) -> int:
        """Number of tokens to generate at most."""
        if self.max_new_tokens is not None:
            return max(0, int(self.max_new_tokens))
        if self.max_length is None:
            return 16
        return max(0, int(self.max_length) - prompt_len)


class SeqState(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2
    PREFILLING = 3          # chunked prefill in progress (KV blocks held, not decoding yet)


@dataclass(eq=False)          # identity semantics: list.remove / `in` must not compare fields
class Sequence:
    seq_id: int
    request_id: str
    prompt_ids: List[int]
    params: SamplingParams
    output_ids: List[int] = field(default_factory=list)
    state: SeqState = SeqState.WAITING
    microbatch: int = 0
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    finish_reason: Optional[str] = None
    seed: int = 0
    num_preemptions: int = 0
    preempt_step: int = -1      # scheduler step id of the last preemption
    num_prefilled: int = 0  # tokens of all_ids() whose KV a scheduled prefill chunk writes

    @property
    def prompt_len(self) -> int:
        return len(self.prompt_ids)

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    @property
    def deadline(self) -> Optional[float]:
        if self.params.timeout_s is None:
            return None
        return self.arrival + float(self.params.timeout_s)


@dataclass
class RequestOutput:
    request_id: str
    prompt_ids: List[int]
    output_ids: List[int]
    finish_reason: str
    latency_s: float
    ttft_s: Optional[float]
    text: Optional[str] = None
    tokenizer: object = field(default=None, repr=False, compare=False)

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    def resolve_text(self) -> Optional[str]:
        """prompt + continuation detokenised (skip_special_tokens), computed on first use
        (off the engine's step loop)."""
        if self.text is None and self.tokenizer is not None:
            self.text = self.tokenizer.decode(self.all_ids, skip_special_tokens=True)
        return self.text


def row_seed(seq_seed: int, index: int) -> int:
    """64-bit per-(request, output position) sampling seed (splitmix64)."""
    z = (seq_seed * 0x9E3779B97F4A7C15 + index + 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    z = z ^ (z >> 31)
    return z - (1 << 64) if z >= (1 << 63) else z
