"""Per-request state of the LLM worker (the reference's `llama_client_slot`,
grpc-server.cpp:188-385): token history, KV block table, sampling parameters, stop handling,
incremental detokenisation with UTF-8 / stop-string hold-back, and timings."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field

from ..ops.sampling import SamplingParams

_ids = itertools.count(1)


def _utf8_incomplete_tail(b: bytes) -> int:
    """Number of trailing bytes that start a UTF-8 character not yet complete (0 if the tail is complete)."""
    n = len(b)
    for k in range(1, min(4, n) + 1):
        c = b[n - k]
        if c & 0xC0 == 0x80:
            continue  # continuation byte: look further back for the lead byte
        need = 2 if c & 0xE0 == 0xC0 else 3 if c & 0xF0 == 0xE0 else 4 if c & 0xF8 == 0xF0 else 1
        return k if need > k else 0
    return 0


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


@dataclass
class Request:
    prompt_ids: list
    params: SamplingParams = field(default_factory=SamplingParams)
    max_tokens: int = 128
    stop: list = field(default_factory=list)
    stop_token_ids: list = field(default_factory=list)
    embedding: bool = False
    grammar: object = None  # engine.grammar.GrammarMatcher factory (optional)
    rid: int = field(default_factory=lambda: next(_ids))
    arrival: float = field(default_factory=time.perf_counter)
    cache_prompt: bool = True
    # multimodal: (prompt position, fp32 [n, hidden] device tensor) spans whose input embeddings
    # replace the placeholder tokens there (llava image embeddings, grpc-server.cpp:1455-1520)
    mm_embeds: list = field(default_factory=list)
    n_draft: int = 0  # speculative decoding: max draft tokens per step for this request (0 = engine's)


@dataclass
class StepOutput:
    rid: int
    text: str = ""
    token_ids: list = field(default_factory=list)
    logprobs: list = field(default_factory=list)
    finished: bool = False
    finish_reason: str | None = None
    prompt_tokens: int = 0
    completion_tokens: int = 0
    cached_tokens: int = 0
    t_prompt_ms: float = 0.0
    t_gen_ms: float = 0.0
    ttft_ms: float = 0.0
    embedding: list | None = None


class Sequence:
    def __init__(self, req: Request, tokenizer):
        self.req = req
        self.rid = req.rid
        self.params = req.params
        self.prompt_ids = list(req.prompt_ids)
        self.output_ids: list[int] = []
        # tokens sampled on the GPU by launched steps whose results the host has not read yet
        # (engine overlap mode): they count towards the sequence length / KV position but their ids
        # are only known after the step's async device->host copy lands (engine._process_inflight)
        self.n_pending = 0
        self.logprobs: list[float] = []
        self.status = Status.WAITING
        self.blocks: list[int] = []
        self.num_computed = 0
        self.num_cached = 0  # tokens served from the prefix cache
        self.block_hashes: list[bytes] = []
        self.tok = tokenizer
        self.t_arrival = req.arrival
        self.t_first_sched: float | None = None
        self.t_first_token: float | None = None
        self.t_finish: float | None = None
        self.finish_reason: str | None = None
        self.grammar = req.grammar() if callable(req.grammar) else req.grammar
        self.mirostat_mu = 2 * self.params.mirostat_tau
        # detokenisation state
        self._prefix_off = 0
        self._read_off = 0
        self._held = ""
        self._pbytes = b""  # byte-level detokenisation: bytes of an incomplete trailing UTF-8 character
        self.emitted_text = ""
        self._pending_ids: list[int] = []
        self._pending_lp: list[float] = []
        self.overlap_static = None  # engine cache: may this request's rows run in the overlap pipeline

    # ---------------------------------------------------------------- token bookkeeping
    @property
    def all_ids(self) -> list[int]:
        return self.prompt_ids + self.output_ids

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids) + self.n_pending

    @property
    def known_len(self) -> int:
        """Tokens whose ids are on the host (excludes in-flight samples)."""
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def prefill_target(self) -> int:
        """KV length to reach before decoding: the whole prompt (its last row yields the first
        token's logits), or all but the newest token when resuming after a preemption."""
        return self.total_len - 1 if (self.output_ids or self.n_pending) else self.total_len

    @property
    def in_decode(self) -> bool:
        return bool(self.output_ids or self.n_pending) and self.num_computed == self.total_len - 1

    @property
    def n_generated(self) -> int:
        return len(self.output_ids) + self.n_pending

    def remaining_prefill(self) -> int:
        return self.prefill_target - self.num_computed

    # ---------------------------------------------------------------- detokenisation
    def append_token(self, tid: int, logprob: float | None):
        self.output_ids.append(int(tid))
        if logprob is not None:
            self.logprobs.append(float(logprob))
        self._pending_ids.append(int(tid))
        if logprob is not None:
            self._pending_lp.append(float(logprob))

    def pop_output(self):
        """Drop the newest output token (an EOS is not part of the visible output)."""
        self.output_ids.pop()
        if self._pending_ids:
            self._pending_ids.pop()

    def _decode_new(self, final: bool = False) -> str:
        sb = getattr(self.tok, "stream_bytes", None)
        if sb is not None:
            return self._decode_bytes(sb())
        ids = self.output_ids
        prefix = self.tok.decode(ids[self._prefix_off:self._read_off])
        full = self.tok.decode(ids[self._prefix_off:])
        if full.endswith("�") and not final:
            return ""  # incomplete UTF-8 sequence: hold back (grpc-server.cpp:1069-1190 partial check)
        new = full[len(prefix):]
        self._prefix_off = max(0, len(ids) - 6) if len(ids) > 6 else self._prefix_off
        self._read_off = len(ids)
        if self._prefix_off > self._read_off:
            self._prefix_off = self._read_off
        return new

    def _decode_bytes(self, table: list) -> str:
        """Byte-level streaming detokenisation: append each new token's bytes, emit the longest valid UTF-8 prefix
        and hold back an incomplete trailing character (grpc-server.cpp:1069-1190 partial-UTF-8 check)."""
        ids = self.output_ids
        new = ids[self._read_off:]
        self._read_off = len(ids)
        if not new:
            return ""
        n = len(table)
        buf = self._pbytes + b"".join([table[i] if 0 <= i < n else b"" for i in new])
        k = _utf8_incomplete_tail(buf)
        self._pbytes = buf[len(buf) - k:] if k else b""
        return (buf[:len(buf) - k] if k else buf).decode("utf-8", errors="replace")

    def flush_text(self, final: bool = False) -> tuple[str, bool]:
        """Returns (text to emit, stop_string_hit)."""
        self._held += self._decode_new(final)
        if final and self._pbytes:  # a generation cut mid-character: emit the partial bytes as U+FFFD
            self._held += self._pbytes.decode("utf-8", errors="replace")
            self._pbytes = b""
        stops = [s for s in self.req.stop if s]
        for s in stops:
            i = self._held.find(s)
            if i >= 0:
                out = self._held[:i]
                self._held = ""
                self.emitted_text += out
                return out, True
        if final or not stops:
            out, self._held = self._held, ""
            self.emitted_text += out
            return out, False
        # keep the longest suffix that is a prefix of a stop string
        keep = 0
        for s in stops:
            for k in range(min(len(s) - 1, len(self._held)), 0, -1):
                if self._held.endswith(s[:k]):
                    keep = max(keep, k)
                    break
        out = self._held[:len(self._held) - keep] if keep else self._held
        self._held = self._held[len(self._held) - keep:] if keep else ""
        self.emitted_text += out
        return out, False

    def take_pending(self):
        ids, lp = self._pending_ids, self._pending_lp
        self._pending_ids, self._pending_lp = [], []
        return ids, lp
