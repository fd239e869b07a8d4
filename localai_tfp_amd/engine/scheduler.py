"""Iteration-level continuous-batching scheduler with chunked prefill (D1 of SURVEY §2.5).

Each `schedule()` call builds one forward step, in the spirit of the reference's `update_slots`
(grpc-server.cpp:1639-2074) but over a paged cache instead of fixed slots:
  1. every running sequence in the decode phase contributes exactly one token;
  2. sequences still prefilling (and then new arrivals, FIFO) fill the remaining token budget with
     prompt chunks (chunked prefill), reusing cached prefix blocks first;
  3. if the pool cannot grow a decode sequence, the most recently admitted sequence is preempted
     (its blocks freed, recomputed later) — the paged equivalent of the reference's
     "KV full -> halve the batch and retry" (grpc-server.cpp:2004-2019).
"""
from __future__ import annotations

import collections
import time
from dataclasses import dataclass, field

from .sequence import Sequence, Status


@dataclass(slots=True)
class ScheduledSeq:
    seq: Sequence
    start: int  # first token index computed this step
    n: int  # tokens computed this step
    sample: bool  # whether this step produces a token for the sequence


@dataclass
class SchedulerOutput:
    decode: list = field(default_factory=list)  # [ScheduledSeq] (n == 1)
    prefill: list = field(default_factory=list)  # [ScheduledSeq]
    preempted: list = field(default_factory=list)

    @property
    def empty(self):
        return not self.decode and not self.prefill

    @property
    def num_tokens(self):
        return len(self.decode) + sum(p.n for p in self.prefill)


def needs_host_state(s: Sequence) -> bool:
    """The next token's sampler input depends on host state advanced by the previous token: a grammar's
    allowed-token mask, mirostat v2's running mu."""
    return s.grammar is not None or s.params.mirostat == 2


class Scheduler:
    def __init__(self, block_manager, block_size: int, max_num_seqs: int = 256, max_batched_tokens: int = 2048,
                 max_model_len: int = 8192, prefill_chunk: int | None = None):
        self.bm = block_manager
        self.bs = block_size
        self.max_num_seqs = max_num_seqs
        self.max_batched_tokens = max_batched_tokens
        self.max_model_len = max_model_len
        self.prefill_chunk = prefill_chunk or max_batched_tokens
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        # finished sequences whose blocks a launched-but-unread step still writes (overlap mode):
        # released by release_deferred() once that step's results were processed
        self.deferred: list[Sequence] = []
        # overlap mode: sequences whose next sample needs host state advanced by their previous token (a
        # grammar, mirostat-2's mu) sit a step out while that token is in flight (engine sets this)
        self.hold_host_state = False

    # ---------------------------------------------------------------- queue management
    def add(self, seq: Sequence):
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def abort(self, rid: int) -> Sequence | None:
        for q in (self.running, self.waiting):
            for s in list(q):
                if s.rid == rid:
                    q.remove(s)
                    if s.n_pending:
                        self.deferred.append(s)  # blocks still written by a launched step
                    else:
                        self.free(s)
                    return s
        return None

    def free(self, seq: Sequence):
        if seq.blocks:
            self.bm.release(seq.blocks)
            seq.blocks = []

    def _blocks_for(self, n_tokens: int) -> int:
        return (n_tokens + self.bs - 1) // self.bs

    def _grow(self, seq: Sequence, n_tokens: int) -> bool:
        need = self._blocks_for(n_tokens) - len(seq.blocks)
        if need <= 0:
            return True
        if need > self.bm.num_free:
            return False
        seq.blocks.extend(self.bm.allocate(need))
        return True

    def _held(self, s: Sequence) -> bool:
        """A sequence whose in-flight samples already reach its length limits: its last step is on
        the GPU, nothing more to schedule; or (hold_host_state) one whose sampler state on the host waits
        for its in-flight token (overlap mode; never true when n_pending == 0)."""
        if not s.n_pending:
            return False
        if s.n_generated >= s.req.max_tokens or s.total_len >= self.max_model_len:
            return True
        return self.hold_host_state and needs_host_state(s)

    def _preempt(self, seq: Sequence, out: SchedulerOutput):
        if seq.n_pending:
            # its in-flight token is not known yet: re-prefill would need it. Overlap mode keeps
            # such sequences (victim selection skips them; see schedule())
            raise RuntimeError("preempting a sequence with in-flight tokens")
        self.running.remove(seq)
        self.free(seq)
        seq.num_computed = 0
        seq.block_hashes = []
        seq.status = Status.WAITING
        self.waiting.appendleft(seq)
        out.preempted.append(seq)

    # ---------------------------------------------------------------- main entry
    def schedule(self) -> SchedulerOutput:
        out = SchedulerOutput()
        budget = self.max_batched_tokens
        # 1. decode phase sequences
        decoding = [s for s in self.running if s.in_decode and not self._held(s)]
        for s in list(decoding):
            if s not in self.running:
                continue
            while not self._grow(s, s.total_len):
                victim = next((v for v in reversed(self.running) if v is not s and not v.n_pending), None)
                if victim is None:
                    break
                self._preempt(victim, out)
                if victim in decoding:
                    decoding.remove(victim)
            if s not in self.running:
                continue
            if self._blocks_for(s.total_len) > len(s.blocks):
                # could not grow even after preemption: preempt itself (or, with a token in flight,
                # sit this step out)
                if not s.n_pending:
                    self._preempt(s, out)
                decoding.remove(s)
                continue
        for s in decoding:
            out.decode.append(ScheduledSeq(s, s.num_computed, 1, True))
        budget -= len(out.decode)
        # 2. continuing prefills of running sequences
        for s in self.running:
            if s.in_decode or budget <= 0:
                continue
            n = min(s.remaining_prefill(), budget, self.prefill_chunk)
            if n <= 0 or not self._grow(s, s.num_computed + n):
                continue
            done = s.num_computed + n >= s.prefill_target
            out.prefill.append(ScheduledSeq(s, s.num_computed, n, done and not s.output_ids and not s.n_pending))
            budget -= n
        # 3. admit new sequences
        while self.waiting and budget > 0 and len(self.running) < self.max_num_seqs:
            s = self.waiting[0]
            if not s.blocks and s.num_computed == 0:
                cached, hashes = self.bm.match_prefix(s.all_ids[: s.prefill_target] if s.req.cache_prompt else [])
                s.blocks = list(cached)
                s.num_computed = len(cached) * self.bs
                s.num_cached = s.num_computed
                s.block_hashes = list(hashes)
            n = min(s.remaining_prefill(), budget, self.prefill_chunk)
            if not self._grow(s, s.num_computed + n):
                if not self.running:
                    # nothing can free memory: fail this request rather than deadlock
                    self.waiting.popleft()
                    self.free(s)
                    s.status = Status.FINISHED
                    s.finish_reason = "error:kv_cache_full"
                    out.preempted.append(s)
                    continue
                break
            self.waiting.popleft()
            s.status = Status.RUNNING
            if s.t_first_sched is None:
                s.t_first_sched = time.perf_counter()
            self.running.append(s)
            done = s.num_computed + n >= s.prefill_target
            out.prefill.append(ScheduledSeq(s, s.num_computed, n, done and not s.output_ids))
            budget -= n
        return out

    def commit(self, sched: SchedulerOutput):
        """Advance KV bookkeeping after the forward pass and register newly full blocks in the
        prefix cache."""
        for item in sched.decode + sched.prefill:
            s = item.seq
            s.num_computed = item.start + item.n
            if not s.req.cache_prompt:  # e.g. image placeholders: token ids do not identify the KV
                continue
            ids = None
            # only blocks whose token ids are all known on the host can be hashed
            nfull = min(s.num_computed, s.known_len) // self.bs
            while len(s.block_hashes) < nfull:
                i = len(s.block_hashes)
                if ids is None:
                    ids = s.all_ids
                parent = s.block_hashes[i - 1] if i > 0 else b""
                h = self.bm.commit_full_block(s.blocks[i], parent, ids[i * self.bs:(i + 1) * self.bs])
                s.block_hashes.append(h)

    def finish(self, seq: Sequence, reason: str):
        seq.status = Status.FINISHED
        seq.finish_reason = reason
        seq.t_finish = time.perf_counter()
        if seq in self.running:
            self.running.remove(seq)
        if seq.n_pending:
            self.deferred.append(seq)  # a launched step still writes its KV blocks
        else:
            self.free(seq)

    def drop_finished(self):
        self.running = [x for x in self.running if x.status != Status.FINISHED]

    def release_deferred(self):
        """Free the blocks of finished sequences whose in-flight steps have all been read."""
        keep = []
        for s in self.deferred:
            if s.n_pending:
                keep.append(s)
            else:
                self.free(s)
        self.deferred = keep
