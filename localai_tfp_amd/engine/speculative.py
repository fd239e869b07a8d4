"""Speculative decoding with a draft model (N12 of SURVEY §2.3).

The reference enables it per model with `draft_model` / `n_draft` (llama.cpp server: a small
draft model proposes tokens, the target verifies them in one batch,
backend/cpp/llama/grpc-server.cpp params `speculative.model` / `n_draft`). Here it plugs into the
paged continuous-batching engine:

* the draft has its own paged KV cache with the SAME block ids as the target (one block table
  per sequence serves both), so no extra allocator; it catches up lazily — the first speculative
  step of a sequence prefills the draft over everything the target already holds;
* a speculative step (decode-only batch of at most `spec_max_batch` sequences without grammars):
    1. draft: one chunked forward over the tokens it has not seen (greedy proposal d1), then
       k-1 decode forwards (d2..dk);
    2. target: ONE prefill-style forward over [t0, d1..dk] per sequence (logits for all k+1 rows —
       the MFMA prefill attention handles the intra-chunk causal mask);
    3. sample the target at every row with the sequence's own sampler and accept while the sample
       equals the draft token (llama.cpp common_sampler_sample_and_accept_n): the output is the
       accepted drafts + one target token, i.e. exactly what plain decoding would have sampled —
       greedy output is identical to non-speculative decoding whatever the draft proposes;
    4. KV written for rejected drafts is simply overwritten later (attention reads seq_len keys).
"""
from __future__ import annotations

import logging
import time

import numpy as np
import torch

from ..models.llama import ForwardBatch, LlamaModel, Workspace
from .kv_cache import KVCache
from .scheduler import SchedulerOutput, ScheduledSeq

log = logging.getLogger("localai_tfp_amd.engine.spec")


class SpeculativeDecoder:
    def __init__(self, engine, draft: LlamaModel, n_draft: int = 4, max_batch: int = 32):
        e = engine
        mc, dc = e.model.cfg, draft.cfg
        if dc.vocab > mc.vocab:
            raise ValueError(f"draft vocab {dc.vocab} larger than the target's {mc.vocab}")
        self.e = e
        self.draft = draft
        self.k = max(1, int(n_draft))
        self.max_batch = max(1, min(int(max_batch), e.cfg.max_num_seqs))
        c = e.cfg
        nb = e.kv.num_blocks
        self.kv = KVCache(dc.n_layers, nb, draft.n_kv, c.block_size, dc.head_dim, e.device, e.kv_dtype,
                          kvf=getattr(e, "kvf", 0))
        rows = self.max_batch * (self.k + 1)
        # draft catch-up chunks can be whole prompts: size its workspace like the engine's
        self.dws = Workspace(dc, max(c.max_batched_tokens, rows), max(self.max_batch, 1), e.device, 1,
                             max(1, -(-c.max_model_len // c.attn_part_size)))
        # target verification: every row of every chunk needs logits
        self.vws = Workspace(mc, rows, rows, e.device, e.model.tp_size, 1)
        self.cap = self.dws.max_tokens
        self.computed: dict[int, int] = {}  # rid -> draft KV length
        self.stats = dict(spec_steps=0, drafted=0, accepted=0, draft_s=0.0, verify_s=0.0)

    # ---------------------------------------------------------------- eligibility
    def eligible(self, so: SchedulerOutput) -> bool:
        if so.prefill or not so.decode or len(so.decode) > self.max_batch:
            return False
        for it in so.decode:
            s = it.seq
            p = s.params
            if s.grammar is not None or s.req.embedding or p.mirostat or s.req.mm_embeds:
                return False
        return True

    def forget(self, rid: int):
        self.computed.pop(rid, None)

    # ---------------------------------------------------------------- helpers
    def _prefill_fb(self, chunks, all_rows: bool) -> ForwardBatch:
        """chunks: [(token ids, start position, blocks)] -> ForwardBatch of prefill rows (logits of
        every row if all_rows, else of each chunk's last row)."""
        dev = self.e.device
        bs = self.e.cfg.block_size
        toks, pos, slots, lidx, cu, ctx = [], [], [], [], [0], []
        maxb = max(len(b) for _, _, b in chunks)
        bt = np.zeros((len(chunks), maxb), np.int32)
        for k, (ids, p0, blocks) in enumerate(chunks):
            n = len(ids)
            r = np.arange(p0, p0 + n)
            blk = np.asarray(blocks, np.int32)
            toks.extend(ids)
            pos.extend(r.tolist())
            slots.extend((blk[r // bs] * bs + r % bs).tolist())
            off = cu[-1]
            lidx.extend(range(off, off + n) if all_rows else [off + n - 1])
            cu.append(off + n)
            ctx.append(p0 + n)
            bt[k, :len(blocks)] = blocks

        def t(x):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(x, np.int32))).to(dev, non_blocking=True)

        fb = ForwardBatch(t(toks), t(pos), t(slots), t(lidx), n_decode=0)
        fb.pf_block_tables, fb.pf_cu_q, fb.pf_ctx_lens = t(bt), t(cu), t(ctx)
        fb.pf_q_lens_host = [cu[i + 1] - cu[i] for i in range(len(chunks))]
        fb.pf_ctx_lens_host = list(ctx)
        return fb

    def _decode_fb(self, toks, positions, seqs) -> ForwardBatch:
        dev = self.e.device
        bs = self.e.cfg.block_size
        B = len(seqs)
        maxb = max(len(s.blocks) for s in seqs)
        bt = np.zeros((B, maxb), np.int32)
        slots = np.empty(B, np.int32)
        for k, s in enumerate(seqs):
            bt[k, :len(s.blocks)] = s.blocks
            p = positions[k]
            slots[k] = s.blocks[p // bs] * bs + p % bs

        def t(x):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(x, np.int32))).to(dev, non_blocking=True)

        lens = np.asarray(positions, np.int32) + 1
        fb = ForwardBatch(t(toks), t(positions), t(slots), t(np.arange(B)), n_decode=B)
        fb.dec_block_tables, fb.dec_seq_lens, fb.dec_max_len = t(bt), t(lens), int(lens.max())
        return fb

    @staticmethod
    def _argmax(logits: torch.Tensor, V: int) -> list[int]:
        return logits[:, :V].argmax(-1).tolist()

    # ---------------------------------------------------------------- one speculative step
    def step(self, so: SchedulerOutput) -> bool:
        """Run a speculative step for a decode-only batch. False = not possible (caller falls back
        to a plain decode step; nothing was changed except possibly pre-grown block tables)."""
        e = self.e
        c = e.cfg
        items = so.decode
        seqs = [it.seq for it in items]
        k = self.k
        for s in seqs:  # never draft past max_tokens / max_model_len (nor the request's n_draft)
            k = min(k, s.req.max_tokens - len(s.output_ids) - 1, c.max_model_len - s.total_len - 1)
            if s.req.n_draft > 0:
                k = min(k, s.req.n_draft)
        if k < 1:
            return False
        for s in seqs:
            if not e.sched._grow(s, s.num_computed + k + 1):
                return False
        Vd = self.draft.cfg.vocab
        t0 = time.perf_counter()
        # 1. draft: catch up (chunked prefill of unseen tokens) -> d1
        L = [s.num_computed for s in seqs]
        first: list[int] = [0] * len(seqs)
        pending = []
        for i, s in enumerate(seqs):
            dc = min(self.computed.get(s.rid, 0), L[i])
            pending.append((i, s.all_ids[dc:L[i] + 1], dc))
        while pending:
            batch, n = [], 0
            while pending and (not batch or n + len(pending[0][1]) <= self.cap):
                i, ids, dc = pending.pop(0)
                if len(ids) > self.cap:  # very long unseen prefix: feed it in cap-sized pieces
                    head, rest = ids[:self.cap], ids[self.cap:]
                    self.draft.forward(self._prefill_fb([(head, dc, seqs[i].blocks)], False), self.kv, self.dws)
                    pending.insert(0, (i, rest, dc + len(head)))
                    continue
                batch.append((i, ids, dc))
                n += len(ids)
            if not batch:
                continue
            lg = self.draft.forward(self._prefill_fb([(ids, dc, seqs[i].blocks) for i, ids, dc in batch], False),
                                    self.kv, self.dws)
            for (i, _, _), tkn in zip(batch, self._argmax(lg, Vd)):
                first[i] = tkn
        drafts = [[d] for d in first]
        cur = first
        for j in range(1, k):  # 2. draft decode: d2..dk
            lg = self.draft.forward(self._decode_fb(cur, [L[i] + j for i in range(len(seqs))], seqs), self.kv,
                                    self.dws)
            cur = self._argmax(lg, Vd)
            for i, d in enumerate(cur):
                drafts[i].append(d)
        t1 = time.perf_counter()
        # 3. target verification over [t0, d1..dk]
        chunks = [([s.all_ids[L[i]]] + drafts[i], L[i], s.blocks) for i, s in enumerate(seqs)]
        logits = e.model.forward(self._prefill_fb(chunks, True), e.kv, self.vws)
        params = [s.params for s in seqs for _ in range(k + 1)]
        hist = [s.all_ids for s in seqs for _ in range(k + 1)]
        steps = [len(s.output_ids) + j for s in seqs for j in range(k + 1)]
        tok, lp = e.sampler.sample(logits, params, hist, steps, None, None)
        tok = tok.cpu().tolist()
        lp = lp.cpu().tolist() if lp is not None else None
        t2 = time.perf_counter()
        # 4. accept / emit / commit
        done_items = []
        for i, s in enumerate(seqs):
            row = tok[i * (k + 1):(i + 1) * (k + 1)]
            rlp = lp[i * (k + 1):(i + 1) * (k + 1)] if lp is not None else None
            n_acc = 0
            while n_acc < k and row[n_acc] == drafts[i][n_acc]:
                n_acc += 1
            self.stats["drafted"] += k
            self.stats["accepted"] += n_acc
            out = row[:n_acc + 1]
            self.computed[s.rid] = min(L[i] + n_acc + 1, L[i] + k)
            emitted, reason = e._accept_tokens(s, out, rlp[:n_acc + 1] if rlp is not None else None)
            if reason is None:  # KV now holds t0, d1..d_n_acc; the last sampled token is the next input
                done_items.append(ScheduledSeq(s, L[i], emitted, True))
        e.sched.commit(SchedulerOutput(decode=done_items))
        st = self.stats
        st["spec_steps"] += 1
        st["draft_s"] += t1 - t0
        st["verify_s"] += t2 - t1
        return True
