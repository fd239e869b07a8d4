"""Python face of the native scheduler + step planner (csrc/runtime/scheduler.cpp in libmxrt).

The per-step host work that scales with the batch — picking the step's rows, growing / preempting KV block lists,
prefix-cache admission and block hashing, and the int32 arrays of the forward (tokens, positions, KV slots, logit
rows, block tables, prefill offsets, overlap fix-up rows) — runs in ONE native call per phase instead of Python
loops over 128+ sequences. Decisions are those of engine/scheduler.py::Scheduler (the reference implementation and
the fallback without libmxrt); tests/test_native_scheduler.py checks the two step by step.

Ownership: the scheduler state of a sequence (computed length, in-flight samples, status, cached tokens, queue)
lives in the native int32 table, which `NativeSequence` maps zero-copy — `s.n_pending += 1` in the engine writes
the native row. Token ids the KV bookkeeping needs (prompt + host-known outputs) are mirrored into the native
sequence as they are appended; block lists and hashes exist only natively (`s.blocks` copies on read). When a
sequence leaves every queue its row is copied back into the object and the slot is recycled (`_detach`).
"""
from __future__ import annotations

import collections
import ctypes as C
import time

import numpy as np

from .. import _native
from .scheduler import ScheduledSeq, SchedulerOutput, needs_host_state
from .sequence import Sequence, Status

# table rows (scheduler.cpp F_*)
F_NC, F_NP, F_ST, F_NCACHED, F_NIDS, F_NPROMPT, F_MAXTOK, F_FLAGS, F_NBLK, F_Q = range(10)
NF = 10
Q_NONE, Q_WAIT, Q_RUN, Q_DEF = 0, 1, 2, 3
_STATUS = (Status.WAITING, Status.RUNNING, Status.FINISHED)
_I32P = C.POINTER(C.c_int32)


def available() -> bool:
    try:
        return hasattr(_native.runtime(), "mxrt_sched_new")
    except Exception:
        return False


def _field(i: int):
    def get(self):
        sl = self._slot
        return self._tab[i * self._cap + sl] if sl >= 0 else self._fin[i]

    def put(self, v):
        sl = self._slot
        if sl >= 0:
            self._tab[i * self._cap + sl] = v
        else:
            self._fin[i] = v
    return property(get, put)


class NativeSequence(Sequence):
    """A Sequence whose scheduler state is a row of the native table while it is queued."""
    num_computed = _field(F_NC)
    n_pending = _field(F_NP)
    num_cached = _field(F_NCACHED)

    def __init__(self, req, tokenizer, sched: "NativeScheduler"):
        self._slot = -1
        self._fin = [0] * NF
        self._tab, self._cap, self._ns = sched.tab, sched.cap, sched
        super().__init__(req, tokenizer)

    @property
    def status(self) -> Status:
        sl = self._slot
        return _STATUS[self._tab[F_ST * self._cap + sl] if sl >= 0 else self._fin[F_ST]]

    @status.setter
    def status(self, v: Status):
        sl = self._slot
        if sl >= 0:
            self._tab[F_ST * self._cap + sl] = v.value
        else:
            self._fin[F_ST] = v.value

    @property
    def blocks(self) -> list:
        return self._ns.blocks_of(self) if self._slot >= 0 else []

    @blocks.setter
    def blocks(self, v):
        if v:
            raise AttributeError("the native scheduler owns block lists")

    def append_token(self, tid: int, logprob):
        tid = int(tid)
        self.output_ids.append(tid)
        self._pending_ids.append(tid)
        if logprob is not None:
            lp = float(logprob)
            self.logprobs.append(lp)
            self._pending_lp.append(lp)
        if self._slot >= 0:  # mirrored in one native call before the scheduler next reads token ids
            self._ns._push += (self._slot, tid)

    def pop_output(self):
        super().pop_output()
        if self._slot >= 0:
            self._ns._push += (self._slot, -1)


class NativeScheduler:
    """Drop-in for engine.scheduler.Scheduler on top of a NativeBlockManager."""

    def __init__(self, block_manager, block_size: int, max_num_seqs: int = 256, max_batched_tokens: int = 2048,
                 max_model_len: int = 8192, prefill_chunk: int | None = None, capacity: int = 0):
        self.rt = rt = _native.runtime()
        self.bm = block_manager
        self.bs = block_size
        self.max_num_seqs = max_num_seqs
        self.max_batched_tokens = max_batched_tokens
        self.max_model_len = max_model_len
        self.prefill_chunk = prefill_chunk or max_batched_tokens
        # slots for running + waiting sequences; more waiting requests queue here in Python until slots free up
        # (>= 2 max_num_seqs + 2: running + deferred never crowd out the head of the waiting queue, so admission
        # order is the Python scheduler's)
        self.cap = max(capacity or max(4096, 16 * max_num_seqs), 2 * max_num_seqs + 2)
        self._h = rt.mxrt_sched_new(block_manager._h, block_size, max_num_seqs, max_batched_tokens, max_model_len,
                                    self.prefill_chunk, self.cap)
        buf = (C.c_int32 * (NF * self.cap)).from_address(rt.mxrt_sched_table(self._h))
        self._buf = buf
        self.tab = memoryview(buf).cast("B").cast("i")
        self._by_slot: dict[int, NativeSequence] = {}
        self._by_rid: dict[int, NativeSequence] = {}
        self._overflow: collections.deque = collections.deque()
        self._hold = False
        self._push: list = []  # (slot, token | -1 = pop) pairs not yet mirrored natively
        self._counts = np.zeros(8, np.int32)
        self._obuf = np.zeros(8 * self.cap + 16, np.int32)
        self._meta = np.zeros(8, np.int32)
        self._blk = np.zeros(1 + (max_model_len + block_size - 1) // block_size, np.int32)

    def __del__(self):
        try:
            self.rt.mxrt_sched_free(self._h)
        except Exception:
            pass

    def new_sequence(self, req, tokenizer) -> NativeSequence:
        return NativeSequence(req, tokenizer, self)

    # ---------------------------------------------------------------- state views
    @property
    def hold_host_state(self) -> bool:
        return self._hold

    @hold_host_state.setter
    def hold_host_state(self, v: bool):
        self._hold = bool(v)
        self.rt.mxrt_sched_set_hold(self._h, int(self._hold))

    def _queue(self, which: int) -> list:
        n = self.rt.mxrt_sched_queue(self._h, which, None, 0)
        if not n:
            return []
        out = np.empty(n, np.int32)
        self.rt.mxrt_sched_queue(self._h, which, out.ctypes.data, n)
        return [self._by_slot[int(x)] for x in out]

    @property
    def waiting(self) -> list:
        return self._queue(0) + list(self._overflow)

    @property
    def running(self) -> list:
        return self._queue(1)

    @property
    def deferred(self) -> list:
        return self._queue(2)

    def has_work(self) -> bool:
        return bool(self._overflow) or bool(self.rt.mxrt_sched_queue(self._h, 0, None, 0)) or bool(
            self.rt.mxrt_sched_queue(self._h, 1, None, 0))

    def blocks_of(self, s: NativeSequence) -> list:
        n = self.rt.mxrt_sched_blocks(self._h, s._slot, self._blk.ctypes.data, len(self._blk))
        return self._blk[:n].tolist()

    # ---------------------------------------------------------------- queue management
    def add(self, seq: NativeSequence):
        if self._overflow or not self._attach(seq):
            self._overflow.append(seq)
        self._by_rid[seq.rid] = seq

    def _attach(self, seq: NativeSequence) -> bool:
        ids = np.asarray(seq.all_ids, np.int32)
        flags = (1 if seq.req.cache_prompt else 0) | (2 if needs_host_state(seq) else 0)
        sl = self.rt.mxrt_sched_add(self._h, ids.ctypes.data, ids.size, int(seq.req.max_tokens), flags)
        if sl < 0:
            return False
        fin = seq._fin
        seq._slot = sl
        self._by_slot[sl] = seq
        # state set before the slot existed (fresh sequences: zeros / WAITING)
        seq.num_computed, seq.n_pending = fin[F_NC], fin[F_NP]
        return True

    def _flush(self):
        if self._push:
            a = np.asarray(self._push, np.int32)
            self._push = []
            self.rt.mxrt_sched_push_many(self._h, a.ctypes.data, len(a) // 2)

    def _detach(self, seq: NativeSequence):
        sl = seq._slot
        if sl < 0:
            return
        self._flush()
        t, cap = self.tab, self.cap
        seq._fin = [t[i * cap + sl] for i in range(NF)]
        seq._slot = -1
        self._by_slot.pop(sl, None)
        self._by_rid.pop(seq.rid, None)
        self.rt.mxrt_sched_release_slot(self._h, sl)
        while self._overflow and self._attach(self._overflow[0]):
            self._overflow.popleft()

    def abort(self, rid: int) -> NativeSequence | None:
        s = self._by_rid.get(rid)
        if s is None:
            return None
        if s._slot < 0:
            if s in self._overflow:
                self._overflow.remove(s)
                self._by_rid.pop(rid, None)
                return s
            return None
        return s if self.rt.mxrt_sched_abort(self._h, s._slot) else None

    def finish(self, seq: NativeSequence, reason: str):
        seq.finish_reason = reason
        seq.t_finish = time.perf_counter()
        if seq._slot < 0:
            seq.status = Status.FINISHED
            self._by_rid.pop(seq.rid, None)
            if seq in self._overflow:
                self._overflow.remove(seq)
            return
        self.rt.mxrt_sched_finish(self._h, seq._slot)
        if self.tab[F_Q * self.cap + seq._slot] == Q_NONE:
            self._detach(seq)

    def release_deferred(self):
        out = np.empty(max(1, len(self._by_slot)), np.int32)
        n = self.rt.mxrt_sched_release_deferred(self._h, out.ctypes.data)
        for sl in out[:n].tolist():
            s = self._by_slot.get(sl)
            if s is not None:
                self._detach(s)

    def drop_finished(self):
        """Finished sequences never stay in the native running queue (finish removes them)."""

    def _grow(self, seq: NativeSequence, n_tokens: int) -> bool:
        self._flush()
        return bool(self.rt.mxrt_sched_grow(self._h, seq._slot, n_tokens))

    # ---------------------------------------------------------------- main entry
    def schedule(self) -> SchedulerOutput:
        while self._overflow and self._attach(self._overflow[0]):
            self._overflow.popleft()
        self._flush()
        rt, h = self.rt, self._h
        c = self._counts
        if rt.mxrt_sched_schedule(h, c.ctypes.data) != 0:
            raise RuntimeError("preempting a sequence with in-flight tokens")
        nd, npf, npre = int(c[0]), int(c[1]), int(c[2])
        by = self._by_slot
        out = SchedulerOutput()
        ob = self._obuf
        n = rt.mxrt_sched_out_packed(h, ob.ctypes.data, len(ob))
        ob = ob[:n].copy()
        dec, pf = ob[:2 * nd], ob[2 * nd:2 * nd + 4 * npf]
        if npre:
            pre = ob[2 * nd + 4 * npf:].tolist()
            for k in range(npre):
                s = by[pre[2 * k]]
                if pre[2 * k + 1]:  # nothing can free memory: the request fails rather than deadlocking
                    s.finish_reason = "error:kv_cache_full"
                    self._detach(s)
                out.preempted.append(s)
        dl = dec.tolist()
        out.decode = [ScheduledSeq(by[dl[k]], dl[k + 1], 1, True) for k in range(0, 2 * nd, 2)]
        if npf:
            pl = pf.tolist()
            now = None
            for k in range(0, 4 * npf, 4):
                s = by[pl[k]]
                if s.t_first_sched is None:
                    s.t_first_sched = now = now or time.perf_counter()
                out.prefill.append(ScheduledSeq(s, pl[k + 1], pl[k + 2], bool(pl[k + 3])))
        out._nat = (dec[0::2].copy(), dec[1::2].copy(), pf, out.decode, out.prefill)
        return out

    @staticmethod
    def _cached(so: SchedulerOutput):
        nat = getattr(so, "_nat", None)
        if nat is not None and nat[3] is so.decode and nat[4] is so.prefill and len(nat[0]) == len(so.decode) \
                and len(nat[2]) == 4 * len(so.prefill):
            return nat
        return None

    def _items(self, so: SchedulerOutput):
        """(decode slots, prefill (slot, start, n, sample) rows) of a SchedulerOutput (cached from schedule())."""
        nat = self._cached(so)
        if nat is not None:
            return nat[0], nat[2]
        dec = np.asarray([it.seq._slot for it in so.decode], np.int32)
        pf = np.asarray([(it.seq._slot, it.start, it.n, int(it.sample)) for it in so.prefill], np.int32).reshape(-1)
        return dec, pf

    def plan_arrays(self, so: SchedulerOutput) -> dict:
        """The step's int32 arrays (engine._plan keys) built natively."""
        self._flush()
        rt, h = self.rt, self._h
        dec, pf = self._items(so)
        nd, npf = len(dec), len(pf) // 4
        dec = np.ascontiguousarray(dec, np.int32)
        pf = np.ascontiguousarray(pf, np.int32)
        m = self._meta
        rc = rt.mxrt_sched_plan(h, dec.ctypes.data, nd, pf.ctypes.data, npf, m.ctypes.data)
        if rc == -2:
            raise KeyError("decode input in flight but not in the last launched step")
        if rc:
            raise RuntimeError(f"native plan failed ({rc})")
        T, S, dmaxb, pmaxb, nfix = (int(x) for x in m[:5])
        sizes = (T, T, T, S, nd * dmaxb, nd, npf * pmaxb, npf + 1 if npf else 0, npf, nfix, nfix)
        buf = np.empty(max(1, sum(sizes)), np.int32)
        rt.mxrt_sched_plan_packed(h, buf.ctypes.data, len(buf))
        a, o = [], 0
        for n in sizes:
            a.append(buf[o:o + n])
            o += n
        plan = {"tokens": a[0], "positions": a[1], "slots": a[2], "lidx": a[3]}
        if nd:
            plan["dec_bt"] = a[4].reshape(nd, dmaxb)
            plan["dec_lens"] = a[5]
        if npf:
            plan["pf_bt"] = a[6].reshape(npf, pmaxb)
            plan["pf_cu"] = a[7]
            plan["pf_ctx"] = a[8]
        if nfix:
            plan["fix"] = (a[9].astype(np.int64), a[10].astype(np.int64))
        return plan

    def item_slots(self, so: SchedulerOutput | None, items) -> np.ndarray:
        """Native slots of a step's sampled rows (decode rows + finishing prefills), in row order."""
        nat = self._cached(so) if so is not None else None
        if nat is not None and len(items) == len(so.decode) + sum(1 for it in so.prefill if it.sample):
            pf = nat[2].reshape(-1, 4)
            sl = np.concatenate([nat[0], pf[pf[:, 3] != 0, 0]]) if len(pf) else nat[0]
            return np.ascontiguousarray(sl, np.int32)
        return np.asarray([it.seq._slot for it in items], np.int32)

    def add_pending(self, slots: np.ndarray, d: int):
        """n_pending += d for every slot (a launched step's sampled rows: +1; their read-back: -1): one native
        call. Slots stay attached while they have samples in flight (finish defers them)."""
        if (slots < 0).any():
            raise RuntimeError("in-flight sample of a released sequence")
        self.rt.mxrt_sched_add_pending(self._h, slots.ctypes.data, len(slots), d)

    def pending_on_device(self, so: SchedulerOutput) -> bool:
        dec = np.ascontiguousarray(self._items(so)[0], np.int32)
        return bool(self.rt.mxrt_sched_pending_ok(self._h, dec.ctypes.data, len(dec)))

    def set_prev(self, items, slots: np.ndarray | None = None):
        """Rows of the last launched sampling step (decode inputs in flight are gathered from it)."""
        sl = slots if slots is not None else np.asarray([it.seq._slot for it in items], np.int32)
        self.rt.mxrt_sched_set_prev(self._h, sl.ctypes.data, sl.size)

    def clear_prev(self):
        self.rt.mxrt_sched_clear_prev(self._h)

    def commit(self, sched: SchedulerOutput):
        nat = self._cached(sched)
        if nat is not None:
            dec, starts, pf = nat[0], nat[1], nat[2]
            nd = len(dec)
            tri = np.empty((nd + len(pf) // 4, 3), np.int32)
            if nd:
                tri[:nd, 0] = dec
                tri[:nd, 1] = starts
                tri[:nd, 2] = 1
            if len(pf):
                p4 = pf.reshape(-1, 4)
                tri[nd:] = p4[:, :3]
        else:
            tri = np.asarray([(it.seq._slot, it.start, it.n) for it in sched.decode + sched.prefill],
                             np.int32).reshape(-1, 3)
        tri = np.ascontiguousarray(tri)
        self._flush()
        self.rt.mxrt_sched_commit(self._h, tri.ctypes.data, len(tri))
