"""Native scheduler + step planner (csrc/runtime/scheduler.cpp) against the Python reference Scheduler and the
engine's Python plan, step by step on randomized workloads: admission with prefix-cache hits, chunked prefill,
overlap-mode in-flight tokens, KV pressure with preemption and resumption, aborts, finishes with deferred block
release, and more requests than native slots (the Python overflow queue)."""
import random
import types

import numpy as np
import pytest

from localai_tfp_amd.engine import native_scheduler as NS
from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
from localai_tfp_amd.engine.scheduler import Scheduler
from localai_tfp_amd.engine.sequence import Request, Sequence, Status
from localai_tfp_amd.ops.sampling import SamplingParams

pytestmark = pytest.mark.skipif(not NS.available(), reason="libmxrt not built")


def _bm(nb, bs):
    from localai_tfp_amd.runtime_native import NativeBlockManager
    return NativeBlockManager(nb, bs, True)


def _stub(bs, sched=None):
    e = types.SimpleNamespace(cfg=EngineConfig(block_size=bs), _prev_dev=None, native_sched=sched is not None,
                              sched=sched, device=types.SimpleNamespace(type="cpu"), model=None)
    e._graph_key = lambda plan: None
    e._graph_get = lambda *a, **k: None
    e._plan_finish = lambda so, plan: LLMEngine._plan_finish(e, so, plan)
    return e


def _key(so):
    return ([(it.seq.rid, it.start, it.n, it.sample) for it in so.decode],
            [(it.seq.rid, it.start, it.n, it.sample) for it in so.prefill],
            [(s.rid, s.status, s.finish_reason) for s in so.preempted])


def _plan_eq(a, b):
    assert set(a) == set(b), (sorted(a), sorted(b))
    for k in a:
        if k == "fix":
            for x, y in zip(a[k], b[k]):
                np.testing.assert_array_equal(x, y)
        elif isinstance(a[k], np.ndarray):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        else:
            assert a[k] == b[k], k


@pytest.mark.parametrize("seed,nb,cap,overlap", [(0, 400, 0, True), (1, 90, 0, True), (2, 60, 0, False),
                                                 (3, 120, 18, True), (4, 70, 0, True)])
def test_native_matches_python_scheduler(seed, nb, cap, overlap):
    rng = random.Random(seed)
    bs, budget, max_seqs, max_len = 16, 96, 8, 512
    py = Scheduler(_bm(nb, bs), bs, max_seqs, budget, max_len)
    nat = NS.NativeScheduler(_bm(nb, bs), bs, max_seqs, budget, max_len, capacity=cap)
    stub, stub_n = _stub(bs), _stub(bs, nat)
    seqs = {}  # rid -> (python seq, native seq)
    shared = [rng.randrange(1000) for _ in range(64)]  # common prefix: prefix-cache hits
    inflight = None
    rid = 10_000 * (seed + 1)
    n_pre = n_hit = 0
    min_free = nb
    max_over = 0
    for step in range(260):
        # arrivals
        for _ in range(rng.choice([0, 0, 1, 2])):
            rid += 1
            n = rng.randrange(5, 150)
            prompt = (shared[:rng.choice([0, 32, 48, 64])] + [rng.randrange(1000) for _ in range(n)])[:max_len - 40]
            mt = rng.randrange(2, 40 if nb >= 100 else 160)
            ps = Sequence(Request(list(prompt), SamplingParams(), max_tokens=mt, rid=rid), None)
            ns = nat.new_sequence(Request(list(prompt), SamplingParams(), max_tokens=mt, rid=rid), None)
            py.add(ps)
            nat.add(ns)
            seqs[rid] = (ps, ns)
        # an abort now and then
        if rng.random() < 0.05 and seqs:
            r = rng.choice(sorted(seqs))
            a, b = py.abort(r), nat.abort(r)
            assert (a is None) == (b is None)
            if a is not None:
                py.finish(a, "abort")
                nat.finish(b, "abort")
        sp, sn = py.schedule(), nat.schedule()
        assert _key(sp) == _key(sn), step
        n_pre += sum(1 for s in sp.preempted if s.status != Status.FINISHED)
        min_free = min(min_free, py.bm.num_free)
        max_over = max(max_over, len(nat._overflow))
        if sp.empty:
            if inflight is None:
                continue
        else:
            _plan_eq(LLMEngine._plan(stub, sp), LLMEngine._plan(stub_n, sn))
        items_p = list(sp.decode) + [it for it in sp.prefill if it.sample]
        items_n = list(sn.decode) + [it for it in sn.prefill if it.sample]
        if overlap:
            for it in items_p + items_n:
                it.seq.n_pending += 1
        py.commit(sp)
        nat.commit(sn)
        # read back: the previous step's tokens (overlap) or this step's (sync)
        if overlap:
            done, inflight = inflight, (items_p, items_n)
            stub._prev_dev = (None, {it.seq.rid: r for r, it in enumerate(items_p)}) if items_p else None
            nat.set_prev(items_n) if items_n else nat.clear_prev()
        else:
            done = (items_p, items_n)
        if done is not None:
            for ip, inn in zip(*done):
                for s in (ip.seq, inn.seq):
                    if overlap:
                        s.n_pending -= 1
                    if s.status == Status.FINISHED:
                        continue
                    t = (s.rid * 31 + len(s.output_ids) * 7) % 1000
                    s.append_token(t, None)
                    if len(s.output_ids) >= s.req.max_tokens or t % 97 == 0:
                        if t % 97 == 0:
                            s.pop_output()
                        (nat if isinstance(s, NS.NativeSequence) else py).finish(s, "stop")
            py.release_deferred()
            nat.release_deferred()
        for r, (a, b) in list(seqs.items()):
            assert (a.status, a.n_pending, a.num_computed, a.num_cached) == \
                (b.status, b.n_pending, b.num_computed, b.num_cached), (step, r)
            if a.status != Status.FINISHED:
                assert a.blocks == b.blocks, (step, r)
            if a.status == Status.FINISHED and not a.n_pending and b._slot < 0:
                del seqs[r]
            n_hit = max(n_hit, a.num_cached)
    assert py.bm.stats() == nat.bm.stats()
    if nb < 100:  # the small pools ran out of blocks (sync mode: with preemptions; overlap mode preempts only
        assert min_free <= 2  # sequences without a token in flight)
        assert n_pre > 0 or overlap
    if cap:
        assert max_over > 0  # requests waited for a native slot
    assert n_hit > 0


def test_native_scheduler_in_engine_and_slot_recycling(monkeypatch):
    """The CPU engine runs on the native scheduler by default, produces the Python scheduler's tokens, and finished
    sequences give their native slots back."""
    from localai_tfp_amd.models.loader import load_llm
    model, tok, cfg, _ = load_llm("synthetic:tiny", "cpu")

    def run():
        e = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=256, use_graphs=False))
        hs = [e.submit(Request(list(range(1, 20 + k)), SamplingParams(temperature=0.0), max_tokens=6))
              for k in range(10)]
        e.run_until_done()
        return e, [[t for o in h for t in o.token_ids] for h in hs]
    e, ids = run()
    assert e.native_sched and isinstance(e.sched, NS.NativeScheduler)
    assert all(ids)
    assert not e.sched._by_slot and not e.sched.running and not e.sched.waiting and not e.sched.deferred
    monkeypatch.setenv("MX_PY_SCHED", "1")
    e2, ids2 = run()
    assert not e2.native_sched
    assert ids == ids2
