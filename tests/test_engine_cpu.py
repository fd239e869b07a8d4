"""Engine plumbing on CPU (fp32 reference ops): scheduling, paged KV, prefix cache, stop
handling, preemption, detokenisation."""
import itertools

import numpy as np
import pytest
import torch

from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
from localai_tfp_amd.engine.kv_cache import PyBlockManager
from localai_tfp_amd.engine.sequence import Request
from localai_tfp_amd.models.config import tiny_config
from localai_tfp_amd.models.llama import LlamaModel
from localai_tfp_amd.models.synthetic import synthetic_source
from localai_tfp_amd.ops.sampling import SamplingParams
from localai_tfp_amd.tokenizer import ByteTokenizer


@pytest.fixture(scope="module")
def model():
    cfg = tiny_config(n_layers=2)
    return LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=11), "cpu")


def mk(model, **kw):
    tok = ByteTokenizer(model.cfg.vocab)
    c = dict(num_blocks=256, max_num_seqs=8, max_batched_tokens=64, max_model_len=512)
    c.update(kw)
    return LLMEngine(model, tok, EngineConfig(**c)), tok


def test_greedy_deterministic_and_prefix_cache(model):
    e, tok = mk(model)
    p = tok.encode("abcdefghijklmnopqrstuvwxyz0123456789 prefix caching test")
    a = e.generate(p, max_tokens=10)
    b = e.generate(p, max_tokens=10)
    assert a.token_ids == b.token_ids
    assert a.cached_tokens == 0 and b.cached_tokens >= 48
    assert a.finish_reason == "length" and len(a.token_ids) == 10


def test_chunked_prefill_equals_single_shot(model):
    p = list(range(300, 400)) + list(range(1, 120))
    e1, _ = mk(model, max_batched_tokens=512, enable_prefix_cache=False)
    e2, _ = mk(model, max_batched_tokens=32, enable_prefix_cache=False)  # forces 7 chunks
    a = e1.generate(p, max_tokens=6)
    b = e2.generate(p, max_tokens=6)
    assert a.token_ids == b.token_ids


def test_batched_equals_sequential(model):
    prompts = [list(range(10 + i, 40 + 3 * i)) for i in range(5)]
    e, _ = mk(model, enable_prefix_cache=False)
    seq = [e.generate(p, max_tokens=5).token_ids for p in prompts]
    e2, _ = mk(model, enable_prefix_cache=False)
    hs = [e2.submit(Request(p, SamplingParams(temperature=0.0), 5)) for p in prompts]
    e2.run_until_done()
    par = []
    for h in hs:
        ids = []
        for o in h:
            ids += o.token_ids
        par.append(ids)
    assert par == seq


def test_preemption_under_tiny_cache(model):
    # 12 blocks of 16 tokens shared by 4 requests of ~60 tokens each -> preemptions must happen
    e, _ = mk(model, num_blocks=13, enable_prefix_cache=False, max_batched_tokens=256)
    prompts = [list(range(5 + i, 50 + i)) for i in range(4)]
    ref_e, _ = mk(model, enable_prefix_cache=False)
    sp = SamplingParams(temperature=0.0, ignore_eos=True)
    ref = [ref_e.generate(p, sp, max_tokens=12).token_ids for p in prompts]
    hs = [e.submit(Request(p, sp, 12)) for p in prompts]
    e.run_until_done(max_steps=5000)
    got = []
    for h in hs:
        ids = []
        for o in h:
            ids += o.token_ids
        got.append(ids)
    assert got == ref
    assert e.stats["preemptions"] > 0


def test_stop_strings_and_eos(model):
    e, tok = mk(model)
    p = tok.encode("stop string test")
    full = e.generate(p, max_tokens=16)
    text = full.text
    if len(text) >= 4:
        stop = text[2:4]
        o = e.generate(p, max_tokens=16, stop=[stop])
        assert o.finish_reason == "stop"
        assert o.text == text[: text.find(stop)]
    # EOS: force via logit_bias on eot id
    sp = SamplingParams(temperature=0.0, logit_bias={tok.eos_token_ids[1]: 1000.0})
    o = e.generate(p, sp, max_tokens=16)
    assert o.finish_reason == "stop" and o.completion_tokens == 0


def test_sampling_seeded_reproducible(model):
    e, tok = mk(model)
    p = tok.encode("sampling")
    sp = SamplingParams(temperature=1.0, top_k=20, top_p=0.9, seed=42)
    a = e.generate(p, sp, max_tokens=8)
    b = e.generate(p, sp, max_tokens=8)
    assert a.token_ids == b.token_ids


def test_block_manager_prefix_and_eviction():
    bm = PyBlockManager(num_blocks=9, block_size=4)
    toks = list(range(17))
    blocks, hashes = bm.match_prefix(toks)
    assert blocks == []
    own = bm.allocate(5)
    parent = b""
    hs = []
    for i in range(4):
        parent = bm.commit_full_block(own[i], parent, toks[4 * i:4 * i + 4])
        hs.append(parent)
    bm.release(own)
    assert bm.num_free == 8
    blocks, hashes = bm.match_prefix(toks)
    assert blocks == own[:4] and hashes == hs
    bm.release(blocks)
    # exhaust the pool: cached blocks must be evicted, not leaked
    got = bm.allocate(8)
    assert len(set(got)) == 8 and 0 not in got
    with pytest.raises(MemoryError):
        bm.allocate(1)


def _run_all(e, reqs):
    hs = [e.submit(r) for r in reqs]
    e.run_until_done()
    out = []
    for h in hs:
        ids, text, last = [], "", None
        while not h.q.empty():
            o = h.q.get_nowait()
            ids += o.token_ids
            text += o.text
            last = o
        out.append((ids, text, last.finish_reason if last else None, last.completion_tokens if last else None))
    return out


def _mixed_requests(seed=0):
    rng = np.random.default_rng(seed)
    reqs = []
    for i in range(10):
        p = [int(x) for x in rng.integers(1, 250, size=int(rng.integers(5, 90)))]
        kw = {}
        if i % 3 == 1:
            sp = SamplingParams(temperature=0.8, top_k=40, top_p=0.9, seed=100 + i)
        elif i % 3 == 2:
            sp = SamplingParams(temperature=0.0, logit_bias={7: 3.0})
        else:
            sp = SamplingParams(temperature=0.0)
        if i == 4:
            kw["stop"] = ["a"]
        if i == 5:
            kw["stop_token_ids"] = [p[-1]]
        reqs.append(Request(p, sp, max_tokens=int(rng.integers(1, 24)), **kw))
    return reqs


@pytest.mark.parametrize("max_tokens_budget", [64, 16])
def test_overlap_mode_matches_sync(model, max_tokens_budget):
    """Overlap mode (step N launched before step N-1's tokens are read; decode inputs gathered on the
    device) must produce exactly the synchronous engine's outputs, incl. length / stop-string /
    stop-token finishes, seeded sampling, logit bias, chunked prefill and preemption (small cache)."""
    for kw in ({}, dict(num_blocks=24)):
        e_sync, _ = mk(model, overlap=False, max_batched_tokens=max_tokens_budget, **kw)
        e_ovl, _ = mk(model, overlap=True, max_batched_tokens=max_tokens_budget, **kw)
        assert e_ovl.overlap and not e_sync.overlap
        a = _run_all(e_sync, _mixed_requests())
        b = _run_all(e_ovl, _mixed_requests())
        assert a == b
        # every block returned once everything finished
        assert e_ovl.bm.num_free == e_sync.bm.num_free
        assert not e_ovl.sched.deferred and not e_ovl._inflight


def _penalty_requests(seed=3):
    rng = np.random.default_rng(seed)
    reqs = []
    for i in range(8):
        p = [int(x) for x in rng.integers(1, 250, size=int(rng.integers(5, 60)))]
        if i % 4 == 0:
            sp = SamplingParams(temperature=0.0, frequency_penalty=0.7, presence_penalty=0.3, repeat_last_n=16)
        elif i % 4 == 1:
            sp = SamplingParams(temperature=0.8, top_k=40, top_p=0.9, repeat_penalty=1.3, seed=50 + i)
        elif i % 4 == 2:
            sp = SamplingParams(temperature=0.0, repeat_penalty=1.5, repeat_last_n=1, logit_bias={9: 1.0})
        else:
            sp = SamplingParams(temperature=0.0)
        reqs.append(Request(p, sp, max_tokens=int(rng.integers(4, 24))))
    return reqs


def test_penalties_stay_on_overlap_pipeline(model):
    """Repeat / presence / frequency penalties no longer force synchronous steps: the sampler counts each
    row's still-in-flight previous token on the device (ops/sampling.py pack, `pend`), so the overlap engine
    gives exactly the synchronous outputs while every step launches overlapped."""
    e_sync, _ = mk(model, overlap=False, max_batched_tokens=64)
    e_ovl, _ = mk(model, overlap=True, max_batched_tokens=64)
    a = _run_all(e_sync, _penalty_requests())
    b = _run_all(e_ovl, _penalty_requests())
    assert a == b
    assert e_ovl.stats.get("overlap_steps", 0) > 0 and e_ovl.stats.get("sync_steps", 0) == 0, e_ovl.stats


def test_grammar_rows_stay_on_overlap_pipeline(model):
    """Grammar-constrained rows mixed with plain rows stay in every overlapped step: the step's forward is
    launched first, the previous step (whose token the mask needs) is read while it runs, then the sampler is
    launched with the current mask. No synchronous steps; outputs equal the synchronous engine's."""
    from localai_tfp_amd.runtime_native import GrammarMatcher, NativeGrammar, NativeVocab
    tok = ByteTokenizer(model.cfg.vocab)
    tb = [bytes([i]) if i < 256 else b"" for i in range(model.cfg.vocab)]
    vocab = NativeVocab(tb)
    g = NativeGrammar('root ::= "{" "\\"a\\"" ":" [0-9]{1,3} "}"')

    def reqs():
        rng = np.random.default_rng(11)
        out = []
        for i in range(8):
            p = [int(x) for x in rng.integers(1, 250, size=int(rng.integers(5, 40)))]
            if i % 2 == 0:
                out.append(Request(p, SamplingParams(temperature=0.0), max_tokens=12,
                                   grammar=lambda: GrammarMatcher(g, vocab, tb, tok.eos_token_id)))
            else:
                out.append(Request(p, SamplingParams(temperature=0.7, top_k=20, seed=i), max_tokens=12))
        return out

    e_sync, _ = mk(model, overlap=False, max_batched_tokens=64)
    e_ovl, _ = mk(model, overlap=True, max_batched_tokens=64)
    a = _run_all(e_sync, reqs())
    b = _run_all(e_ovl, reqs())
    assert a == b
    for i in range(0, 8, 2):  # the grammar rows produced valid documents
        txt = a[i][1]
        assert txt.startswith('{"a":') and txt.endswith("}"), txt
    assert e_ovl.stats.get("overlap_steps", 0) > 0 and e_ovl.stats.get("sync_steps", 0) == 0, e_ovl.stats


@pytest.mark.parametrize("depth", [1, 3])
def test_overlap_depth_matches_sync(model, depth):
    """Deeper overlap pipelines (several launched-but-unread steps) give the synchronous outputs too."""
    e_sync, _ = mk(model, overlap=False, max_batched_tokens=64)
    e_ovl, _ = mk(model, overlap=True, max_batched_tokens=64, overlap_depth=depth)
    assert _run_all(e_sync, _mixed_requests()) == _run_all(e_ovl, _mixed_requests())
    assert e_ovl.bm.num_free == e_sync.bm.num_free and not e_ovl._inflight


def test_overlap_abort_mid_flight(model):
    e, tok = mk(model, overlap=True)
    free0 = e.bm.num_free
    r1 = Request(list(range(20, 60)), SamplingParams(temperature=0.0), max_tokens=40)
    r2 = Request(list(range(70, 90)), SamplingParams(temperature=0.0), max_tokens=8)
    h1, h2 = e.submit(r1), e.submit(r2)
    e._drain_inbox()
    for _ in range(6):
        e.step()
    e.abort(r1.rid)
    e.run_until_done()
    outs1 = []
    while not h1.q.empty():
        outs1.append(h1.q.get_nowait())
    assert outs1[-1].finished and outs1[-1].finish_reason == "abort"
    assert e.bm.num_free == free0 or e.cfg.enable_prefix_cache  # cached blocks may stay resident
    assert not e.sched.deferred and not e._inflight


@pytest.mark.parametrize("native", [False, True])
def test_step_failure_frees_deferred(model, native, monkeypatch):
    """a step that raises while a finished sequence is deferred (its blocks still awaited by an
    in-flight step) must free those blocks — the in-flight results are dropped and will never be read back."""
    monkeypatch.setenv("MX_PY_SCHED", "0" if native else "1")
    e, tok = mk(model, overlap=True, overlap_depth=3, enable_prefix_cache=False)
    assert e.native_sched == native or not native
    free0 = e.bm.num_free
    r1 = Request(list(range(20, 60)), SamplingParams(temperature=0.0), max_tokens=40)
    r2 = Request(list(range(70, 90)), SamplingParams(temperature=0.0), max_tokens=40)
    e.submit(r1), e.submit(r2)
    e._drain_inbox()
    for _ in range(4):
        e.step()
    e.abort(r2.rid)
    e._drain_inbox()
    e.step()  # r2 leaves the running set with samples still in flight -> deferred
    assert e.sched.deferred and e._inflight
    e._fail_step(RuntimeError("injected"))
    assert not e.sched.deferred and not e._inflight
    assert not e.sched.running and not e.sched.waiting
    assert e.bm.num_free == free0
