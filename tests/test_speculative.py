"""Speculative decoding (engine/speculative.py, N12): a draft model proposes k tokens, the target
verifies them in one prefill-style forward and keeps the longest prefix its own sampler agrees with.

Invariant tested (llama.cpp common_sampler_sample_and_accept_n semantics): the output stream is
exactly what plain decoding produces — greedy, and seeded sampling (the sampler's RNG is keyed by
(seed, step)) — whatever the draft proposes; only the number of target forwards changes."""
import numpy as np
import pytest

from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
from localai_tfp_amd.engine.sequence import Request
from localai_tfp_amd.models.config import tiny_config
from localai_tfp_amd.models.llama import LlamaModel
from localai_tfp_amd.models.synthetic import synthetic_source
from localai_tfp_amd.ops.sampling import SamplingParams
from localai_tfp_amd.tokenizer import ByteTokenizer


def _models(dev="cpu"):
    cfg = tiny_config(n_layers=2)
    target = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=11), dev)
    dcfg = tiny_config(n_layers=1)
    other = LlamaModel.load(dcfg, synthetic_source(dcfg, "Q4_K_M", seed=5), dev)
    return target, other


@pytest.fixture(scope="module")
def models():
    return _models()


def _engine(model, draft=None, n_draft=4, **kw):
    c = dict(num_blocks=256, max_num_seqs=8, max_batched_tokens=64, max_model_len=512, n_draft=n_draft)
    c.update(kw)
    return LLMEngine(model, ByteTokenizer(model.cfg.vocab), EngineConfig(**c), draft=draft)


def _run(eng, prompts, sp, max_tokens):
    hs = [eng.submit(Request(list(p), sp, max_tokens)) for p in prompts]
    eng.run_until_done(max_steps=10000)
    out = []
    for h in hs:
        ids = []
        for o in h:
            ids += o.token_ids
        out.append(ids)
    return out


PROMPTS = [list(range(10 + i, 40 + 3 * i)) for i in range(4)]


@pytest.mark.parametrize("which", ["self", "other"])
def test_greedy_output_independent_of_draft(models, which):
    target, other = models
    draft = target if which == "self" else other
    sp = SamplingParams(temperature=0.0, ignore_eos=True)
    ref = _run(_engine(target), PROMPTS, sp, 20)
    eng = _engine(target, draft, n_draft=4)
    got = _run(eng, PROMPTS, sp, 20)
    assert got == ref
    st = eng.spec.stats
    assert st["spec_steps"] > 0
    rate = st["accepted"] / max(1, st["drafted"])
    if which == "self":
        assert rate > 0.9, st  # the target drafting for itself: (almost) everything accepted
        assert eng.stats["steps"] < 20 + 8  # far fewer target steps than tokens


def test_seeded_sampling_identical(models):
    target, _ = models
    sp = SamplingParams(temperature=0.9, top_k=40, top_p=0.95, seed=1234, ignore_eos=True)
    ref = _run(_engine(target), PROMPTS[:2], sp, 16)
    got = _run(_engine(target, target, n_draft=3), PROMPTS[:2], sp, 16)
    assert got == ref


def test_limits_stops_and_per_request_cap(models):
    target, other = models
    tok = ByteTokenizer(target.cfg.vocab)
    eng = _engine(target, target, n_draft=5)
    # max_tokens not a multiple of k+1 is honoured exactly
    for n in (1, 2, 7, 13):
        o = eng.generate(PROMPTS[0], SamplingParams(temperature=0.0, ignore_eos=True), max_tokens=n)
        assert len(o.token_ids) == n and o.finish_reason == "length"
    # stop strings cut the accepted run
    plain = _engine(target).generate(PROMPTS[1], SamplingParams(temperature=0.0, ignore_eos=True), max_tokens=16)
    if len(plain.text) >= 6:
        stop = plain.text[4:6]
        o = eng.generate(PROMPTS[1], SamplingParams(temperature=0.0, ignore_eos=True), max_tokens=16, stop=[stop])
        assert o.finish_reason == "stop" and o.text == plain.text[: plain.text.find(stop)]
    # per-request n_draft cap
    e2 = _engine(target, target, n_draft=6)
    r = Request(list(PROMPTS[2]), SamplingParams(temperature=0.0, ignore_eos=True), 12)
    r.n_draft = 1
    h = e2.submit(r)
    e2.run_until_done()
    assert sum(len(o.token_ids) for o in h) == 12
    assert e2.spec.stats["drafted"] == e2.spec.stats["spec_steps"]  # one draft token per step


def test_preemption_and_prefix_cache(models):
    target, other = models
    sp = SamplingParams(temperature=0.0, ignore_eos=True)
    prompts = [list(range(5 + i, 50 + i)) for i in range(4)]
    ref = _run(_engine(target, enable_prefix_cache=False), prompts, sp, 12)
    eng = _engine(target, other, n_draft=3, num_blocks=14, enable_prefix_cache=False, max_batched_tokens=256)
    assert _run(eng, prompts, sp, 12) == ref
    assert eng.stats["preemptions"] > 0
    # shared prefixes: the second request reuses cached target blocks; its draft catches up itself
    eng = _engine(target, target, n_draft=3)
    a = eng.generate(prompts[0], sp, max_tokens=10)
    b = eng.generate(prompts[0], sp, max_tokens=10)
    assert a.token_ids == b.token_ids == ref[0][:10] and b.cached_tokens > 0


def test_worker_loads_draft_model():
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    s = LLMServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:tiny", DraftModel="synthetic:tiny-draft",
                                    Options=["lazy_graphs", "n_draft:3"]), None)
    assert r.success, r.message
    assert s.engine.spec is not None and s.engine.spec.k == 3
    req = s._request(pb.PredictOptions(Prompt="hello speculative world", Tokens=9, NDraft=2, IgnoreEOS=True))
    assert req.n_draft == 2
    s.engine.shutdown()


@pytest.mark.gpu
def test_speculative_gpu():
    target, other = _models("cuda")
    sp = SamplingParams(temperature=0.0, ignore_eos=True)
    ref = _run(_engine(target), PROMPTS, sp, 24)
    eng = _engine(target, target, n_draft=4)
    got = _run(eng, PROMPTS, sp, 24)
    st = eng.spec.stats
    assert st["spec_steps"] > 0 and st["accepted"] / st["drafted"] > 0.6, st
    # verification runs the prefill kernels, plain decoding the GEMV path: streams agree until a
    # near-tie flips; require a long common prefix on every request
    for a, b in zip(got, ref):
        assert len(a) == 24
        n = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), 24)
        assert n >= 8, (a, b)
    got2 = _run(_engine(target, other, n_draft=3), PROMPTS, sp, 24)
    assert all(len(a) == 24 for a in got2)
