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
