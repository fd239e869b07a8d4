"""Native host runtime (libmxrt.so, csrc/runtime/*.cpp): block manager parity with the Python
reference implementation, GBNF matcher + vocabulary masks, vector store."""
import random

import numpy as np
import pytest

from localai_tfp_amd.engine.kv_cache import PyBlockManager

rn = pytest.importorskip("localai_tfp_amd.runtime_native")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from localai_tfp_amd import _build
    _build.build_runtime()


def test_block_manager_matches_python_reference():
    rng = random.Random(0)
    py, nat = PyBlockManager(64, 4), rn.NativeBlockManager(64, 4)
    live = []  # (py_blocks, nat_blocks)
    prompts = [[rng.randrange(50) for _ in range(rng.randrange(5, 40))] for _ in range(6)]
    for step in range(300):
        op = rng.random()
        if op < 0.5 and py.num_free > 12:
            toks = rng.choice(prompts)
            pb, ph = py.match_prefix(toks)
            nb, nh = nat.match_prefix(toks)
            assert len(pb) == len(nb) and len(nh) == len(nb)  # hash functions differ; structure must not
            need = (len(toks) + 3) // 4 - len(pb)
            pb = pb + py.allocate(need)
            nb = nb + nat.allocate(need)
            pp = ph[-1] if ph else b""
            npar = nh[-1] if nh else b""
            for i in range(len(ph), len(toks) // 4):
                pp = py.commit_full_block(pb[i], pp, toks[4 * i:4 * i + 4])
                npar = nat.commit_full_block(nb[i], npar, toks[4 * i:4 * i + 4])
                assert len(npar) == 16
            live.append((pb, nb))
        elif live:
            pb, nb = live.pop(rng.randrange(len(live)))
            py.release(pb)
            nat.release(nb)
        assert py.num_free == nat.num_free
    assert nat.stats()["hits"] == py.hits > 0
    with pytest.raises(MemoryError):
        nat.allocate(10_000)


def test_grammar_parse_errors():
    with pytest.raises(rn.GrammarError):
        rn.NativeGrammar('root ::= "unterminated')
    with pytest.raises(rn.GrammarError):
        rn.NativeGrammar("root ::= undefined-rule")


@pytest.mark.timeout(30)
def test_grammar_left_recursion_rejected():
    # direct, indirect and behind a nullable prefix: rejected at parse time (llama.cpp semantics),
    # instead of an exponential expansion when the matcher is created
    for src in ('root ::= root "a" | root "b" | "c"',
                'root ::= x "z"\nx ::= root "y" | "w"',
                'root ::= opt root "a" | "b"\nopt ::= "q"?'):
        with pytest.raises(rn.GrammarError, match="left recursion"):
            rn.NativeGrammar(src)
    # right recursion stays legal
    g = rn.NativeGrammar('root ::= "a" root | "c"')
    assert g is not None


def _allowed(m, V):
    mk = m.allowed_mask(V)
    return {i for i in range(V) if (int(mk[i // 32]) >> (i % 32)) & 1}


def test_mask_multibyte_tokens_and_utf8():
    # vocab: single bytes + some multi-byte pieces incl. a token ending mid code point
    tb = [bytes([i]) for i in range(256)] + [b"", "é".encode(), "é".encode()[:1], b"ab", b"abc", b"ba"]
    EOS = 256
    v = rn.NativeVocab(tb)
    g = rn.NativeGrammar('root ::= "ab" [é]+')
    m = rn.GrammarMatcher(g, v, tb, EOS)
    assert _allowed(m, len(tb)) == {ord("a"), 259}  # "a", "ab"; never a bare lead byte like 0xC1
    assert m.accept(259)
    allowed = _allowed(m, len(tb))
    assert allowed == {0xC3, 257, 258}  # lead byte, whole "é", and the token holding its first byte
    assert m.accept(258) and not m.is_done()
    assert _allowed(m, len(tb)) == {0xA9}
    assert m.accept(0xA9) and m.is_done()
    assert EOS in _allowed(m, len(tb))


def test_mask_unicode_range_and_negation():
    tb = [bytes([i]) for i in range(256)]
    v = rn.NativeVocab(tb)
    m = rn.GrammarMatcher(rn.NativeGrammar("root ::= [一-鿿]+"), v, tb)
    assert _allowed(m, 256) == set(range(0xE4, 0xEA))
    m = rn.GrammarMatcher(rn.NativeGrammar('root ::= [^"]*'), v, tb)
    a = _allowed(m, 256)
    assert ord('"') not in a and ord("x") in a and 0xC0 not in a and 0xC2 in a


def test_matcher_repetition_alternation():
    tb = [bytes([i]) for i in range(256)]
    g = rn.NativeGrammar('root ::= item ("," item){1,2}\nitem ::= [0-9]+ | "x"')
    for s, ok in [("1,2", True), ("1,x,33", True), ("1", False), ("1,2,3,4", False)]:
        m = rn.GrammarMatcher(g, rn.NativeVocab(tb), tb)
        assert (m.accept_bytes(s.encode()) and m.is_done()) == ok, s


def test_tokenizer_token_bytes_drive_matcher():
    from localai_tfp_amd.tokenizer import ByteTokenizer
    tok = ByteTokenizer(300)
    tb = tok.token_bytes()
    assert len(tb) == 300 and tb[65] == b"A" and tb[tok.eos_token_id] == b""
    m = rn.GrammarMatcher(rn.NativeGrammar('root ::= "yes" | "no"'), rn.NativeVocab(tb), tb, tok.eos_token_id)
    assert _allowed(m, 300) == {ord("y"), ord("n")}
    for t in tok.encode("no", add_special=False):
        assert m.accept(t)
    assert m.is_done() and tok.eos_token_id in _allowed(m, 300)


def test_vector_store():
    s = rn.NativeStore()
    rng = np.random.default_rng(0)
    keys = rng.standard_normal((50, 8)).astype(np.float32)
    s.set(keys, [f"v{i}".encode() for i in range(50)])
    assert len(s) == 50 and s.dim == 8
    ks, vs = s.get(keys[[3, 7]])
    assert vs == [b"v3", b"v7"] and np.allclose(ks[0], keys[3])
    q = keys[10] + 0.01
    _, vs, sims = s.find(q, 3)
    assert vs[0] == b"v10" and sims[0] > 0.99 and sims == sorted(sims, reverse=True)
    # overwrite + delete
    s.set(keys[:1], [b"new"])
    assert s.get(keys[:1])[1] == [b"new"] and len(s) == 50
    assert s.delete(keys[:5]) == 5 and len(s) == 45
    assert s.get(keys[:1]) == ([], [])
    with pytest.raises(ValueError):
        s.set(np.zeros((1, 4), np.float32), [b"x"])


def test_grammar_mask_batch_matches_rows():
    """mxrt_matcher_mask_batch (rows on several threads, memoised stack-set transitions) gives every row the
    mask the single-row call gives, along random walks through a JSON grammar over a byte + word vocabulary."""
    from localai_tfp_amd import functions as F
    from localai_tfp_amd.runtime_native import GrammarMatcher, NativeGrammar, NativeVocab
    words = [b"{", b"}", b"[", b"]", b'"', b'":', b", ", b"true", b"null", b"12", b"-3.5", b'"a', b'b"', b"\\n",
             "é".encode(), "日本".encode(), b"e+", b" ", b"\n"]
    tb = [bytes([i]) for i in range(256)] + words
    V = len(tb)
    vocab = NativeVocab(tb)
    g = NativeGrammar(F.JSON_BNF)
    rng = np.random.default_rng(5)
    ms = [GrammarMatcher(g, vocab, tb, -1) for _ in range(12)]
    W = (V + 31) // 32
    for _ in range(25):
        out = np.zeros((len(ms), W), np.uint32)
        GrammarMatcher.masks_into(ms, out, list(range(len(ms))))
        for i, m in enumerate(ms):
            assert (out[i] == m.allowed_mask(V)).all()
            allowed = np.flatnonzero(np.unpackbits(out[i].view(np.uint8), bitorder="little")[:V])
            if len(allowed):
                assert m.accept(int(rng.choice(allowed)))


def _mask_rows_ok(ms, V, steps, seed):
    from localai_tfp_amd.runtime_native import GrammarMatcher
    rng = np.random.default_rng(seed)
    W = (V + 31) // 32
    for _ in range(steps):
        out = np.zeros((len(ms), W), np.uint32)
        GrammarMatcher.masks_into(ms, out, list(range(len(ms))))
        for i, m in enumerate(ms):
            if not (out[i] == m.allowed_mask(V)).all():
                return False
            allowed = np.flatnonzero(np.unpackbits(out[i].view(np.uint8), bitorder="little")[:V])
            if len(allowed):
                m.accept(int(rng.choice(allowed)))
    return True


def _fork_child(q):
    from localai_tfp_amd import functions as F
    from localai_tfp_amd.runtime_native import GrammarMatcher, NativeGrammar, NativeVocab
    tb = [bytes([i]) for i in range(256)] + [b'{"', b'":', b"true", b", "]
    g = NativeGrammar(F.JSON_BNF)
    vocab = NativeVocab(tb)
    q.put(_mask_rows_ok([GrammarMatcher(g, vocab, tb, -1) for _ in range(6)], len(tb), 5, 1))


def test_grammar_mask_pool_concurrent_callers_and_fork():
    """The batched mask runs on a persistent worker pool (csrc/runtime/grammar.cpp MaskPool): concurrent callers are
    serialised, grammars freed between calls do not leak stale transition tables into later grammars, and a forked
    child (whose parent's workers do not exist) builds its own pool."""
    import multiprocessing as mp
    import threading
    from localai_tfp_amd import functions as F
    from localai_tfp_amd.runtime_native import GrammarMatcher, NativeGrammar, NativeVocab
    tb = [bytes([i]) for i in range(256)] + [b"{", b"}", b'"', b'":', b", ", b"true", b"12", b" "]
    V = len(tb)
    vocab = NativeVocab(tb)
    res = []

    def caller(seed):
        for k in range(4):  # a fresh grammar (new serial) each round, the old one freed
            g = NativeGrammar(F.JSON_BNF)
            res.append(_mask_rows_ok([GrammarMatcher(g, vocab, tb, -1) for _ in range(8)], V, 6, seed + k))

    ths = [threading.Thread(target=caller, args=(s,)) for s in (10, 20, 30)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert len(res) == 12 and all(res)
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_fork_child, args=(q,))
    p.start()
    p.join(timeout=120)
    assert p.exitcode == 0 and q.get(timeout=5) is True
