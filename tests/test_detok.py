"""Byte-level streaming detokenisation (engine/sequence.py `_decode_bytes` over the tokenizer's stream_bytes table):
token by token, the emitted pieces concatenate to the full decode, multi-byte characters split across tokens are
held back until complete, special tokens emit nothing."""
import numpy as np

from localai_tfp_amd.engine.sequence import Request, Sequence, _utf8_incomplete_tail


def test_incomplete_tail():
    assert _utf8_incomplete_tail(b"abc") == 0
    s = "é日😀".encode()
    assert _utf8_incomplete_tail(s) == 0
    assert _utf8_incomplete_tail(s[:-1]) == 3      # 4-byte emoji missing its last byte
    assert _utf8_incomplete_tail(s[:1]) == 1       # lead byte of é
    assert _utf8_incomplete_tail(b"\\x80") == 0     # stray continuation: decoded with replacement, not held


def test_stream_matches_full_decode():
    from localai_tfp_amd.tokenizer.synth_bpe import llama3_like_tokenizer
    tok = llama3_like_tokenizer()
    text = "streaming café 日本語 😀 tokens — 1234! " * 3
    ids = tok.encode(text, add_special=False)
    rng = np.random.default_rng(0)
    # interleave byte-fallback-like splits: random single-byte tokens of a multi-byte character
    seq = Sequence(Request(prompt_ids=[1, 2, 3]), tok)
    out = []
    for i, t in enumerate(ids):
        seq.append_token(t, None)
        out.append(seq._decode_new())
        if i % 7 == 3:  # a special token in the stream emits nothing
            sp = next(iter(tok.special_ids.values()))
            seq.append_token(sp, None)
            out.append(seq._decode_new())
    assert "".join(out) == tok.decode(ids) == text
    assert rng is not None


def test_final_flush_emits_partial_character():
    """a generation that stops (max_tokens) in the middle of a multi-byte character must not silently
    drop the held bytes — the final flush emits them as U+FFFD, like a full decode with errors='replace'."""
    from localai_tfp_amd.tokenizer import ByteTokenizer
    from localai_tfp_amd.tokenizer.synth_bpe import llama3_like_tokenizer
    for tok in (ByteTokenizer(512), llama3_like_tokenizer()):  # decode-based and byte-table streaming
        seq = Sequence(Request(prompt_ids=[1, 2, 3]), tok)
        raw = "ab日".encode()[:-1]  # cut inside the 3-byte character
        if hasattr(tok, "stream_bytes"):  # the vocabulary's single-byte tokens
            table = tok.stream_bytes()
            ids = [table.index(bytes([b])) for b in raw]
        else:
            ids = list(raw)
        for t in ids:
            seq.append_token(t, None)
        text, stop = seq.flush_text(final=False)
        tail, stop2 = seq.flush_text(final=True)
        assert not stop and not stop2
        assert text + tail == "ab\ufffd" and seq.emitted_text == "ab\ufffd", (type(tok).__name__, text, tail)
