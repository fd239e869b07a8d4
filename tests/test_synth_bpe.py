"""CPU check of the synthetic Llama-3-sized BPE vocabulary used by bench.py."""


def test_synthetic_bpe_vocabulary():
    from localai_tfp_amd.tokenizer.synth_bpe import llama3_like_tokenizer
    tok = llama3_like_tokenizer()
    assert tok.vocab_size == 128256
    s = "the model serves tokens fast on MI355X — café 日本語 😀 1234!"
    ids = tok.encode(s, add_special=False)
    assert tok.decode(ids) == s
    assert max(ids) < 128000
    assert tok.eos_token_ids == [128009]
    # incremental detokenisation must survive tokens that end inside a UTF-8 character
    pieces = b"".join(tok.token_bytes()[i] for i in ids)
    assert pieces.decode("utf-8") == s
