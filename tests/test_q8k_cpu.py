"""CPU checks of the Q8_K activation format (ggml quantize_row_q8_K semantics, the operand of the int8-MFMA
GEMM) and of the synthetic Llama-3-sized BPE vocabulary used by bench.py."""
import numpy as np
import torch

from localai_tfp_amd.ops import core as K
from localai_tfp_amd.ops import linear as L
from localai_tfp_amd.ops import quant as Q
from localai_tfp_amd.formats.gguf import QType


def _ggml_q8k(x: np.ndarray):
    """Direct transcription of ggml's scalar quantize_row_q8_K loop (per 256 block)."""
    out_q, out_d, out_bs = [], [], []
    for blk in x.reshape(-1, 256).astype(np.float32):
        amax, mx = np.float32(0), np.float32(0)
        for v in blk:
            if abs(v) > amax:
                amax, mx = np.float32(abs(v)), v
        if amax == 0:
            out_q.append(np.zeros(256, np.int8)), out_d.append(0.0), out_bs.append(np.zeros(16))
            continue
        iscale = np.float32(-127.0) / mx
        q = np.minimum(127, np.rint(iscale * blk)).astype(np.int8)
        out_q.append(q)
        out_d.append(np.float32(1.0) / iscale)
        out_bs.append(q.reshape(16, 16).astype(np.int32).sum(1))
    return np.stack(out_q), np.array(out_d, np.float32), np.stack(out_bs)


def test_q8k_ref_matches_ggml_loop():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal((3, 512)) * 2).astype(np.float32)
    x[1, 300] = -25.0
    x[2, :256] = 0
    a = K.Q8KAct.empty(3, 512, "cpu")
    K.quant_q8k_ref(torch.from_numpy(x), a)
    q, d, bs = _ggml_q8k(x)
    assert np.array_equal(a.q.numpy().reshape(-1, 256), q)
    assert np.array_equal(a.d.numpy().reshape(-1), d)
    assert np.array_equal(a.bs.numpy().reshape(-1, 16).astype(np.int32), bs)


def test_qmatmul8_cpu_reference():
    """The CPU branch of qmatmul8 is the fp32 product of the dequantised operands."""
    n, k = 64, 512
    raw = Q.random_quantized(np.random.default_rng(1), int(QType.Q4_K), n, k)
    W = L.QWeight.from_ggml(raw, int(QType.Q4_K), n, k, "cpu")
    x = torch.randn(5, k)
    a = K.Q8KAct.empty(5, k, "cpu")
    K.quant_q8k(x, a)
    out = torch.empty(5, n)
    L.qmatmul8(W, a, L.EPI_F32, out)
    ref = a.dequant() @ W.dense_f32().t()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5)
    assert float((out - x @ W.dense_f32().t()).norm() / out.norm()) < 2e-2


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
