import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import GGUFReader, GGUFWriter, QType
from localai_tfp_amd.ops import quant as Q


@pytest.mark.parametrize("qt,tol", [(QType.Q4_K, 0.12), (QType.Q6_K, 0.03), (QType.Q8_0, 0.01)])
def test_quantize_roundtrip(qt, tol):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((16, 512), dtype=np.float32)
    raw = Q.QUANTIZERS[qt](x)
    y = Q.dequantize(raw, qt, (512, 16))
    err = np.linalg.norm(y - x) / np.linalg.norm(x)
    assert err < tol, err


def test_q4k_scale_pack_roundtrip():
    rng = np.random.default_rng(1)
    sc = rng.integers(0, 64, size=(100, 8))
    mn = rng.integers(0, 64, size=(100, 8))
    packed = Q._pack_q4k_scales(sc, mn)
    s2, m2 = Q.q4k_scale_min(packed)
    assert np.array_equal(s2.astype(int), sc) and np.array_equal(m2.astype(int), mn)


def _decode_q6k_repacked(blocks, d):
    """inverse of repack_q6_k: per block -> 256 signed codes * scale"""
    nb = blocks.shape[0]
    out = np.empty((nb, 256), np.float32)
    dd = d.view(np.float16).astype(np.float32).reshape(-1)
    for g in range(4):
        ql = blocks[:, 32 * g:32 * g + 32].astype(np.int32)
        qh = blocks[:, 128 + 16 * g:128 + 16 * g + 16].astype(np.int32)
        sc = blocks[:, 192 + 4 * g:192 + 4 * g + 4].view(np.int8).astype(np.float32)
        for e in range(64):
            lo = (ql[:, e % 32] >> (4 * (e // 32))) & 0xF
            hi = (qh[:, e % 16] >> (2 * (e // 16))) & 3
            q = (lo | (hi << 4)) - 32
            out[:, 64 * g + e] = q * sc[:, e // 16] * dd
    return out


def test_q6k_repack_is_lossless():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((4, 512), dtype=np.float32)
    raw = Q.quantize_q6_k(x)
    ref = Q.dequantize(raw, QType.Q6_K, (512, 4)).reshape(-1, 256)
    blocks, d = Q.repack_q6_k(raw, 4, 512)
    got = _decode_q6k_repacked(blocks.reshape(-1, 208), d.reshape(-1).view(np.uint16))
    assert np.allclose(got, ref, atol=1e-6)


def test_random_quantized_stats():
    rng = np.random.default_rng(3)
    for qt in (QType.Q4_K, QType.Q6_K, QType.Q8_0):
        raw = Q.random_quantized(rng, qt, 64, 1024, std=0.02)
        y = Q.dequantize(raw, qt, (1024, 64))
        assert np.isfinite(y).all()
        assert 0.01 < y.std() < 0.04, (qt, y.std())
        assert abs(y.mean()) < 0.005


def test_interleave_rows16():
    a = np.arange(32 * 3).reshape(32, 3)
    b = -np.arange(32 * 3).reshape(32, 3)
    c = Q.interleave_rows16(a, b)
    assert np.array_equal(c[:16], a[:16]) and np.array_equal(c[16:32], b[:16]) and np.array_equal(c[32:48], a[16:])


def test_other_dequantizers_finite():
    rng = np.random.default_rng(4)
    for qt in (QType.Q4_0, QType.Q4_1, QType.Q5_0, QType.Q5_1, QType.Q2_K, QType.Q3_K, QType.Q5_K):
        from localai_tfp_amd.formats.gguf import BLOCK
        be, bb = BLOCK[qt]
        raw = rng.integers(0, 256, size=(8, bb), dtype=np.uint8)
        # make fp16 scale fields finite and small
        y = Q.dequantize(raw.reshape(-1), qt, (be * 8,))
        assert y.shape == (be * 8,)


def test_q4_0_known_values():
    # one block: d = 1.0, nibbles 0..15 -> values -8..7
    blk = np.zeros(18, np.uint8)
    blk[0:2] = np.array([1.0], np.float16).view(np.uint8)
    qs = np.arange(16, dtype=np.uint8)
    blk[2:18] = qs | (qs << 4)
    y = Q.dequantize(blk, QType.Q4_0, (32,))
    assert np.array_equal(y[:16], np.arange(16) - 8) and np.array_equal(y[16:], np.arange(16) - 8)


def test_gguf_roundtrip(tmp_path):
    rng = np.random.default_rng(5)
    w = GGUFWriter(tmp_path / "t.gguf")
    w.add("general.architecture", "llama")
    w.add("llama.block_count", 2)
    w.add("llama.rope.freq_base", 10000.0)
    w.add("tokenizer.ggml.tokens", ["a", "b", "<s>"])
    w.add("tokenizer.ggml.scores", np.array([0.1, 0.2, 0.0], np.float32))
    w.add("some.bool", True)
    dense = rng.standard_normal((3, 64), dtype=np.float32)
    w.add_tensor("dense", dense)
    q = Q.quantize_q4_k(rng.standard_normal((2, 256), dtype=np.float32))
    w.add_tensor("q4", q, shape=(256, 2), qtype=QType.Q4_K)
    w.write()
    r = GGUFReader(tmp_path / "t.gguf")
    assert r.metadata["llama.block_count"] == 2
    assert r.metadata["tokenizer.ggml.tokens"] == ["a", "b", "<s>"]
    assert r.metadata["some.bool"] is True
    assert np.allclose(r.tensor("dense"), dense)
    assert np.array_equal(r.tensor_bytes("q4"), q)
    assert r.tensors["q4"].shape == (256, 2)
    r.close()
