"""HIP kernel numerics vs plain PyTorch fp32 references of the same op (run on MI355X)."""
import math

import numpy as np
import pytest
import torch

from localai_tfp_amd import _native as N
from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import core as K
from localai_tfp_amd.ops import quant as Q
from localai_tfp_amd.ops.linear import EPI_ADD_F32, EPI_BF16, EPI_F32, EPI_SWIGLU, QWeight, qmatmul

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def make_w(qt, n, k, seed=0):
    rng = np.random.default_rng(seed)
    if QType(qt) not in Q.QUANTIZERS:  # Q2_K / Q3_K: random blocks in the quantised domain
        raw = Q.random_quantized(rng, int(qt), n, k, std=0.05)
        dense = Q.dequantize(raw, qt, (k, n))
        return raw.reshape(n, -1), torch.from_numpy(dense)
    x = rng.standard_normal((n, k), dtype=np.float32) * 0.05
    raw = Q.QUANTIZERS[QType(qt)](x)
    dense = Q.dequantize(raw, qt, (k, n))
    return raw.reshape(n, -1), torch.from_numpy(dense)


def test_native_loaded():
    lib = N.kernels()
    assert lib is not None
    assert any("libmxk.so" in p for p in N.loaded_library_paths())


@pytest.mark.parametrize("H", [4096, 2048, 5120, 320])
def test_rmsnorm(H):
    torch.manual_seed(0)
    M = 7
    x = torch.randn(M, H, device=DEV) * 3
    w = torch.rand(H, device=DEV) + 0.5
    ob = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    xq = torch.empty(M, H, dtype=torch.int8, device=DEV)
    xds = torch.empty(M, H // 32, 2, device=DEV)
    K.rmsnorm(x, w, 1e-5, out_bf16=ob, out_q8=(xq, xds))
    ref = (x.cpu() * torch.rsqrt(x.cpu().pow(2).mean(-1, keepdim=True) + 1e-5) * w.cpu())
    assert rel(ob, ref) < 5e-3
    deq = xq.float().cpu().reshape(M, H // 32, 32) * xds.cpu()[:, :, :1]
    assert rel(deq.reshape(M, H), ref) < 1.5e-2
    s = xds.cpu()[:, :, 1]
    assert torch.allclose(s, xds.cpu()[:, :, 0] * xq.cpu().float().reshape(M, H // 32, 32).sum(-1), rtol=1e-4, atol=1e-4)


def test_quant_q8():
    x = (torch.randn(5, 14336, device=DEV) * 2).bfloat16()
    xq = torch.empty(5, 14336, dtype=torch.int8, device=DEV)
    xds = torch.empty(5, 14336 // 32, 2, device=DEV)
    K.quant_q8(x, xq, xds)
    xq_r = torch.empty(5, 14336, dtype=torch.int8)
    xds_r = torch.empty(5, 14336 // 32, 2)
    K.quant_q8(x.cpu(), xq_r, xds_r)
    assert (xq.cpu().int() - xq_r.int()).abs().max() <= 1
    assert torch.allclose(xds.cpu()[..., 0], xds_r[..., 0], rtol=1e-5)


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
def test_dequant_rows(qt):
    raw, dense = make_w(qt, 48, 1024, seed=int(qt))
    W = QWeight.from_ggml(raw, qt, 48, 1024, DEV)
    out = W.dequant_gpu(torch.float32)
    assert torch.allclose(out.cpu(), dense, atol=1e-6, rtol=1e-3)
    rows = torch.tensor([3, 0, 47, 3], dtype=torch.int32, device=DEV)
    sel = W.dequant_gpu(torch.float32, rows)
    assert torch.allclose(sel.cpu(), dense[[3, 0, 47, 3]], atol=1e-6, rtol=1e-3)


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_qgemv(qt, M):
    n, k = 512, 4096
    raw, dense = make_w(qt, n, k, seed=M)
    W = QWeight.from_ggml(raw, qt, n, k, DEV)
    x = torch.randn(M, k, device=DEV).half()
    xq = torch.empty(M, k, dtype=torch.int8, device=DEV)
    xds = torch.empty(M, k // 32, 2, device=DEV)
    K.quant_q8(x.bfloat16(), xq, xds)
    xd = xq.float().cpu().reshape(M, k // 32, 32) * xds.cpu()[:, :, :1]
    ref = xd.reshape(M, k) @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, None, EPI_F32, out, xq=xq, xds=xds)
    assert rel(out, ref) < 2e-3
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, None, EPI_ADD_F32, acc, xq=xq, xds=xds)  # split-K over workgroups (atomics)
    assert rel(acc - acc0, ref) < 2e-3
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, None, EPI_F32, z, xq=xq, xds=xds, out_zeroed=True)
    assert rel(z, ref) < 2e-3
    sw = torch.empty(M, n // 2, dtype=torch.bfloat16, device=DEV)
    qmatmul(W, None, EPI_SWIGLU, sw, xq=xq, xds=xds)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
@pytest.mark.parametrize("M", [5, 16, 33, 64, 100, 257])
def test_qgemm_mfma(qt, M):
    n, k = 384, 2048
    raw, dense = make_w(qt, n, k, seed=M + 7)
    W = QWeight.from_ggml(raw, qt, n, k, DEV)
    x = torch.randn(M, k, device=DEV).bfloat16()
    ref = x.float().cpu() @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, out)
    assert rel(out, ref) < 1e-2
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, z, out_zeroed=True)  # may split-K through atomics
    assert rel(z, ref) < 1e-2
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, x, EPI_ADD_F32, acc)
    assert rel(acc - acc0, ref) < 1e-2
    ob = torch.empty(M, n, dtype=torch.bfloat16, device=DEV)
    qmatmul(W, x, EPI_BF16, ob)
    assert rel(ob, ref) < 1.5e-2
    sw = torch.empty(M, n // 2, dtype=torch.bfloat16, device=DEV)
    qmatmul(W, x, EPI_SWIGLU, sw)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 2e-2


def test_qgemm_strided_out_and_lda():
    qt = QType.Q4_K
    raw, dense = make_w(qt, 256, 1024, seed=3)
    W = QWeight.from_ggml(raw, qt, 256, 1024, DEV)
    xb = torch.randn(20, 2048, device=DEV).bfloat16()
    x = xb[:, :1024]
    big = torch.zeros(20, 600, device=DEV)
    qmatmul(W, x, EPI_F32, big[:, 100:356])
    ref = x.float().cpu() @ dense.t()
    assert rel(big[:, 100:356], ref) < 1e-2
    assert float(big[:, :100].abs().sum()) == 0.0


def _rope_setup(T, Hq, Hkv, D, nb, bs, seed=0):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, generator=g)
    pos = torch.randint(0, 3000, (T,), generator=g, dtype=torch.int32)
    slots = torch.randperm(nb * bs, generator=g)[:T].to(torch.int32)
    slots[0] = -1
    return qkv, pos, slots


@pytest.mark.parametrize("qkn", [False, True])
@pytest.mark.parametrize("neox", [False, True])
@pytest.mark.parametrize("D,rot", [(128, 128), (64, 64), (128, 64)])
def test_rope_kv(neox, D, rot, qkn):
    """RoPE + KV append (the vectorised kernel for rot == D in {64, 128}, incl. the QK-norm form; the general kernel
    for partial rotation) against the fp32 CPU path."""
    T, Hq, Hkv, nb, bs = 9, 8, 2, 8, 16
    qkv, pos, slots = _rope_setup(T, Hq, Hkv, D, nb, bs)
    bias = torch.randn((Hq + 2 * Hkv) * D) * 0.1
    inv, af = K.rope_inv_freq(rot, 500000.0)
    g = torch.Generator().manual_seed(5)
    nq, nk = 1 + 0.3 * torch.randn(D, generator=g), 1 + 0.3 * torch.randn(D, generator=g)
    outs = []
    for dev in ("cpu", DEV):
        q = torch.empty(T, Hq, D, dtype=torch.bfloat16, device=dev)
        kc = torch.zeros(nb, Hkv, bs, D, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        K.rope_kv(qkv.to(dev), bias.to(dev), pos.to(dev), slots.to(dev), inv.to(dev), af, Hq, Hkv, D, rot, neox, q, kc, vc, bs,
                  qk_norm=(nq.to(dev), nk.to(dev), 1e-6) if qkn else None)
        outs.append((q.cpu(), kc.cpu(), vc.cpu()))
    if qkn:
        for a, b in zip(*outs):
            assert rel(b, a) < 1e-2
        return
    for a, b in zip(*outs):
        assert rel(b, a) < 1e-2
    # zero_after: the fp32 QKV rows are handed back zeroed (the next split-K GEMM accumulates into them)
    qd = qkv.to(DEV)
    q = torch.empty(T, Hq, D, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(nb, Hkv, bs, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    K.rope_kv(qd, bias.to(DEV), pos.to(DEV), slots.to(DEV), inv.to(DEV), af, Hq, Hkv, D, rot, neox, q, kc, vc, bs,
              zero_after=True)
    assert int((qd != 0).sum()) == 0
    for a, b in zip(outs[0], (q.cpu(), kc.cpu(), vc.cpu())):
        assert rel(b, a) < 1e-2


def _paged_kv(nb, Hkv, bs, D, seed):
    g = torch.Generator().manual_seed(seed)
    kc = (torch.randn(nb, Hkv, bs, D, generator=g)).bfloat16()
    vc = (torch.randn(nb, Hkv, bs, D, generator=g)).bfloat16()
    return kc, vc


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 8, 128), (28, 4, 128), (32, 8, 64), (64, 8, 128)])
@pytest.mark.parametrize("lens", [[1, 17, 300], [1200, 5, 2049]])
@pytest.mark.parametrize("impl", ["mfma", "valu"])
def test_attn_decode(Hq, Hkv, D, lens, impl):
    bs, nb = 16, 512
    kc, vc = _paged_kv(nb, Hkv, bs, D, 1)
    B = len(lens)
    maxb = max((l + bs - 1) // bs for l in lens)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    perm = torch.randperm(nb - 1)[: B * maxb] + 1
    for b in range(B):
        bt[b] = perm[b * maxb:(b + 1) * maxb].int()
    seq = torch.tensor(lens, dtype=torch.int32)
    q = torch.randn(B, Hq, D).bfloat16()
    scale = 1 / math.sqrt(D)
    ref = torch.empty(B, Hq, D)
    K.attn_decode(q, kc, vc, bt, seq, scale, ref)
    for part in (512, 128, 64):
        out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=DEV)
        K.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), seq.to(DEV), scale, out, part_size=part,
                      impl=impl)
        assert rel(out, ref) < 1e-2, part
    # graph-style launch: partition count for a long max_seq_len, most partitions empty; 512-key partitions run
    # the 16-wave single-pass form at B < 8 (sequences of <= 512 keys written directly, the reduce skips them)
    for part in (256, 512):
        out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=DEV)
        nparts = -(-4096 // part)
        ws = (torch.empty(B * Hq * nparts, 2, device=DEV), torch.empty(B * Hq * nparts, D, device=DEV))
        K.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), seq.to(DEV), scale, out, part_size=part,
                      workspace=ws, max_seq_len=4096, impl=impl)
        assert rel(out, ref) < 1e-2, part
    # the opt-in in-kernel partition merge (MFMA path): arrival counters reset themselves across launches
    K.FUSED_DECODE_MERGE, saved = True, K.FUSED_DECODE_MERGE
    cnt = torch.zeros(B * Hkv, dtype=torch.int32, device=DEV)
    nparts = -(-4096 // 64)
    ws = (torch.empty(B * Hq * nparts, 2, device=DEV), torch.empty(B * Hq * nparts, D, device=DEV))
    for part in (64, 256, 512, 64):
        out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=DEV)
        K.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), seq.to(DEV), scale, out, part_size=part,
                      workspace=ws + (cnt,), max_seq_len=4096, impl=impl)
        assert rel(out, ref) < 1e-2, part
        assert int(cnt.abs().sum()) == 0
    K.FUSED_DECODE_MERGE = saved


def test_probe_tr16_semantics():
    out = torch.zeros(256, dtype=torch.int16, device=DEV)
    N.kcall("mxk_probe_tr16", out.data_ptr(), N.stream_ptr())
    got = out.cpu().view(64, 4).tolist()
    # expected (guide §5.5 T10): lane i of a 16-lane group receives column i of the group's 4 rows
    exp = [[(4 * (l >> 4) + e) * 16 + (l & 15) for e in range(4)] for l in range(64)]
    print("tr16 lanes 0..7:", got[:8])
    assert got == exp


@pytest.mark.parametrize("vmode", [0, 1])
@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 8, 128), (16, 8, 128), (28, 4, 128), (32, 8, 64), (64, 8, 128)])
def test_attn_prefill(Hq, Hkv, D, vmode):
    bs, nb = 16, 256
    kc, vc = _paged_kv(nb, Hkv, bs, D, 2)
    q_lens = [37, 1, 130, 64]
    ctx = [37, 20, 300, 64]  # seq 1 and 2 have cached prefixes
    S = len(q_lens)
    maxb = max((c + bs - 1) // bs for c in ctx)
    bt = torch.zeros(S, maxb, dtype=torch.int32)
    perm = torch.randperm(nb - 1)[: S * maxb] + 1
    for s in range(S):
        bt[s] = perm[s * maxb:(s + 1) * maxb].int()
    cu = torch.tensor([0] + list(np.cumsum(q_lens)), dtype=torch.int32)
    T = int(cu[-1])
    q = torch.randn(T, Hq, D).bfloat16()
    ctx_t = torch.tensor(ctx, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    ref = torch.empty(T, Hq, D)
    K.attn_prefill(q, kc, vc, bt, cu, ctx_t, scale, ref, q_lens, ctx)
    out = torch.empty(T, Hq, D, dtype=torch.bfloat16, device=DEV)
    K.attn_prefill(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cu.to(DEV), ctx_t.to(DEV), scale, out, q_lens, ctx,
                   vmode=vmode)
    errs = []
    off = 0
    for s, ql in enumerate(q_lens):
        errs.append(round(rel(out[off:off + ql], ref[off:off + ql]), 4))
        off += ql
    assert rel(out, ref) < 1.5e-2, errs


def test_sampling_greedy_and_topk():
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    torch.manual_seed(0)
    V = 128256
    logits = torch.randn(6, V, device=DEV) * 3
    am = logits.argmax(-1).cpu()
    sb = SamplerBatch(DEV)
    ps = [SamplingParams(temperature=0.0)] * 3 + [SamplingParams(temperature=0.7, top_k=1)] * 3
    tok, _ = sb.sample(logits.clone(), ps, [[]] * 6, [0] * 6)
    assert torch.equal(tok.cpu().long(), am)
    # top-k=5: samples must be inside the top-5 set
    p5 = [SamplingParams(temperature=1.0, top_k=5, top_p=1.0, min_p=0.0, seed=i) for i in range(6)]
    top5 = logits.topk(5, -1).indices.cpu()
    for step in range(20):
        tok, lp = sb.sample(logits.clone(), p5, [[]] * 6, [step] * 6)
        for r in range(6):
            assert int(tok[r]) in top5[r].tolist()
        assert torch.all(lp.cpu() <= 0)


def test_sampling_distribution():
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    V = 1000
    logits = torch.full((1, V), -30.0, device=DEV)
    logits[0, :4] = torch.log(torch.tensor([0.1, 0.2, 0.3, 0.4], device=DEV))
    sb = SamplerBatch(DEV)
    cnt = np.zeros(4)
    for s in range(2000):
        tok, _ = sb.sample(logits.clone(), [SamplingParams(temperature=1.0, top_k=0, top_p=1.0, min_p=0.0, seed=s)], [[]], [0])
        cnt[int(tok[0])] += 1
    freq = cnt / cnt.sum()
    assert np.allclose(freq, [0.1, 0.2, 0.3, 0.4], atol=0.04), freq


def test_penalties_and_bias():
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    V = 5000
    logits = torch.zeros(1, V, device=DEV)
    logits[0, 10] = 5.0
    logits[0, 11] = 4.0
    sb = SamplerBatch(DEV)
    p = SamplingParams(temperature=0.0, repeat_penalty=2.0, repeat_last_n=8)
    tok, _ = sb.sample(logits.clone(), [p], [[10]], [0])
    assert int(tok[0]) == 11  # 5/2 < 4
    p2 = SamplingParams(temperature=0.0, logit_bias={42: 100.0})
    tok, _ = sb.sample(logits.clone(), [p2], [[]], [0])
    assert int(tok[0]) == 42


# ------------------------------------------------------------------------------------------------
# f16 activation path (qgemm16.hip packed-f16 dequant; f16 outputs of the producers)

@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
@pytest.mark.parametrize("M", [5, 16, 33, 64, 100, 128, 257])
def test_qgemm16(qt, M):
    n, k = 384, 2048
    raw, dense = make_w(qt, n, k, seed=M + 11)
    W = QWeight.from_ggml(raw, qt, n, k, DEV)
    x = torch.randn(M, k, device=DEV).half()
    ref = x.float().cpu() @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, out)
    assert rel(out, ref) < 5e-3
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, z, out_zeroed=True)
    assert rel(z, ref) < 5e-3
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, x, EPI_ADD_F32, acc)
    assert rel(acc - acc0, ref) < 5e-3
    ob = torch.empty(M, n, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_BF16, ob)
    assert rel(ob, ref) < 5e-3
    sw = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_SWIGLU, sw)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
@pytest.mark.parametrize("M,wm,wn,splits", [(48, 2, 1, 1), (77, 4, 2, 2), (128, 4, 1, 1), (128, 2, 2, 4),
                                             (200, 4, 2, 2), (33, 1, 1, 1)])
def test_qgemm32(qt, M, wm, wn, splits, monkeypatch):
    """qgemm32.hip (32x32x16 f16 MFMA tiles) for every epilogue and tile / split-K choice."""
    from localai_tfp_amd.ops import linear as L
    monkeypatch.setattr(L, "Q32_MIN_M", 1)
    monkeypatch.setattr(L, "Q32_FORCE", (wm, wn, splits))
    n, k = 512, 2048
    raw, dense = make_w(qt, n, k, seed=M + 3 * wm)
    W = QWeight.from_ggml(raw, qt, n, k, DEV)
    x = torch.randn(M, k, device=DEV).half()
    ref = x.float().cpu() @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, out)
    assert rel(out, ref) < 5e-3
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, z, out_zeroed=True)
    assert rel(z, ref) < 5e-3
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, x, EPI_ADD_F32, acc)
    assert rel(acc - acc0, ref) < 5e-3
    ob = torch.empty(M, n, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_BF16, ob)
    assert rel(ob, ref) < 5e-3
    sw = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_SWIGLU, sw)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q3_K, QType.Q2_K, QType.Q5_K, QType.Q8_0])
@pytest.mark.parametrize("M,wm,ks,wn,splits", [
    (64, 2, 1, 1, 1), (64, 2, 2, 1, 3), (17, 2, 2, 1, 1), (128, 4, 2, 1, 1), (77, 4, 2, 1, 2), (128, 4, 1, 1, 4),
    (256, 8, 1, 1, 1), (300, 8, 1, 1, 3), (511, 8, 1, 1, 1), (100, 2, 1, 1, 5),
    (64, 1, 2, 2, 1), (40, 1, 2, 2, 3), (128, 2, 1, 2, 1), (200, 2, 2, 2, 2), (256, 4, 1, 2, 1), (300, 4, 1, 2, 3),
    (511, 4, 1, 2, 2), (64, 2, 9, 1, 1), (300, 2, 10, 1, 3), (100, 2, 10, 1, 8), (40, 1, 10, 2, 1), (200, 1, 10, 2, 5),
    (384, 6, 1, 1, 1), (250, 6, 2, 1, 2), (400, 3, 2, 2, 3), (448, 7, 1, 1, 1), (300, 7, 1, 1, 3),
    # ks 17: wide tiles (8 column groups per workgroup; 416 columns = 1.625 tiles)
    (128, 4, 17, 1, 1), (300, 4, 17, 1, 3), (384, 6, 17, 1, 1), (250, 6, 17, 1, 2), (400, 3, 17, 2, 1),
    (64, 2, 17, 1, 2), (100, 2, 17, 1, 1), (448, 7, 17, 1, 1), (300, 7, 17, 1, 2),
    # ks 18: 4-wave wide tiles (2 column groups per wave)
    (384, 6, 18, 2, 1), (250, 6, 18, 2, 2), (128, 4, 18, 2, 1), (77, 2, 18, 2, 3),
    # ks | 32: 6-slot ring (128-row tiles)
    (128, 4, 34, 1, 1), (77, 4, 34, 1, 3), (128, 4, 33, 1, 2), (300, 4, 33, 1, 1), (128, 2, 34, 2, 1), (200, 2, 33, 2, 2)])
def test_qmm2(qt, M, wm, ks, wn, splits, monkeypatch):
    """qmm2.hip for every epilogue and tile / split-K choice, incl. ragged M / N tails (416 columns = 3.25
    workgroup tiles; with wn = 2 a wave's second group may lie past N), split counts that do not divide the
    super-blocks, the 8-wave k-step split (ks = 2) and the 2-group wave tiles (wn = 2), against the fp32
    product of the dequantised weight."""
    from localai_tfp_amd.ops import linear as L
    if ks == 18 and qt != QType.Q4_K:
        pytest.skip("the 4-wave wide form is compiled for Q4_K / MX4F only")
    if qt == QType.Q8_0 and ks != 18 and (32 * wm * wn == 256 or (ks == 17 and 32 * wm * wn >= 192)):
        pytest.skip("a 256-row (wide: 192-row) Q8_0 stage ring exceeds the LDS (not compiled)")
    if ks == 17 and wm == 7 and qt not in (QType.Q4_K, QType.Q2_K):
        pytest.skip("the 224-row wide ring fits the LDS for Q4_K / Q2_K only (not compiled)")
    monkeypatch.setattr(L, "QMM2", True)
    monkeypatch.setattr(L, "QMM2_FORCE", (wm, ks, wn, splits))
    n, k = 416, 2304
    raw, dense = make_w(qt, n, k, seed=M + 7 * wm)
    W = QWeight.from_ggml(raw, qt, n, k, DEV, t32=True)
    assert W.to_t32() and W.layout == "t32"
    x = torch.randn(M, k, device=DEV).half()
    ref = x.float().cpu() @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, out)
    assert rel(out, ref) < 5e-3
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, z, out_zeroed=True)
    assert rel(z, ref) < 5e-3
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, x, EPI_ADD_F32, acc)
    assert rel(acc - acc0, ref) < 5e-3
    ob = torch.empty(M, n, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_BF16, ob)
    assert rel(ob, ref) < 5e-3
    sw = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_SWIGLU, sw)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q3_K, QType.Q2_K, QType.Q5_K, QType.Q8_0])
@pytest.mark.parametrize("M,wm,splits", [
    (64, 1, 1), (40, 1, 3), (128, 2, 1), (77, 2, 2), (200, 2, 5), (256, 4, 1), (300, 4, 3), (511, 4, 2), (17, 1, 1),
    (384, 3, 1), (250, 3, 3)])
def test_qmm3(qt, M, wm, splits, monkeypatch):
    """qmm3.hip (warp-specialised producer / consumer waves) for every epilogue, row tile and split-K choice,
    incl. ragged M / N tails (416 columns: a consumer's second group past N) and split counts that do not
    divide the super-blocks, against the fp32 product of the dequantised weight."""
    from localai_tfp_amd.ops import linear as L
    monkeypatch.setattr(L, "QMM3", True)
    monkeypatch.setattr(L, "QMM3_MIN_M", 1)
    monkeypatch.setattr(L, "QMM3_FORCE", (wm, splits))
    n, k = 416, 2304
    raw, dense = make_w(qt, n, k, seed=M + 7 * wm)
    W = QWeight.from_ggml(raw, qt, n, k, DEV, t32=True)
    assert W.to_t32() and W.layout == "t32"
    x = torch.randn(M, k, device=DEV).half()
    ref = x.float().cpu() @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, out)
    assert rel(out, ref) < 5e-3
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, x, EPI_F32, z, out_zeroed=True)
    assert rel(z, ref) < 5e-3
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, x, EPI_ADD_F32, acc)
    assert rel(acc - acc0, ref) < 5e-3
    ob = torch.empty(M, n, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_BF16, ob)
    assert rel(ob, ref) < 5e-3
    sw = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
    qmatmul(W, x, EPI_SWIGLU, sw)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2


@pytest.mark.parametrize("name,qt,n,k,epi", [
    ("qkv", QType.Q4_K, 6144, 4096, EPI_F32), ("o_proj", QType.Q4_K, 4096, 4096, EPI_ADD_F32),
    ("gate_up", QType.Q4_K, 28672, 4096, EPI_SWIGLU), ("down", QType.Q4_K, 4096, 14336, EPI_ADD_F32),
    ("down_q6", QType.Q6_K, 4096, 14336, EPI_ADD_F32), ("v_q6", QType.Q6_K, 1024, 4096, EPI_F32)])
@pytest.mark.parametrize("M", [7, 128, 320])
def test_qmatmul_llama3_8b_shapes(name, qt, n, k, epi, M):
    """Production Llama-3-8B projection shapes through the DEFAULT dispatch (qmm tiles and split-K as
    chosen for these M) against an fp32 reference of the dequantised weight."""
    raw, dense = make_w(qt, n, k, seed=n + k + M)
    W = QWeight.from_ggml(raw, qt, n, k, DEV, t32=True)
    assert W.to_t32()
    torch.manual_seed(M)
    x = torch.randn(M, k, device=DEV).half()
    ref = x.float().cpu() @ dense.t()
    if epi == EPI_SWIGLU:
        out = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
        qmatmul(W, x, epi, out)
        g = ref.reshape(M, n // 32, 2, 16)
        ref = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
        assert rel(out, ref) < 1e-2
        return
    if epi == EPI_ADD_F32:
        out = torch.randn(M, n, device=DEV)
        base = out.clone()
        qmatmul(W, x, epi, out)
        assert rel(out - base, ref) < 5e-3
        return
    out = torch.zeros(M, n, device=DEV)
    qmatmul(W, x, epi, out, out_zeroed=True)
    assert rel(out, ref) < 5e-3


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0, QType.Q5_K, QType.Q3_K, QType.Q2_K])
@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_qmv_t32(qt, M):
    """qmv.hip decode GEMV on t32 weights (q8 activations) for every epilogue, and the t32 row
    dequantisation (embedding gather), against fp32 references."""
    n, k = 384, 2816
    raw, dense = make_w(qt, n, k, seed=11 * M)
    W = QWeight.from_ggml(raw, qt, n, k, DEV, t32=True)
    assert W.to_t32()
    x = torch.randn(M, k, device=DEV).half()
    xq = torch.empty(M, k, dtype=torch.int8, device=DEV)
    xds = torch.empty(M, k // 32, 2, dtype=torch.float32, device=DEV)
    K.quant_q8(x, xq, xds)
    xr = (xq.float().reshape(M, k // 32, 32) * xds[:, :, :1]).reshape(M, k).cpu()  # the operand qmv sees
    ref = xr @ dense.t()
    out = torch.empty(M, n, device=DEV)
    qmatmul(W, None, EPI_F32, out, xq=xq, xds=xds)
    assert rel(out, ref) < 2e-3
    acc = torch.randn(M, n, device=DEV)
    acc0 = acc.clone()
    qmatmul(W, None, EPI_ADD_F32, acc, xq=xq, xds=xds)  # split-K over workgroups (atomics)
    assert rel(acc - acc0, ref) < 2e-3
    z = torch.zeros(M, n, device=DEV)
    qmatmul(W, None, EPI_F32, z, xq=xq, xds=xds, out_zeroed=True)
    assert rel(z, ref) < 2e-3
    ob = torch.empty(M, n, dtype=torch.float16, device=DEV)
    qmatmul(W, None, EPI_BF16, ob, xq=xq, xds=xds)
    assert rel(ob, ref) < 3e-3
    sw = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
    qmatmul(W, None, EPI_SWIGLU, sw, xq=xq, xds=xds)
    g = ref.reshape(M, n // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2
    rows = torch.tensor([0, 5, n - 1, 37], dtype=torch.int32, device=DEV)
    deq = W.dequant_gpu(torch.float32, rows)
    assert rel(deq, dense[rows.long().cpu()]) < 1e-5


def test_f16_producers():
    M, H = 7, 4096
    x = torch.randn(M, H, device=DEV) * 3
    w = torch.rand(H, device=DEV) + 0.5
    ref = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * w).cpu()
    for dt in (torch.float16, torch.bfloat16, torch.float16):  # mode switches back and forth
        ob = torch.empty(M, H, dtype=dt, device=DEV)
        K.rmsnorm(x.clone(), w, 1e-5, out_bf16=ob)
        assert rel(ob, ref) < (2e-3 if dt == torch.float16 else 1e-2)
    # quant_q8 reads f16
    xh = ref.to(DEV).half()
    xq = torch.empty(M, H, dtype=torch.int8, device=DEV)
    xds = torch.empty(M, H // 32, 2, device=DEV)
    K.quant_q8(xh, xq, xds)
    deq = xq.float().view(M, H // 32, 32) * xds[..., :1]
    assert rel(deq.view(M, H), ref) < 1e-2
    # swiglu / glu / cast in f16
    g = torch.randn(M, 256, device=DEV).half()
    u = torch.randn(M, 256, device=DEV).half()
    o = torch.empty(M, 256, dtype=torch.float16, device=DEV)
    K.glu(g, u, o)
    assert rel(o, (torch.nn.functional.silu(g.float()) * u.float()).cpu()) < 5e-3
    c = torch.empty(M, H, dtype=torch.float16, device=DEV)
    K.cast_act(x, c)
    assert rel(c, x.cpu()) < 1e-3


def test_dense_cache_f16():
    qt = QType.Q4_K
    raw, dense = make_w(qt, 512, 1024, seed=5)
    W = QWeight.from_ggml(raw, qt, 512, 1024, DEV)
    W.build_bf16_cache(torch.float16)
    assert W.bf16_cache.dtype == torch.float16
    assert rel(W.bf16_cache, dense) < 1e-3
    x = torch.randn(600, 1024, device=DEV).half()
    out = torch.zeros(600, 512, device=DEV)
    qmatmul(W, x, EPI_ADD_F32, out)  # M=600 -> hipBLASLt f16 path
    assert rel(out, x.float().cpu() @ dense.t()) < 5e-3


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_attn_outputs_act16(dt):
    Hq, Hkv, D, bs, nb = 32, 8, 128, 16, 64
    kc, vc = _paged_kv(nb, Hkv, bs, D, 3)
    lens = [40, 300]
    B = len(lens)
    maxb = max((l + bs - 1) // bs for l in lens)
    bt = (torch.randperm(nb - 1)[: B * maxb] + 1).int().view(B, maxb)
    seq = torch.tensor(lens, dtype=torch.int32)
    q = torch.randn(B, Hq, D).bfloat16()
    ref = torch.empty(B, Hq, D)
    K.attn_decode(q, kc, vc, bt, seq, 0.088, ref)
    out = torch.empty(B, Hq, D, dtype=dt, device=DEV)
    K.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), seq.to(DEV), 0.088, out, part_size=128)
    assert rel(out, ref) < 1e-2


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("D,Hq,Hkv", [(64, 8, 8), (128, 8, 2), (40, 8, 8), (80, 4, 4), (512, 1, 1), (320, 2, 2)])
@pytest.mark.parametrize("causal", [False, True])
def test_attn_dense(dt, D, Hq, Hkv, causal):
    """(D = 512: the SD VAE mid-block's single head; 320 pads to it.)"""
    B, Sq, Sk = 2, 77, 150 if not causal else 77
    g = torch.Generator().manual_seed(D + Hq)
    q = torch.randn(B * Sq, Hq * D, generator=g).to(dt)
    k = torch.randn(B * Sk, Hkv * D, generator=g).to(dt)
    v = torch.randn(B * Sk, Hkv * D, generator=g).to(dt)
    klen = torch.tensor([Sk, Sk - 13], dtype=torch.int32)
    ref = torch.empty(B * Sq, Hq * D)
    K.attn_dense(q, k, v, ref, B, Sq, Sk, Hq, Hkv, D, 0.125, causal, klen=klen)
    out = torch.empty(B * Sq, Hq * D, dtype=dt, device=DEV)
    K.attn_dense(q.to(DEV), k.to(DEV), v.to(DEV), out, B, Sq, Sk, Hq, Hkv, D, 0.125, causal, klen=klen.to(DEV))
    assert rel(out, ref) < 1.5e-2


@pytest.mark.parametrize("D", [64, 32])
def test_attn_dense_relative_bias(D):
    """T5's relative-position bias as an additive [H, Sq + Sk - 1] table by key-minus-query offset, with key
    padding, against an explicit [B, H, Sq, Sk] bias + mask in fp32."""
    from localai_tfp_amd.models.diffusion.text_encoders import t5_buckets
    B, S, H = 2, 77, 8
    g = torch.Generator().manual_seed(5)
    q, k, v = (torch.randn(B * S, H * D, generator=g).half() for _ in range(3))
    table = torch.randn(32, H, generator=g) * 2
    offs = torch.arange(-(S - 1), S)
    rb = table[t5_buckets(offs, 32, 128)].t().contiguous()
    klen = torch.tensor([S, 50], dtype=torch.int32)
    pos = torch.arange(S)
    bias = table[t5_buckets(pos[None, :] - pos[:, None], 32, 128)].permute(2, 0, 1)  # [H, S, S]
    qf, kf, vf = (t.float().view(B, S, H, D).transpose(1, 2) for t in (q, k, v))
    sc = qf @ kf.transpose(-1, -2) + bias[None]
    sc = sc.masked_fill(pos[None, None, None, :] >= klen.view(B, 1, 1, 1), float("-inf"))
    ref = (sc.softmax(-1) @ vf).transpose(1, 2).reshape(B * S, H * D)
    cpu = torch.empty(B * S, H * D)
    K.attn_dense(q, k, v, cpu, B, S, S, H, H, D, 1.0, klen=klen, rbias=rb)
    assert rel(cpu, ref) < 1e-2
    out = torch.empty(B * S, H * D, dtype=torch.float16, device=DEV)
    K.attn_dense(q.to(DEV), k.to(DEV), v.to(DEV), out, B, S, S, H, H, D, 1.0, klen=klen.to(DEV), rbias=rb.to(DEV))
    assert rel(out, ref) < 1.5e-2


@pytest.mark.parametrize("causal", [False, True])
def test_attn_dense_kv_capacity(causal):
    """Fixed-capacity KV cache read in place (kv_rows): Whisper decoder self-attention layout."""
    B, Sq, Sk, cap, H, D = 3, 5 if causal else 1, 37, 64, 8, 64
    dt = torch.float16
    g = torch.Generator().manual_seed(11)
    q = torch.randn(B * Sq, H * D, generator=g).to(dt)
    k = torch.randn(B * cap, H * D, generator=g).to(dt)
    v = torch.randn(B * cap, H * D, generator=g).to(dt)
    klen = torch.tensor([Sk, Sk - 3, 9], dtype=torch.int32)
    ref = torch.empty(B * Sq, H * D)
    kw = dict(klen=None if causal else klen, kv_rows=cap)
    K.attn_dense(q, k, v, ref, B, Sq, Sk, H, H, D, 0.125, causal, **kw)
    kref = k.view(B, cap, -1)[:, :Sk].reshape(B * Sk, -1)
    vref = v.view(B, cap, -1)[:, :Sk].reshape(B * Sk, -1)
    ref2 = torch.empty(B * Sq, H * D)
    K.attn_dense(q, kref, vref, ref2, B, Sq, Sk, H, H, D, 0.125, causal, klen=None if causal else klen)
    assert torch.allclose(ref, ref2)
    out = torch.empty(B * Sq, H * D, dtype=dt, device=DEV)
    kw = dict(klen=None if causal else klen.to(DEV), kv_rows=cap)
    K.attn_dense(q.to(DEV), k.to(DEV), v.to(DEV), out, B, Sq, Sk, H, H, D, 0.125, causal, **kw)
    assert rel(out, ref) < 1.5e-2


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_qmv_fused_input(qt, M):
    """qmv with the q8 quantisation (src 16-bit) or RMSNorm + quantisation (src fp32 residual) fused into
    the prologue == rmsnorm / quant_q8 kernels followed by the plain qmv, for every epilogue incl. the
    K-split accumulate (ks > 1) and the interleaved SwiGLU; and both against the fp32 reference."""
    from localai_tfp_amd.ops.linear import qmv_fusable, qmv_fused
    n, k = 512, 2048
    raw, dense = make_w(qt, n, k, seed=3 * M + int(qt))
    W = QWeight.from_ggml(raw, qt, n, k, DEV)
    assert W.to_t32()
    g = torch.Generator().manual_seed(M)
    h = torch.randn(M, k, generator=g).to(DEV) * 3
    nw = (torch.rand(k, generator=g) + 0.5).to(DEV)
    eps = 1e-5
    x16 = (torch.randn(M, k, generator=g) * 2).half().to(DEV)
    N.ensure_act(torch.float16)
    xq = torch.empty(M, k, dtype=torch.int8, device=DEV)
    xds = torch.empty(M, k // 32, 2, device=DEV)
    y_ref_norm = (h / torch.sqrt(h.pow(2).mean(-1, keepdim=True) + eps) * nw).cpu() @ dense.t()
    y_ref_act = x16.float().cpu() @ dense.t()
    for src in ("norm", "act"):
        if src == "norm":
            K.rmsnorm(h, nw, eps, out_q8=(xq, xds))
        else:
            K.quant_q8(x16, xq, xds)
        xin, kw = (h, dict(norm=nw, eps=eps)) if src == "norm" else (x16, {})
        ref = y_ref_norm if src == "norm" else y_ref_act
        # fp32 store (zeroed -> split-K over workgroups)
        assert qmv_fusable(W, M, EPI_F32, True)
        a = torch.zeros(M, n, device=DEV)
        b = torch.zeros(M, n, device=DEV)
        qmatmul(W, None, EPI_F32, a, xq=xq, xds=xds, out_zeroed=True)
        assert qmv_fused(W, xin, EPI_F32, b, out_zeroed=True, **kw)
        assert rel(b, a) < 1e-5 and rel(b, ref) < 2e-2, (src, rel(b, a), rel(b, ref))
        # accumulate
        acc0 = torch.randn(M, n, device=DEV)
        a, b = acc0.clone(), acc0.clone()
        qmatmul(W, None, EPI_ADD_F32, a, xq=xq, xds=xds)
        assert qmv_fused(W, xin, EPI_ADD_F32, b, **kw)
        assert rel(b - acc0, a - acc0) < 1e-5
        # SwiGLU over interleaved gate|up rows
        sa = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
        sb = torch.empty_like(sa)
        qmatmul(W, None, EPI_SWIGLU, sa, xq=xq, xds=xds)
        assert qmv_fused(W, xin, EPI_SWIGLU, sb, **kw)
        assert rel(sb, sa) < 2e-3


@pytest.mark.parametrize("V", [1001, 4096, 128256, 128259])
def test_argmax_rows(V):
    """argmax_kernel: 16-B loads on aligned rows, scalar tail / unaligned rows, first index on ties."""
    g = torch.Generator().manual_seed(V)
    x = torch.randn(5, V, generator=g)
    x[1] = 0.5  # all ties -> index 0
    x[2, V - 1] = 100.0  # maximum in the tail
    x[3, 7] = x[3, V // 2] = 50.0  # tie -> the lower index
    xd = x.to(DEV)
    out = torch.empty(5, dtype=torch.int32, device=DEV)
    N.kcall("mxk_argmax", xd.data_ptr(), xd.stride(0), 5, V, out.data_ptr(), N.stream_ptr())
    assert out.cpu().tolist() == [int(x[0].argmax()), 0, V - 1, 7, int(x[4].argmax())]


def _kept_set_ref(row: torch.Tensor, temp: float, top_k: int, top_p: float, min_p: float):
    """Kept token set + normaliser of the sampler chain (temperature, top-k with ties, top-p over the top-k
    mass measured within the min-p set, min-p), on the CPU."""
    v = row.double() / temp
    mx = float(v.max())
    order = torch.argsort(v, descending=True, stable=True)
    sv = v[order]
    keep = len(sv)
    if 0 < top_k < keep:
        kv = sv[top_k - 1]
        keep = top_k
        while keep < len(sv) and sv[keep] == kv:
            keep += 1
    zk = float(torch.exp(sv[:keep] - mx).sum())
    if min_p > 0:
        mv = mx + np.log(min_p)
        while keep > 1 and sv[keep - 1] < mv:
            keep -= 1
    if 0 < top_p < 1:
        cum, k = 0.0, 0
        while k < keep:
            cum += float(torch.exp(sv[k] - mx))
            k += 1
            if cum >= top_p * zk:
                break
        while k < keep and sv[k] == sv[k - 1]:
            k += 1
        keep = max(1, k)
    kept = order[:keep]
    return set(kept.tolist()), float(torch.exp(sv[:keep] - mx).sum()), mx


@pytest.mark.parametrize("top_k,top_p,min_p", [(40, 0.95, 0.05), (40, 1.0, 0.0), (0, 0.9, 0.0), (0, 1.0, 0.1),
                                                (1000, 0.95, 0.05)])
def test_sampling_fast_path_kept_set(top_k, top_p, min_p):
    """The histogram / candidate-set sampler (llama.cpp defaults top_k 40, top_p 0.95, min_p 0.05 at 128k
    vocabulary) draws inside the exact kept set and reports the log-probability under it."""
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    torch.manual_seed(3)
    V, B = 128256, 8
    logits = torch.randn(B, V, device=DEV) * 2.5
    logits[0, :50] += 6.0  # a peaked row
    sb = SamplerBatch(DEV)
    ps = [SamplingParams(temperature=0.9, top_k=top_k, top_p=top_p, min_p=min_p, seed=r) for r in range(B)]
    refs = [_kept_set_ref(logits[r].cpu(), 0.9, top_k, top_p, min_p) for r in range(B)]
    for step in range(3):
        tok, lp = sb.sample(logits.clone(), ps, [[]] * B, [step] * B)
        tok, lp = tok.cpu().tolist(), lp.cpu().tolist()
        for r in range(B):
            kept, z, mx = refs[r]
            assert tok[r] in kept, (r, tok[r], len(kept))
            want = float(logits[r, tok[r]].double().cpu() / 0.9 - mx - np.log(z))
            assert abs(lp[r] - want) < 1e-3, (lp[r], want)


def test_sampling_fast_path_distribution():
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    V = 1000
    logits = torch.full((1, V), -30.0, device=DEV)
    logits[0, :4] = torch.log(torch.tensor([0.1, 0.2, 0.3, 0.4], device=DEV))
    sb = SamplerBatch(DEV)
    cnt = np.zeros(4)
    for s in range(2000):
        tok, _ = sb.sample(logits.clone(), [SamplingParams(temperature=1.0, top_k=3, top_p=1.0, min_p=0.0, seed=s)],
                           [[]], [0])
        cnt[int(tok[0])] += 1
    freq = cnt / cnt.sum()
    assert np.allclose(freq, [0.0, 0.2 / 0.9, 0.3 / 0.9, 0.4 / 0.9], atol=0.04), freq


@pytest.mark.parametrize("B", [1, 3, 16, 128])
def test_sampling_topk_split_matches_row_kernel(B):
    """Small batches with top-k on go through the split-vocabulary sampler (B x S slice workgroups + a merge);
    with the same seeds it draws exactly the token the one-workgroup-per-row kernel draws, with the same
    log-probability, including penalties, logit bias, an allow mask and greedy rows."""
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    torch.manual_seed(5)
    V = 128256
    logits = torch.randn(B, V, device=DEV) * 2.0
    logits[0, 100:140] += 5.0
    mask = torch.full((B, (V + 31) // 32), -1, dtype=torch.int32, device=DEV)
    if B > 1:
        mask[1] = 0
        mask[1, 10:20] = -1  # row 1: only 320 tokens allowed, spread over one slice
    ps = []
    for r in range(B):
        if r == 2:
            ps.append(SamplingParams(temperature=0.0, seed=r))
        else:
            ps.append(SamplingParams(temperature=0.8, top_k=[40, 64, 1, 7][r % 4], top_p=[0.95, 1.0, 0.9][r % 3],
                                     min_p=[0.05, 0.0][r % 2], repeat_penalty=1.1, frequency_penalty=0.2,
                                     logit_bias={5: 2.0, 120: -3.0}, seed=100 + r))
    hist = [[120, 121, 5, 121] for _ in range(B)]
    split, full = SamplerBatch(DEV), SamplerBatch(DEV)
    full.SPLIT_MAX_B = 0
    assert split._split_slices(ps, B, V) > 0 and full._split_slices(ps, B, V) == 0
    for step in range(4):
        t1, l1 = split.sample(logits.clone(), ps, hist, [step] * B, allow_mask=mask)
        t2, l2 = full.sample(logits.clone(), ps, hist, [step] * B, allow_mask=mask)
        assert t1.cpu().tolist() == t2.cpu().tolist(), step
        assert torch.allclose(l1.cpu(), l2.cpu(), atol=2e-3), (l1, l2)


@pytest.mark.parametrize("split", [True, False])
def test_sampling_pending_token_penalties(split):
    """Overlap pipeline: a row's previous token still in flight (device tensor + index `pend`) is counted by
    the penalty kernels exactly as if it were the newest history entry (window one shorter on the host)."""
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    torch.manual_seed(3)
    B, V = 6, 32000
    logits = torch.randn(B, V, device=DEV) * 3
    ps = [SamplingParams(temperature=[0.0, 0.7][r % 2], top_k=40, top_p=0.95, repeat_penalty=1.4,
                         frequency_penalty=0.5, presence_penalty=0.2, repeat_last_n=[8, 1, 64][r % 3], seed=r)
          for r in range(B)]
    hist = [[int(x) for x in torch.randint(0, V, (20,))] for _ in range(B)]
    prev = torch.randint(0, V, (B + 2,), dtype=torch.int32, device=DEV)
    prev[3] = hist[1][-1]  # row 1's pending token already in its window: its count goes up
    pend = [2, 3, -1, 5, 0, 7]
    for r in range(B):  # make the pending tokens matter: push them to the top of their rows
        if pend[r] >= 0:
            logits[r, int(prev[pend[r]])] = 20.0
    full_hist = [h + [int(prev[i])] if i >= 0 else h for h, i in zip(hist, pend)]
    a, b = SamplerBatch(DEV), SamplerBatch(DEV)
    if not split:
        a.SPLIT_MAX_B = b.SPLIT_MAX_B = 0
    for step in range(3):
        t1, l1 = a.sample(logits.clone(), ps, hist, [step] * B, pend_tok=prev, pend=pend)
        t2, l2 = b.sample(logits.clone(), ps, full_hist, [step] * B)
        assert t1.cpu().tolist() == t2.cpu().tolist(), step
        assert torch.allclose(l1.cpu(), l2.cpu(), atol=1e-4)


def test_sampling_topk_split_ties_and_flat_rows():
    """Rows with massive exact ties (a flat row, a tied top block larger than a slice's candidate capacity)
    and near-ties (values within 1e-6) through the split sampler: the slices flag the tie overflow and the
    merge falls back to the full-row chain, so the draw still matches the one-workgroup-per-row kernel."""
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    torch.manual_seed(9)
    B, V = 4, 128256
    logits = torch.randn(B, V, device=DEV)
    logits[0] = 1.5                               # flat row: every value tied
    logits[1, 1000:3000] = 9.0                    # 2000 exact ties above the rest, inside one slice
    logits[2] = 3.0 + 1e-6 * torch.randn(V, device=DEV)  # near-flat
    logits[3, 5000:5300] = 7.0 + 1e-5 * torch.arange(300, device=DEV)
    ps = [SamplingParams(temperature=0.9, top_k=40, top_p=0.95, min_p=0.0, seed=7 + r) for r in range(B)]
    hist = [[] for _ in range(B)]
    split, full = SamplerBatch(DEV), SamplerBatch(DEV)
    full.SPLIT_MAX_B = 0
    assert split._split_slices(ps, B, V) > 0
    kth = torch.topk(logits[2], 40).values[-1]
    for step in range(3):
        t1, l1 = split.sample(logits.clone(), ps, hist, [step] * B)
        t2, l2 = full.sample(logits.clone(), ps, hist, [step] * B)
        t1, t2 = t1.cpu().tolist(), t2.cpu().tolist()
        # rows 0, 1, 3: identical draws (row 2's row-kernel path is the value-bisection chain, whose
        # threshold resolution lumps these near-ties differently); row 2: a member of the exact top-40
        assert [t1[i] for i in (0, 1, 3)] == [t2[i] for i in (0, 1, 3)], step
        assert float(logits[2, t1[2]]) >= float(kth), step
        assert 3000 > t1[1] >= 1000 and 5300 > t1[3] >= 5260


@pytest.mark.parametrize("tp", [2, 8])
def test_argmax_keys_merge(tp):
    """Vocab-parallel greedy head: per-shard 64-bit (value, global index) keys, merged across shards, pick the
    argmax of the whole row (lowest index on ties, padding columns of the last shard excluded)."""
    V, S = 128256, 7
    g = torch.Generator().manual_seed(tp)
    full = torch.randn(S, V, generator=g)
    full[1, 5] = full[1, V - 3] = 40.0  # tie across shards
    full[2] = -2.0  # all equal
    full[3] = -torch.inf
    full[3, 77777] = -1e30
    vl = -(-V // tp)
    keys = torch.empty(tp * S, dtype=torch.int64, device=DEV)
    for r in range(tp):
        lo, hi = r * vl, min(V, (r + 1) * vl)
        loc = torch.full((S, vl), 1e9)
        loc[:, :hi - lo] = full[:, lo:hi]
        loc = loc.to(DEV)
        N.kcall("mxk_argmax_keys", loc.data_ptr(), loc.stride(0), S, hi - lo, lo, keys[r * S:].data_ptr(),
                N.stream_ptr())
    out = torch.empty(S, dtype=torch.int32, device=DEV)
    N.kcall("mxk_argmax_merge", keys.data_ptr(), tp, S, out.data_ptr(), N.stream_ptr())
    want = full.argmax(1).tolist()
    assert out.cpu().tolist() == want and want[1] == 5 and want[2] == 0 and want[3] == 77777


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q3_K])
def test_qmv1_batch1(qt):
    """The batch-1 qmv1 kernel (activation slice read before the weights, no unit loop): unsplit RMSNorm input at
    K = 4096 / 8192 (two / four units per wave; fp32 store and the interleaved SwiGLU) and split 16-bit input at
    K = 14336 (accumulate), against
    the fp32 reference and against the generic kernel (mxk_qmv1_enable(0))."""
    from localai_tfp_amd.ops.linear import qmv_fused
    g = torch.Generator().manual_seed(int(qt))
    eps = 1e-5
    for k, src in ((4096, "norm"), (8192, "norm"), (14336, "act")):
        n = 512
        raw, dense = make_w(qt, n, k, seed=k + int(qt))
        W = QWeight.from_ggml(raw, qt, n, k, DEV)
        assert W.to_t32()
        if src == "norm":
            h = torch.randn(1, k, generator=g).to(DEV) * 3
            nw = (torch.rand(k, generator=g) + 0.5).to(DEV)
            xin, kw = h, dict(norm=nw, eps=eps)
            ref = (h / torch.sqrt(h.pow(2).mean(-1, keepdim=True) + eps) * nw).cpu() @ dense.t()
            epis = (EPI_F32, EPI_SWIGLU)
        else:
            N.ensure_act(torch.float16)
            xin, kw = (torch.randn(1, k, generator=g) * 2).half().to(DEV), {}
            ref = xin.float().cpu() @ dense.t()
            epis = (EPI_ADD_F32,)
        for epi in epis:
            outs = []
            for on in (1, 0):
                N.kcall("mxk_qmv1_enable", on)
                if epi == EPI_SWIGLU:
                    o = torch.empty(1, n // 2, dtype=torch.float16, device=DEV)
                else:
                    o = torch.zeros(1, n, device=DEV)
                assert qmv_fused(W, xin, epi, o, out_zeroed=True, **kw)
                outs.append(o.float().cpu())
            N.kcall("mxk_qmv1_enable", 1)
            if epi == EPI_SWIGLU:
                gu = ref.reshape(1, n // 32, 2, 16)
                r = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(1, n // 2)
            else:
                r = ref
            assert rel(outs[0], outs[1]) < 5e-3 and rel(outs[0], r) < 2e-2, (src, epi)


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K])
@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("k", [4096, 8192])
@pytest.mark.parametrize("split", [False, True])
def test_qmv_rope_fused(qt, bias, k, split, monkeypatch):
    """Batch-1 qkv GEMV with RoPE + paged KV append in the epilogue == the unfused qmv + rope_kv kernels: q rows,
    the K and V cache rows at the slot, and nothing else in the caches touched. split: K split over several
    workgroups per column group, the last one running the epilogue; its workspace and tickets end re-zeroed."""
    from localai_tfp_amd.ops.linear import qmv_fused, qmv_rope_fused
    Hq, Hkv, D, bs, nb = 8, 2, 128, 16, 8
    n = (Hq + 2 * Hkv) * D
    raw, _ = make_w(qt, n, k, seed=11)
    W = QWeight.from_ggml(raw, qt, n, k, DEV)
    assert W.to_t32()
    g = torch.Generator().manual_seed(5)
    h = torch.randn(1, k, generator=g).to(DEV) * 2
    nw = (torch.rand(k, generator=g) + 0.5).to(DEV)
    bq = (torch.randn(n, generator=g) * 0.1).to(DEV) if bias else None
    pos = torch.tensor([37], dtype=torch.int32, device=DEV)
    slots = torch.tensor([3 * bs + 5], dtype=torch.int32, device=DEV)
    inv_freq = (1.0 / (500000.0 ** (torch.arange(0, D, 2).float() / D))).to(DEV)
    # reference: GEMV to fp32 qkv, then rope_kv
    qkv = torch.zeros(1, n, device=DEV)
    assert qmv_fused(W, h, EPI_F32, qkv, norm=nw, eps=1e-5, out_zeroed=True)
    q_ref = torch.zeros(1, Hq, D, dtype=torch.bfloat16, device=DEV)
    kc_ref = torch.zeros(nb, Hkv, bs, D, dtype=torch.bfloat16, device=DEV)
    vc_ref = torch.zeros_like(kc_ref)
    K.rope_kv(qkv, bq, pos, slots, inv_freq, 1.0, Hq, Hkv, D, D, False, q_ref, kc_ref, vc_ref, bs)
    # fused, as two parts (q|k and v) like a checkpoint whose attn_v has its own block format
    q = torch.zeros_like(q_ref)
    kc = torch.zeros_like(kc_ref)
    vc = torch.zeros_like(vc_ref)
    cut = (Hq + Hkv) * D
    sk = (torch.zeros(n, device=DEV), torch.zeros(n // 32, dtype=torch.int32, device=DEV)) if split else None
    for off, rows in ((0, slice(0, cut)), (cut, slice(cut, n))):
        Wp = QWeight.from_ggml(raw.reshape(n, -1)[rows], qt, rows.stop - rows.start, k, DEV)
        assert Wp.to_t32()
        if split:
            from localai_tfp_amd.ops import linear as L
            monkeypatch.setattr(L, "QMV_ROPE_SPLIT", True)
            assert L.qmv_rope_split(Wp) > 1
        b = bq[rows] if bq is not None else None
        assert qmv_rope_fused(Wp, h, nw, 1e-5, off, pos, slots, inv_freq, b, 1.0, Hq, Hkv, D, q, kc, vc, bs, sk=sk)
    if split:
        assert float(sk[0].abs().sum()) == 0.0 and int(sk[1].abs().sum()) == 0
    assert rel(q.float(), q_ref.float()) < 2e-2
    assert rel(kc.float(), kc_ref.float()) < 2e-2 and rel(vc.float(), vc_ref.float()) < 2e-2
    touched = torch.zeros(nb, bs, dtype=torch.bool)
    touched[3, 5] = True
    assert float(kc.float().abs().sum(dim=(1, 3)).cpu()[~touched].sum()) == 0.0
