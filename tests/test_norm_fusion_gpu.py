"""The RMSNorm split across two K-quant GEMMs (qmm2_impl.h Q2Fuse, ops/linear.py NormFuse) against the fp32 oracle:
the producer (residual-add GEMM) must leave h = h0 + x W^T, xn = f16(h * gamma), the rows' sums of squares of h, a
re-zeroed ss_zero and zeroed tickets; the consumer must equal rmsnorm(h) * gamma through its own epilogue. Plus the
whole model: a fused-norm forward matches the separate-launch forward."""
import pytest
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops.linear import EPI_ADD_F32, EPI_F32, EPI_SWIGLU, NormFuse, QWeight, qmatmul

from test_kernels_gpu import make_w, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q5_K, QType.Q8_0])
@pytest.mark.parametrize("M,wm,ks,wn,splits", [
    (128, 2, 2, 1, 1), (128, 2, 2, 1, 4), (77, 4, 2, 1, 3), (200, 2, 1, 2, 2), (416, 7, 1, 1, 1), (300, 4, 17, 1, 3),
    (128, 4, 34, 1, 2), (64, 2, 10, 1, 5)])
def test_norm_fusion_producer_consumer(qt, M, wm, ks, wn, splits, monkeypatch):
    from localai_tfp_amd.ops import linear as L
    if qt == QType.Q8_0 and (32 * wm * wn == 256 or (ks == 17 and 32 * wm * wn >= 192)):
        pytest.skip("a 256-row (wide: 192-row) Q8_0 stage ring exceeds the LDS (not compiled)")
    if wm == 7 and qt not in (QType.Q4_K,):
        pytest.skip("the 224-row rings fit the LDS for Q4_K only here")
    monkeypatch.setattr(L, "QMM2", True)
    H, K1, F = 512, 768, 416
    torch.manual_seed(M + splits)
    # producer: h += x Wp^T (Wp: [H, K1])
    monkeypatch.setattr(L, "QMM2_FORCE", (wm, ks, wn, splits))
    rawp, densep = make_w(qt, H, K1, seed=3 + M)
    Wp = QWeight.from_ggml(rawp, qt, H, K1, DEV, t32=True)
    assert Wp.to_t32()
    x = torch.randn(M, K1, device=DEV).half()
    h0 = torch.randn(M, H, device=DEV)
    h = h0.clone()
    gamma = (torch.rand(H, device=DEV) + 0.5)
    ss = torch.zeros(2, M + 5, 32, device=DEV)
    ss[1].fill_(7.0)  # the buffer the producer must re-zero
    tick = torch.zeros(-(-M // 32) * (H // 32), dtype=torch.int32, device=DEV)
    xn = torch.full((M, H + 64), 3.0, dtype=torch.float16, device=DEV)[:, :H]
    qmatmul(Wp, x, EPI_ADD_F32, h, fuse=NormFuse(1, ss_out=ss[0], ss_zero=ss[1], gamma=gamma, xn=xn, tick=tick))
    torch.cuda.synchronize()
    href = h0.cpu() + x.float().cpu() @ densep.t()
    assert rel(h, href) < 5e-3
    assert rel(xn.float(), (h * gamma).cpu()) < 2e-3
    assert rel(ss[0, :M, 0], (h.cpu() ** 2).sum(1)) < 1e-4
    assert float(ss[0, :M, 1:].abs().max()) == 0.0 and float(ss[0, M:].abs().max()) == 0.0
    assert float(ss[1, :M, 0].abs().max()) == 0.0  # re-zeroed (the first float of each row line is the sum)
    assert int(tick.abs().max()) == 0
    eps = 1e-5
    xnorm = (h.cpu() * torch.rsqrt((h.cpu() ** 2).mean(1, keepdim=True) + eps) * gamma.cpu()).half().float()
    # consumer: SwiGLU over gate|up (Wc: [F, H]) and the split-K fp32 qkv form
    rawc, densec = make_w(qt, F, H, seed=11 + M)
    Wc = QWeight.from_ggml(rawc, qt, F, H, DEV, t32=True)
    assert Wc.to_t32()
    ref = xnorm @ densec.t()
    monkeypatch.setattr(L, "QMM2_FORCE", (wm, ks, wn, 1))
    sw = torch.empty(M, F // 2, dtype=torch.float16, device=DEV)
    qmatmul(Wc, xn, EPI_SWIGLU, sw, fuse=NormFuse(2, ss_in=ss[0], eps=eps))
    g = ref.reshape(M, F // 32, 2, 16)
    ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
    assert rel(sw, ref_sw) < 1e-2
    monkeypatch.setattr(L, "QMM2_FORCE", (wm, ks, wn, splits))
    z = torch.zeros(M, F, device=DEV)
    qmatmul(Wc, xn, EPI_F32, z, out_zeroed=True, fuse=NormFuse(2, ss_in=ss[0], eps=eps))
    assert rel(z, ref) < 5e-3


@pytest.mark.parametrize("P", [40, 200])
@pytest.mark.parametrize("norm,rope", [(True, False), (False, True), (True, True)])
def test_norm_fusion_model_forward(P, norm, rope, monkeypatch):
    """A Llama-shaped model's M > 4 forward with the norms split across the GEMMs and / or RoPE + KV append in the
    q|k|v GEMM epilogue equals the forward with separate norm / rope_kv launches: logits and the paged KV cache,
    over repeated forwards on one workspace (buffer ping-pong, re-zeroing, self-resetting tickets), and the fused
    path is the one taken."""
    import numpy as np
    from localai_tfp_amd.engine.kv_cache import KVCache
    from localai_tfp_amd.models.config import tiny_config
    from localai_tfp_amd.models.llama import ForwardBatch, LlamaModel, Workspace
    from localai_tfp_amd.models.synthetic import synthetic_source
    from localai_tfp_amd.ops import linear as L
    cfg = tiny_config(hidden=512, ffn=1024, n_heads=8, n_kv_heads=2, head_dim=64, rope_dim=64, vocab=1024, n_layers=4)
    m = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=5), "cuda")
    prompt = list(np.random.default_rng(0).integers(0, cfg.vocab, P))
    bs = 16

    # qmm2 plans for every GEMM (an earlier test's load-time tuning may have put some of these shapes on qmm3)
    monkeypatch.setattr(L, "QMM2", True)

    def run(nf, rf):
        monkeypatch.setattr(L, "NORM_FUSE", nf)
        monkeypatch.setattr(L, "ROPE_FUSE", rf)
        m.__dict__.pop("_nf_cache", None)
        kv = KVCache(cfg.n_layers, 64, m.n_kv, bs, cfg.head_dim, "cuda")
        ws = Workspace(cfg, 256, 8, "cuda", m.tp_size)
        blocks = list(range(1, 2 + (P + bs) // bs))
        bt = torch.tensor([blocks], dtype=torch.int32, device=DEV)
        slots = torch.tensor([blocks[p // bs] * bs + p % bs for p in range(P)], dtype=torch.int32, device=DEV)
        fb = ForwardBatch(torch.tensor(prompt, dtype=torch.int32, device=DEV),
                          torch.arange(P, dtype=torch.int32, device=DEV), slots,
                          torch.tensor([P - 1], dtype=torch.int32, device=DEV), n_decode=0, pf_block_tables=bt,
                          pf_cu_q=torch.tensor([0, P], dtype=torch.int32, device=DEV),
                          pf_ctx_lens=torch.tensor([P], dtype=torch.int32, device=DEV), pf_q_lens_host=[P],
                          pf_ctx_lens_host=[P])
        outs = [m.forward(fb, kv, ws).float().cpu().clone() for _ in range(2)]
        cache = torch.cat([kv.layer(li)[j][1:len(blocks) + 1].float().flatten().cpu()
                           for li in range(cfg.n_layers) for j in (0, 1)])
        taken = {k: v for k, v in m.__dict__.get("_nf_cache", {}).items() if v}
        assert float(ws.norm_ss.abs().max()) == 0.0 and int(ws.norm_tick.abs().max()) == 0
        assert float(ws.qkv.abs().max()) == 0.0  # the split-K q|k|v buffer is left zeroed either way
        return outs, cache, taken

    (f1, f2), fc, taken = run(norm, rope)
    if norm:
        assert any(isinstance(k[0], int) for k in taken), "the fused-norm path did not apply"
    if rope:
        assert any(k[0] == "rope" for k in taken), "the RoPE epilogue did not apply"
    (u1, _), uc, taken_u = run(False, False)
    assert not taken_u
    assert float((f1 - f2).norm() / f1.norm()) < 1e-2  # split-K fp32 atomics: order-dependent rounding
    r = float((f1 - u1).norm() / u1.norm())
    assert r < 1e-2, r
    rc = float((fc - uc).norm() / uc.norm())
    assert rc < 1e-2, rc
