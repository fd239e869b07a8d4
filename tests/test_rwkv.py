"""RWKV-6 models: engine outputs vs an independent token-by-token fp32 reference of llama.cpp's
rwkv6 graph (llm_build_rwkv6), chunked prefill / batching state carry-over, GGUF round trip, and the
HIP shift_mix / wkv6 kernels vs the fp32 path.

Parity note: no RWKV-6 implementation is importable here (transformers ships RWKV-4 only) and the
reference's llama.cpp is external, so numerics are pinned to the reference formula re-derived below,
not to llama.cpp outputs ("parity unpinned" against llama.cpp itself)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
from localai_tfp_amd.models import rwkv as RW
from localai_tfp_amd.ops.sampling import SamplingParams
from localai_tfp_amd.tokenizer import ByteTokenizer


def _model(device="cpu", seed=2, **kw):
    cfg = RW.tiny_rwkv_config(**kw)
    src = RW.synthetic_rwkv_source(cfg, seed=seed, qtype="F32")
    return RW.RwkvModel.load(cfg, src, device), src


def _ref_logits(cfg, get, ids):
    """Sequential fp32 RWKV-6 over one sequence -> logits [T, V] (weights read from the GGUF-named source)."""
    def t(name):
        raw, qt, shp = get(name)
        return torch.from_numpy(np.asarray(raw, np.float32).reshape(tuple(reversed(shp))).copy())
    C, H, N, eps = cfg.hidden, cfg.n_head, cfg.head_size, cfg.norm_eps
    ln = lambda x, p: F.layer_norm(x, (C,), t(p + ".weight").reshape(C), t(p + ".bias").reshape(C), eps)  # noqa: E731
    L = cfg.n_layers
    att_prev = [torch.zeros(C) for _ in range(L)]
    ffn_prev = [torch.zeros(C) for _ in range(L)]
    S = [torch.zeros(H, N, N) for _ in range(L)]
    out = []
    E = t("token_embd.weight")
    for tok in ids:
        x = ln(E[tok], "token_embd_norm")
        for i in range(L):
            p = f"blk.{i}."
            xn = ln(x, p + "attn_norm")
            sx = att_prev[i] - xn
            att_prev[i] = xn
            xxx = xn + sx * t(p + "time_mix_lerp_x.weight").reshape(C)
            m = torch.tanh(t(p + "time_mix_w1.weight") @ xxx).view(5, cfg.mix_dim)
            w2 = t(p + "time_mix_w2.weight")  # [5, C, 32]
            mm = torch.stack([w2[j] @ m[j] for j in range(5)])
            lerp = [t(p + f"time_mix_lerp_{n}.weight").reshape(C) for n in "wkvrg"]
            xw, xk, xv, xr, xg = [xn + sx * (lerp[j] + mm[j]) for j in range(5)]
            r = t(p + "time_mix_receptance.weight") @ xr
            k = t(p + "time_mix_key.weight") @ xk
            v = t(p + "time_mix_value.weight") @ xv
            g = F.silu(t(p + "time_mix_gate.weight") @ xg)
            w = t(p + "time_mix_decay.weight").reshape(C) + t(p + "time_mix_decay_w2.weight") @ torch.tanh(
                t(p + "time_mix_decay_w1.weight") @ xw)
            w = torch.exp(-torch.exp(w)).view(H, N)
            u = t(p + "time_mix_first.weight").reshape(H, N)
            rh, kh, vh = r.view(H, N), k.view(H, N), v.view(H, N)
            y = torch.zeros(H, N)
            for hh in range(H):
                kv = torch.outer(kh[hh], vh[hh])
                y[hh] = rh[hh] @ (u[hh][:, None] * kv + S[i][hh])
                S[i][hh] = w[hh][:, None] * S[i][hh] + kv
            y = F.group_norm(y.reshape(1, C), H, t(p + "time_mix_ln.weight").reshape(C),
                             t(p + "time_mix_ln.bias").reshape(C), RW.LN_X_EPS).view(C)
            x = x + t(p + "time_mix_output.weight") @ (y * g)
            xn = ln(x, p + "attn_norm_2")
            sx = ffn_prev[i] - xn
            ffn_prev[i] = xn
            xk = xn + sx * t(p + "channel_mix_lerp_k.weight").reshape(C)
            xr = xn + sx * t(p + "channel_mix_lerp_r.weight").reshape(C)
            kk = torch.relu(t(p + "channel_mix_key.weight") @ xk) ** 2
            x = x + torch.sigmoid(t(p + "channel_mix_receptance.weight") @ xr) * (t(p + "channel_mix_value.weight") @ kk)
        out.append(t("output.weight") @ ln(x, "output_norm"))
    return torch.stack(out)


def _engine(model, mbt=64, **kw):
    return LLMEngine(model, ByteTokenizer(model.cfg.vocab),
                     EngineConfig(max_num_seqs=4, max_batched_tokens=mbt, max_model_len=256, **kw))


def _tokens(h):
    toks = []
    for o in h:
        toks += o.token_ids
    return toks


def _check_greedy(cfg, get, prompt, out_ids, tol):
    lg = _ref_logits(cfg, get, prompt + out_ids)
    P = len(prompt)
    for k, tk in enumerate(out_ids):
        row = lg[P - 1 + k]
        assert row[tk] >= row.max() - tol, (k, tk, int(row.argmax()), float(row[tk]), float(row.max()))


def test_rwkv6_greedy_matches_reference():
    model, src = _model()
    prompt = [3, 77, 150, 9, 200, 41, 5]
    out = _engine(model).generate(prompt, SamplingParams(temperature=0.0), max_tokens=8)
    assert len(out.token_ids) == 8
    _check_greedy(model.cfg, src, prompt, out.token_ids, tol=2e-2)


def test_rwkv6_chunked_prefill_and_batching_match_single():
    model, _ = _model(seed=4)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (37, 6, 20)]
    solo = [_engine(model, mbt=256).generate(p, SamplingParams(temperature=0.0), max_tokens=5).token_ids
            for p in prompts]
    eng = _engine(model, mbt=16)
    from localai_tfp_amd.engine.sequence import Request
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 5)) for p in prompts]
    eng.run_until_done()
    assert [_tokens(h) for h in hs] == solo


def test_rwkv6_gguf_roundtrip(tmp_path):
    """A GGUF written with llama.cpp's rwkv6 names + metadata loads through the worker's loader."""
    from localai_tfp_amd.formats.gguf import GGUFWriter
    from localai_tfp_amd.models.loader import load_llm
    cfg = RW.tiny_rwkv_config()
    src = RW.synthetic_rwkv_source(cfg, seed=1, qtype="Q8_0")
    names = ["token_embd.weight", "token_embd_norm.weight", "token_embd_norm.bias", "output_norm.weight",
             "output_norm.bias", "output.weight"]
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        names += [p + n for n in (
            "attn_norm.weight", "attn_norm.bias", "attn_norm_2.weight", "attn_norm_2.bias", "time_mix_lerp_x.weight",
            "time_mix_w1.weight", "time_mix_w2.weight", "time_mix_decay.weight", "time_mix_decay_w1.weight",
            "time_mix_decay_w2.weight", "time_mix_first.weight", "time_mix_receptance.weight", "time_mix_key.weight",
            "time_mix_value.weight", "time_mix_gate.weight", "time_mix_output.weight", "time_mix_ln.weight",
            "time_mix_ln.bias", "channel_mix_lerp_k.weight", "channel_mix_lerp_r.weight", "channel_mix_key.weight",
            "channel_mix_value.weight", "channel_mix_receptance.weight")]
        names += [p + f"time_mix_lerp_{n}.weight" for n in "wkvrg"]
    path = str(tmp_path / "rwkv6.gguf")
    w = GGUFWriter(path)
    a = "rwkv6"
    for k, v in {"general.architecture": a, "general.name": "tiny-rwkv6", f"{a}.embedding_length": cfg.hidden,
                 f"{a}.block_count": cfg.n_layers, f"{a}.feed_forward_length": cfg.ffn,
                 f"{a}.vocab_size": cfg.vocab, f"{a}.wkv.head_size": 64, f"{a}.time_mix_extra_dim": 32,
                 f"{a}.time_decay_extra_dim": 64, f"{a}.attention.layer_norm_epsilon": 1e-5,
                 f"{a}.rescale_every_n_layers": 0}.items():
        w.add(k, v)
    for n in names:
        raw, qt, shp = src(n)
        w.add_tensor(n, np.asarray(raw).tobytes(), tuple(shp), int(qt))
    w.write()
    model, tok, lcfg, md = load_llm(path, "cpu")
    assert isinstance(model, RW.RwkvModel) and lcfg.n_layers == 2 and lcfg.hidden == 256
    out = _engine(model).generate([1, 2, 3], SamplingParams(temperature=0.0), max_tokens=4)
    assert len(out.token_ids) == 4


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_rwkv6_kernels_vs_reference():
    from localai_tfp_amd.models.mamba import _Segments
    from localai_tfp_amd.ops.linear import ACT_DTYPE
    from test_mamba import _FB, _seg_inputs
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    C, H, slot_div = 256, 4, 256
    T, n_dec, cu, slots, pos = _seg_inputs(dev, slot_div)
    x = torch.randn(T, C)
    maa = torch.rand(5, C)
    dm = torch.randn(5, T, C) * 0.1
    shift0 = torch.randn(4, C)
    r, k, v, g = (torch.randn(T, C) * 0.5 for _ in range(4))
    w = torch.randn(T, C) * 0.5 - 1.5
    u = torch.rand(C)
    lnw, lnb = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    S0 = torch.randn(4, H, 64, 64) * 0.1
    res = {}
    for d in (torch.device("cpu"), dev):
        seg = _Segments(_FB(T, n_dec, cu.to(d), slots.to(d), pos.to(d)), T, slot_div)
        st = shift0.clone().to(d)
        sx = torch.zeros(T, C, device=d)
        o1 = torch.zeros(1, T, C, dtype=ACT_DTYPE, device=d)
        RW.shift_mix(x.to(d), st, maa[:1].to(d), None, o1, seg, sx_out=sx)
        o5 = torch.zeros(5, T, C, dtype=ACT_DTYPE, device=d)
        RW.shift_mix(x.to(d), st, maa.to(d), dm.to(d), o5, seg, sx_in=sx)
        S = S0.clone().to(d)
        y = torch.zeros(T, C, dtype=ACT_DTYPE, device=d)
        RW.wkv6(r.to(d), k.to(d), v.to(d), w.to(d), g.to(d), u.to(d), S, lnw.to(d), lnb.to(d), seg, 64, y)
        torch.cuda.synchronize()
        res[d.type] = [t.float().cpu() for t in (st, sx, o1, o5, S, y)]
    for a, b in zip(res["cuda"][:2], res["cpu"][:2]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    for a, b in zip(res["cuda"][2:4], res["cpu"][2:4]):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(res["cuda"][4], res["cpu"][4], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(res["cuda"][5][:-1], res["cpu"][5][:-1], rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_rwkv6_engine_gpu_graphs():
    model, src = _model("cuda:0", seed=6)
    eng = _engine(model, use_graphs=True)
    eng.precapture_graphs()
    from localai_tfp_amd.engine.sequence import Request
    rng = np.random.default_rng(3)
    prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 8)) for p in prompts]
    eng.run_until_done()
    assert eng.stats["graph_steps"] > 0
    for p, h in zip(prompts, hs):
        toks = _tokens(h)
        assert len(toks) == 8
        _check_greedy(model.cfg, src, p, toks, tol=5e-2)


@pytest.mark.gpu
def test_synthetic_rwkv6_1b6_gpu():
    from localai_tfp_amd.models.loader import load_llm
    model, _, cfg, _ = load_llm("synthetic:rwkv6-1b6", "cuda:0")
    out = _engine(model, use_graphs=True).generate(list(range(1, 50)), SamplingParams(temperature=0.0), max_tokens=12)
    assert len(out.token_ids) == 12


@pytest.mark.gpu
def test_rwkv6_engine_workspace_nan_filled_gpu():
    """Every workspace buffer is written before it is read: NaN-filled workspace + state, eager engine, greedy
    tokens still match the fp32 reference (caught the strided shift-mix view that read stale rows when
    T < max_tokens)."""
    model, src = _model("cuda:0", seed=6)
    eng = _engine(model, use_graphs=False)
    for t in list(vars(eng.ws).values()) + list(vars(eng.kv).values()):
        if isinstance(t, torch.Tensor) and t.is_floating_point():
            t.fill_(float("nan"))
    rng = np.random.default_rng(3)
    prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
    from localai_tfp_amd.engine.sequence import Request
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 4)) for p in prompts]
    eng.run_until_done()
    for p, h in zip(prompts, hs):
        toks = _tokens(h)
        assert len(toks) == 4
        _check_greedy(model.cfg, src, p, toks, tol=5e-2)
