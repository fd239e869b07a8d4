"""RWKV-6 ("Finch") language models on the continuous-batching engine.

Reference parity: llama.cpp's `rwkv6` architecture (llm_build_rwkv6: time mix with data-dependent
token-shift lerps and decay, GGML_OP_RWKV_WKV6, per-head GroupNorm, channel mix; SURVEY.md §2.6
K17), which the reference serves through its llama-cpp backend — fixture
tests/models_fixtures/rwkv.yaml and gallery `rwkv-6-world-7b` (rwkv-6-world-7b-Q4_K_M.gguf).

Per layer over a ragged engine step (decode rows + prefill chunks):

    xn  = layernorm(h)                                   (norm.hip)
    xxx = xn + sx*maa_x, sx = shift(xn) - xn            (rwkv.hip shift_mix; shift state carried)
    m   = tanh(xxx W1^T) -> 5 x (m_i W2_i^T)             (hipBLASLt; 5 x 32-wide LoRA)
    xw,xk,xv,xr,xg = xn + sx*(maa_i + m_i)              (rwkv.hip shift_mix, 5 act16 operands)
    r,k,v = GEMMs; g = silu(GEMM); w = decay + tanh(xw D1^T) D2^T
    y   = GroupNorm_head(wkv6(r, k, v, w, u)) * g       (rwkv.hip wkv6, norm + gate fused)
    h  += y Wo^T
    xn  = layernorm(h); xk,xr = shift_mix(2)            (second shift state)
    h  += sigmoid(xr Wr^T) * ((relu(xk Wk^T))^2 Wv^T)

Recurrent state per sequence (one engine block each, like models/mamba.py): two token-shift rows
and the [H, 64, 64] WKV matrix per layer.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from ..formats.gguf import QType
from ..ops import core as K
from ..ops.linear import ACT_DTYPE, EPI_ADD_F32, EPI_F32, QWeight, qmatmul
from .mamba import _seg_state, _Segments

LN_X_EPS = 64e-5  # llama.cpp rwkv6 GroupNorm eps


@dataclass
class RwkvConfig:
    name: str = "rwkv6"
    arch: str = "rwkv6"
    hidden: int = 4096
    n_layers: int = 32
    vocab: int = 65536
    ffn: int = 14336
    head_size: int = 64
    mix_dim: int = 32  # time_mix_extra_dim
    decay_dim: int = 64  # time_decay_extra_dim
    norm_eps: float = 1e-5
    rescale_every: int = 0
    ctx_train: int = 1 << 20
    tie_embeddings: bool = False
    extra: dict = field(default_factory=dict)
    head_dim: int = 1
    n_heads: int = 1
    n_kv_heads: int = 1
    embed_scale: float = 1.0

    @property
    def n_head(self) -> int:
        return self.hidden // self.head_size

    @classmethod
    def from_gguf_metadata(cls, md: dict) -> "RwkvConfig":
        a = str(md.get("general.architecture", "rwkv6"))
        g = lambda k, dflt=None: md.get(f"{a}.{k}", dflt)  # noqa: E731
        return cls(name=str(md.get("general.name", a)), arch=a, hidden=int(g("embedding_length")),
                   n_layers=int(g("block_count")), ffn=int(g("feed_forward_length")),
                   vocab=int(g("vocab_size", 0) or len(md.get("tokenizer.ggml.tokens", []) or [0])),
                   head_size=int(g("wkv.head_size", 64)), mix_dim=int(g("time_mix_extra_dim", 32)),
                   decay_dim=int(g("time_decay_extra_dim", 64)),
                   norm_eps=float(g("attention.layer_norm_epsilon", 1e-5)),
                   rescale_every=int(g("rescale_every_n_layers", 0) or 0))


RWKV6_WORLD_7B = RwkvConfig(name="rwkv-6-world-7b")
RWKV6_WORLD_1B6 = RwkvConfig(name="rwkv-6-world-1b6", hidden=2048, n_layers=24, ffn=7168)


def tiny_rwkv_config(**kw) -> RwkvConfig:
    c = RwkvConfig(name="tiny-rwkv6", hidden=256, n_layers=2, vocab=512, ffn=512)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@dataclass
class RwkvLayer:
    ln1_w: torch.Tensor
    ln1_b: torch.Tensor
    ln2_w: torch.Tensor
    ln2_b: torch.Tensor
    maa_x: torch.Tensor  # [C]
    maa5: torch.Tensor  # [5, C]  (w, k, v, r, g)
    w1: QWeight  # [5*32, C]
    w2: torch.Tensor  # [5, C, 32] 16-bit
    decay: torch.Tensor  # [C]
    decay_w1: QWeight  # [64, C]
    decay_w2: QWeight  # [C, 64]
    u: torch.Tensor  # [C] time_first
    wr: QWeight
    wk: QWeight
    wv: QWeight
    wg: QWeight
    wo: QWeight
    lnx_w: torch.Tensor
    lnx_b: torch.Tensor
    cmaa: torch.Tensor  # [2, C] (k, r)
    cwk: QWeight  # [F, C]
    cwv: QWeight  # [C, F]
    cwr: QWeight  # [C, C]


class RwkvState:
    """Per layer: time-mix shift rows [slots, C], channel-mix shift rows [slots, C], WKV [slots, H, 64, 64]."""

    def __init__(self, cfg: RwkvConfig, num_slots: int, device):
        self.num_blocks = num_slots
        L, C, H, N = cfg.n_layers, cfg.hidden, cfg.n_head, cfg.head_size
        self.att_shift = torch.zeros((L, num_slots, C), dtype=torch.float32, device=device)
        self.ffn_shift = torch.zeros((L, num_slots, C), dtype=torch.float32, device=device)
        self.wkv = torch.zeros((L, num_slots, H, N, N), dtype=torch.float32, device=device)

    def layer(self, i: int):
        return self.att_shift[i], self.ffn_shift[i], self.wkv[i]


class RwkvWorkspace:
    def __init__(self, cfg: RwkvConfig, T: int, max_seqs: int, device):
        dev = torch.device(device)
        C, Fd = cfg.hidden, cfg.ffn
        self.max_tokens, self.max_seqs = T, max_seqs
        self.h = torch.empty((T, C), dtype=torch.float32, device=dev)
        self.xn = torch.empty((T, C), dtype=torch.float32, device=dev)
        self.sx = torch.empty((T, C), dtype=torch.float32, device=dev)
        self.x16 = torch.empty((5, T, C), dtype=ACT_DTYPE, device=dev)
        self.t1 = torch.empty((T, 5 * cfg.mix_dim), dtype=torch.float32, device=dev)
        self.rkvwg = torch.empty((5, T, C), dtype=torch.float32, device=dev)
        self.d1 = torch.empty((T, cfg.decay_dim), dtype=torch.float32, device=dev)
        self.y16 = torch.empty((T, C), dtype=ACT_DTYPE, device=dev)
        self.f = torch.empty((T, Fd), dtype=torch.float32, device=dev)
        self.f16 = torch.empty((T, Fd), dtype=ACT_DTYPE, device=dev)
        self.hs = torch.empty((max_seqs, C), dtype=torch.float32, device=dev)
        self.hs16 = torch.empty((max_seqs, C), dtype=ACT_DTYPE, device=dev)
        self.logits = torch.empty((max_seqs, cfg.vocab), dtype=torch.float32, device=dev)


class RwkvModel:
    recurrent = True

    def __init__(self, cfg: RwkvConfig, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.layers: list[RwkvLayer] = []
        self.tp_size, self.n_kv, self.n_heads = 1, 1, 1
        self.slot_div = 1
        self.last_hidden = None

    def make_state_cache(self, num_slots: int, block_size: int) -> RwkvState:
        self.slot_div = block_size
        return RwkvState(self.cfg, num_slots, self.device)

    def make_workspace(self, max_tokens: int, max_seqs: int) -> RwkvWorkspace:
        return RwkvWorkspace(self.cfg, max_tokens, max_seqs, self.device)

    def weight_bytes(self) -> int:
        n = 0
        for L in self.layers:
            n += sum(w.nbytes() for w in (L.w1, L.decay_w1, L.decay_w2, L.wr, L.wk, L.wv, L.wg, L.wo, L.cwk, L.cwv,
                                          L.cwr))
        return n + self.lm_head.nbytes() + self.tok_embd.nbytes()

    # ------------------------------------------------------------------ loading
    @classmethod
    def load(cls, cfg: RwkvConfig, get_tensor, device="cpu") -> "RwkvModel":
        """`get_tensor(gguf_name) -> (raw, qtype, ggml_shape) | None`, llama.cpp rwkv6 tensor names."""
        m = cls(cfg, device)
        dev = m.device
        C = cfg.hidden
        from ..ops.quant import dequantize

        def f32(name):
            t = get_tensor(name)
            if t is None:
                return None
            raw, qt, shp = t
            a = np.asarray(dequantize(raw, qt, tuple(int(s) for s in shp)), np.float32).reshape(-1)
            return torch.from_numpy(a.copy()).to(dev)

        def qw(name):
            raw, qt, shp = get_tensor(name)
            K_ = int(shp[0])
            N_ = int(np.prod([int(s) for s in shp[1:]]))
            return QWeight.from_ggml(np.asarray(raw).view(np.uint8).reshape(N_, -1), qt, N_, K_, dev, name,
                                     dense_dtype=ACT_DTYPE)

        for i in range(cfg.n_layers):
            p = f"blk.{i}."
            fused = f32(p + "time_mix_lerp_fused.weight")
            if fused is not None:  # newer converters: [w, k, v, r, g] stacked
                maa5 = fused.view(5, C)
            else:
                maa5 = torch.stack([f32(p + f"time_mix_lerp_{n}.weight") for n in "wkvrg"])
            m.layers.append(RwkvLayer(
                ln1_w=f32(p + "attn_norm.weight"), ln1_b=f32(p + "attn_norm.bias"),
                ln2_w=f32(p + "attn_norm_2.weight"), ln2_b=f32(p + "attn_norm_2.bias"),
                maa_x=f32(p + "time_mix_lerp_x.weight"), maa5=maa5.contiguous(),
                w1=qw(p + "time_mix_w1.weight"),
                w2=f32(p + "time_mix_w2.weight").view(5, C, cfg.mix_dim).to(ACT_DTYPE).contiguous(),
                decay=f32(p + "time_mix_decay.weight"),
                decay_w1=qw(p + "time_mix_decay_w1.weight"), decay_w2=qw(p + "time_mix_decay_w2.weight"),
                u=f32(p + "time_mix_first.weight"),
                wr=qw(p + "time_mix_receptance.weight"), wk=qw(p + "time_mix_key.weight"),
                wv=qw(p + "time_mix_value.weight"), wg=qw(p + "time_mix_gate.weight"),
                wo=qw(p + "time_mix_output.weight"),
                lnx_w=f32(p + "time_mix_ln.weight"), lnx_b=f32(p + "time_mix_ln.bias"),
                cmaa=torch.stack([f32(p + "channel_mix_lerp_k.weight"), f32(p + "channel_mix_lerp_r.weight")]),
                cwk=qw(p + "channel_mix_key.weight"), cwv=qw(p + "channel_mix_value.weight"),
                cwr=qw(p + "channel_mix_receptance.weight"),
            ))
        m.tok_embd = qw("token_embd.weight")
        m.ln0_w, m.ln0_b = f32("token_embd_norm.weight"), f32("token_embd_norm.bias")
        m.lnf_w, m.lnf_b = f32("output_norm.weight"), f32("output_norm.bias")
        m.lm_head = qw("output.weight")
        return m

    # ------------------------------------------------------------------ forward
    def forward(self, fb, state: RwkvState, ws: RwkvWorkspace) -> torch.Tensor:
        cfg = self.cfg
        T, C = fb.T, cfg.hidden
        eps = cfg.norm_eps
        h = ws.h[:T]
        xn = ws.xn[:T]
        E = self.tok_embd
        if E.device.type == "cpu":
            xn.copy_(E.dense_f32()[fb.tokens.long()])
        elif E.is_quant:
            from .. import _native as N
            N.kcall("mxk_dequant_rows", int(E.qtype), E.data.data_ptr(), N.ptr(E.dplane), fb.tokens.data_ptr(), T, E.K,
                    None, xn.data_ptr(), xn.stride(0), N.stream_ptr())
        else:
            K.gather_rows(E.data, fb.tokens, xn, 1.0)
        if fb.embed_rows:
            for r0, e in fb.embed_rows:
                xn[r0:r0 + e.shape[0]].copy_(e)
        K.layernorm(xn, self.ln0_w, self.ln0_b, eps, h)  # ln0 on the embeddings
        seg = _Segments(fb, T, self.slot_div)
        sx = ws.sx[:T]
        # the shift-mix kernel writes mix m at m*T*C (a contiguous [n_mix, T, C] block): take a contiguous view of
        # the workspace, not the strided ws.x16[:, :T] (whose mixes sit max_tokens*C apart)
        x16 = ws.x16.view(-1)[:5 * T * C].view(5, T, C)
        rkvwg = ws.rkvwg[:, :T]
        for li, L in enumerate(self.layers):
            att_shift, ffn_shift, wkv = state.layer(li)
            # ---- time mix ----
            K.layernorm(h, L.ln1_w, L.ln1_b, eps, xn)
            shift_mix(xn, att_shift, L.maa_x[None], None, x16[:1], seg, sx_out=sx)
            t1 = ws.t1[:T]
            qmatmul(L.w1, x16[0], EPI_F32, t1)
            t16 = torch.tanh(t1).to(ACT_DTYPE).view(T, 5, cfg.mix_dim).transpose(0, 1)  # [5, T, 32]
            dm = torch.bmm(t16, L.w2.transpose(1, 2)).float()  # [5, T, C]
            shift_mix(xn, att_shift, L.maa5, dm, x16, seg, sx_in=sx)
            r, k, v, w, g = rkvwg[3], rkvwg[1], rkvwg[2], rkvwg[0], rkvwg[4]
            qmatmul(L.wr, x16[3], EPI_F32, r)
            qmatmul(L.wk, x16[1], EPI_F32, k)
            qmatmul(L.wv, x16[2], EPI_F32, v)
            qmatmul(L.wg, x16[4], EPI_F32, g)
            F.silu(g, inplace=True)
            d1 = ws.d1[:T]
            qmatmul(L.decay_w1, x16[0], EPI_F32, d1)
            d16 = torch.tanh(d1).to(ACT_DTYPE)
            w.copy_(L.decay.expand(T, C))
            qmatmul(L.decay_w2, d16, EPI_ADD_F32, w)
            y16 = ws.y16[:T]
            wkv6(r, k, v, w, g, L.u, wkv, L.lnx_w, L.lnx_b, seg, cfg.head_size, y16)
            qmatmul(L.wo, y16, EPI_ADD_F32, h)
            # ---- channel mix ----
            K.layernorm(h, L.ln2_w, L.ln2_b, eps, xn)
            shift_mix(xn, ffn_shift, L.cmaa, None, x16[:2], seg)
            f = ws.f[:T]
            qmatmul(L.cwk, x16[0], EPI_F32, f)
            f16 = ws.f16[:T]
            torch.square(torch.relu_(f), out=f)
            f16.copy_(f)
            rr = rkvwg[0]
            qmatmul(L.cwr, x16[1], EPI_F32, rr)
            vv = rkvwg[1]
            qmatmul(L.cwv, f16, EPI_F32, vv)
            h.addcmul_(torch.sigmoid_(rr), vv)
            if cfg.rescale_every and (li + 1) % cfg.rescale_every == 0:
                h.mul_(0.5)
        S = fb.logits_idx.numel()
        hs = ws.hs[:S]
        K.select_rows(h, fb.logits_idx, hs)
        if fb.want_hidden or fb.keep_hidden:
            hn = F.layer_norm(hs, (C,), self.lnf_w, self.lnf_b, eps)
            if fb.want_hidden:
                return hn
            self.last_hidden = hn
        hs16 = ws.hs16[:S]
        K.layernorm(hs, self.lnf_w, self.lnf_b, eps, hs16)
        logits = ws.logits[:S]
        qmatmul(self.lm_head, hs16, EPI_F32, logits)
        return logits


# ------------------------------------------------------------------------------------------------ ops
def shift_mix(x, shift_state, maa, dm, out16, seg: _Segments, sx_in=None, sx_out=None):
    """out16[m] = x + sx * (maa[m] + dm[m]); sx = x_prev - x (computed + saved unless sx_in given)."""
    T, C = x.shape
    n_mix = maa.shape[0]
    if x.is_cuda:
        from .. import _native as N
        # the kernel addresses out16 / dm as contiguous [n_mix, T, C] blocks (mix m at m*T*C)
        if not out16.is_contiguous() or (dm is not None and not dm.is_contiguous()):
            raise ValueError("shift_mix: out16 / dm must be contiguous [n_mix, T, C]")
        N.ensure_act(out16.dtype)
        N.kcall("mxk_rwkv_shift_mix", x.data_ptr(), x.stride(0), shift_state.data_ptr(), N.ptr(sx_in), N.ptr(sx_out),
                maa.data_ptr(), N.ptr(dm), out16.data_ptr(), n_mix, seg.slots.data_ptr(), seg.positions.data_ptr(),
                seg.slot_div, seg.n_dec, N.ptr(seg.pf_cu), seg.n_pf, T, C, N.stream_ptr())
        return out16
    if sx_in is None:
        sx = torch.empty_like(x)
        for row0, n in seg.host_segments():
            si, reset = _seg_state(seg, row0)
            prev = torch.zeros(C) if (reset or si is None) else shift_state[si].clone()
            xp = torch.cat([prev[None], x[row0:row0 + n - 1]], 0)
            sx[row0:row0 + n] = xp - x[row0:row0 + n]
            if si is not None:
                shift_state[si] = x[row0 + n - 1]
        if sx_out is not None:
            sx_out.copy_(sx)
    else:
        sx = sx_in
    mu = maa[:, None, :] + (dm if dm is not None else 0)
    out16.copy_((x[None] + sx[None] * mu).to(out16.dtype))
    return out16


def wkv6(r, k, v, w, g, u, state, lnw, lnb, seg: _Segments, head_size: int, out16):
    """RWKV-6 recurrence + per-head GroupNorm (ln_x) + gate; state [slots, H, 64, 64] (k-major)."""
    T, C = r.shape
    H = C // head_size
    if r.is_cuda:
        from .. import _native as N
        N.ensure_act(out16.dtype)
        assert r.stride(0) == k.stride(0) == v.stride(0) == w.stride(0) == g.stride(0)
        N.kcall("mxk_rwkv_wkv6", r.data_ptr(), k.data_ptr(), v.data_ptr(), w.data_ptr(), g.data_ptr(), r.stride(0),
                u.data_ptr(), state.data_ptr(), lnw.data_ptr(), lnb.data_ptr(), float(LN_X_EPS), out16.data_ptr(),
                out16.stride(0), seg.slots.data_ptr(), seg.positions.data_ptr(), seg.slot_div, seg.n_dec,
                N.ptr(seg.pf_cu), seg.n_pf, H, head_size, N.stream_ptr())
        return out16
    N_ = head_size
    uu = u.view(H, N_)
    for row0, n in seg.host_segments():
        si, reset = _seg_state(seg, row0)
        S = torch.zeros(H, N_, N_) if (reset or si is None) else state[si].clone()
        for t in range(row0, row0 + n):
            rt, kt, vt = r[t].view(H, N_), k[t].view(H, N_), v[t].view(H, N_)
            wt = torch.exp(-torch.exp(w[t].view(H, N_)))
            kv = kt[:, :, None] * vt[:, None, :]  # [H, i, j]
            y = torch.einsum("hi,hij->hj", rt, uu[:, :, None] * kv + S)
            S = wt[:, :, None] * S + kv
            y = F.group_norm(y.reshape(1, C), H, lnw, lnb, LN_X_EPS).view(C)
            out16[t] = (y * g[t]).to(out16.dtype)
        if si is not None:
            state[si] = S
    return out16


# ------------------------------------------------------------------------------------------------ weights
def synthetic_rwkv_source(cfg: RwkvConfig, seed: int = 0, qtype: str = "Q4_K"):
    """Random-init RWKV-6 weights under llama.cpp's GGUF names (RWKV init statistics: decay speeds
    spread over channels, lerps in [0, 1], time_first ~ 0.5). Large matrices in a real quantised
    block format when K allows it, so the GPU runs the same GEMM kernels as a Q4_K_M file."""
    from ..ops.quant import random_quantized
    rng = np.random.default_rng(seed)
    C, Fd, V, D1, D2 = cfg.hidden, cfg.ffn, cfg.vocab, cfg.mix_dim, cfg.decay_dim
    qt = {"Q4_K": QType.Q4_K, "Q8_0": QType.Q8_0, "F32": QType.F32}[qtype]

    def mat(N_, K_, std=0.02):
        if K_ % 256 == 0 and qt != QType.F32:
            return random_quantized(rng, qt, N_, K_, std), qt, (K_, N_)
        return (rng.standard_normal((N_, K_)) * std).astype(np.float32), QType.F32, (K_, N_)

    def vec(a, shape=None):
        a = np.ascontiguousarray(np.asarray(a, np.float32))
        return a, QType.F32, shape or tuple(reversed(a.shape))
    ones, zeros = (lambda: vec(np.ones(C))), (lambda: vec(np.zeros(C)))
    plan = {"token_embd.weight": lambda: mat(V, C, 0.5), "token_embd_norm.weight": ones,
            "token_embd_norm.bias": zeros, "output_norm.weight": ones, "output_norm.bias": zeros,
            "output.weight": lambda: mat(V, C, 0.05)}
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        ratio = 1 - i / cfg.n_layers
        plan.update({
            p + "attn_norm.weight": ones, p + "attn_norm.bias": zeros,
            p + "attn_norm_2.weight": ones, p + "attn_norm_2.bias": zeros,
            p + "time_mix_lerp_x.weight": (lambda: vec(rng.uniform(0, 1, C), (C, 1, 1))),
            p + "time_mix_w1.weight": (lambda: mat(5 * D1, C, 0.01)),
            p + "time_mix_w2.weight": (lambda: vec(rng.uniform(-0.01, 0.01, (5, C, D1)), (D1, C, 5))),
            p + "time_mix_decay.weight": (lambda r=ratio: vec(-6 + 5 * (np.arange(C) / (C - 1)) ** (0.7 + 1.3 * r),
                                                              (C, 1, 1))),
            p + "time_mix_decay_w1.weight": (lambda: mat(D2, C, 0.01)),
            p + "time_mix_decay_w2.weight": (lambda: mat(C, D2, 0.01)),
            p + "time_mix_first.weight": (lambda: vec(rng.uniform(0.2, 0.8, (C // cfg.head_size, cfg.head_size)))),
            p + "time_mix_receptance.weight": (lambda: mat(C, C)), p + "time_mix_key.weight": (lambda: mat(C, C)),
            p + "time_mix_value.weight": (lambda: mat(C, C)), p + "time_mix_gate.weight": (lambda: mat(C, C)),
            p + "time_mix_output.weight": (lambda: mat(C, C, 0.02 / math.sqrt(2 * cfg.n_layers))),
            p + "time_mix_ln.weight": ones, p + "time_mix_ln.bias": zeros,
            p + "channel_mix_lerp_k.weight": (lambda: vec(rng.uniform(0, 1, C), (C, 1, 1))),
            p + "channel_mix_lerp_r.weight": (lambda: vec(rng.uniform(0, 1, C), (C, 1, 1))),
            p + "channel_mix_key.weight": (lambda: mat(Fd, C)),
            p + "channel_mix_value.weight": (lambda: mat(C, Fd, 0.02 / math.sqrt(2 * cfg.n_layers))),
            p + "channel_mix_receptance.weight": (lambda: mat(C, C)),
        })
        for n in "wkvrg":
            plan[p + f"time_mix_lerp_{n}.weight"] = (lambda: vec(rng.uniform(0, 1, C), (C, 1, 1)))
    cache = {}

    def get_tensor(name):
        if name not in plan:
            return None
        if name not in cache:
            cache[name] = plan[name]()
        return cache[name]
    return get_tensor
