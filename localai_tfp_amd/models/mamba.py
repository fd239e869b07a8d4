"""Mamba (selective state-space) language models on the continuous-batching engine.

Reference parity: llama.cpp's `mamba` architecture (build_mamba + GGML_OP_SSM_CONV / SSM_SCAN,
SURVEY.md §2.6 K17; gallery/fixture models run through the llama-cpp backend) and the transformers
backend's `Type: Mamba` path (backend/python/transformers/backend.py:68-284, MambaForCausalLM).

Per layer, one engine step over a ragged batch (decode rows + prefill chunks, engine/engine.py):

    x    = rmsnorm(h) -> act16                       (norm.hip)
    xz   = x W_in^T -> fp32 [T, 2*Di]                (qgemm / hipBLASLt)
    xc   = silu(causal_conv1d(xz[:, :Di]) + b)       (ssm.hip ssm_conv; window carried in conv_state)
    dbc  = xc W_x^T -> fp32 [T, R + 2N]              (dt_low | B | C)
    y    = ssm_scan(...) * silu(z)                   (ssm.hip ssm_scan; dt_proj + softplus, D skip,
                                                      SiLU(z) gate fused; h carried in ssm_state)
    h   += y W_out^T                                 (EPI_ADD_F32 into the residual)

The recurrent state replaces the paged KV cache: the engine gives a recurrent model one cache
"block" per sequence (block_size = max_model_len, no prefix sharing), and the block id is the
state slot, so scheduling, preemption (recompute) and hipGraph decode buckets work unchanged.

Weights come from a GGUF (`general.architecture = mamba`), an HF checkpoint directory
(MambaForCausalLM safetensors) or `synthetic:mamba-*` random init.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from ..formats.gguf import QType
from ..ops import core as K
from ..ops.linear import ACT_DTYPE, EPI_ADD_F32, EPI_F32, QWeight, qmatmul


@dataclass
class MambaConfig:
    name: str = "mamba"
    arch: str = "mamba"
    hidden: int = 768
    n_layers: int = 24
    vocab: int = 50280
    d_inner: int = 1536
    d_state: int = 16
    d_conv: int = 4
    dt_rank: int = 48
    rms_eps: float = 1e-5
    ctx_train: int = 1 << 20  # no positional limit; the engine clamps to max_model_len
    tie_embeddings: bool = True
    conv_bias: bool = True
    extra: dict = field(default_factory=dict)
    # fields the engine / workers read off every model config
    head_dim: int = 1
    n_heads: int = 1
    n_kv_heads: int = 1
    embed_scale: float = 1.0

    @classmethod
    def from_hf(cls, d: dict, name: str = "mamba") -> "MambaConfig":
        H = int(d["hidden_size"])
        di = int(d.get("intermediate_size") or d.get("expand", 2) * H)
        r = d.get("time_step_rank", "auto")
        return cls(name=name, hidden=H, n_layers=int(d["num_hidden_layers"]), vocab=int(d["vocab_size"]), d_inner=di,
                   d_state=int(d.get("state_size", 16)), d_conv=int(d.get("conv_kernel", 4)),
                   dt_rank=math.ceil(H / 16) if r in ("auto", None) else int(r),
                   rms_eps=float(d.get("layer_norm_epsilon", 1e-5)),
                   tie_embeddings=bool(d.get("tie_word_embeddings", True)),
                   conv_bias=bool(d.get("use_conv_bias", True)))

    @classmethod
    def from_gguf_metadata(cls, md: dict) -> "MambaConfig":
        a = str(md.get("general.architecture", "mamba"))
        g = lambda k, dflt=None: md.get(f"{a}.{k}", dflt)  # noqa: E731
        H = int(g("embedding_length"))
        return cls(name=str(md.get("general.name", a)), arch=a, hidden=H, n_layers=int(g("block_count")),
                   vocab=int(g("vocab_size", 0) or len(md.get("tokenizer.ggml.tokens", []) or [0])),
                   d_inner=int(g("ssm.inner_size")), d_state=int(g("ssm.state_size")),
                   d_conv=int(g("ssm.conv_kernel")), dt_rank=int(g("ssm.time_step_rank")),
                   rms_eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)))


MAMBA_130M = MambaConfig(name="mamba-130m")
MAMBA_1_4B = MambaConfig(name="mamba-1.4b", hidden=2048, n_layers=48, d_inner=4096, dt_rank=128)
MAMBA_2_8B = MambaConfig(name="mamba-2.8b", hidden=2560, n_layers=64, d_inner=5120, dt_rank=160)


def tiny_mamba_config(**kw) -> MambaConfig:
    c = MambaConfig(name="tiny-mamba", hidden=256, n_layers=2, vocab=512, d_inner=512, dt_rank=16)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@dataclass
class MambaLayer:
    norm: torch.Tensor  # [H] fp32
    w_in: QWeight  # [2*Di, H]
    conv_w: torch.Tensor  # [Di, KC] fp32
    conv_b: torch.Tensor  # [Di] fp32
    w_x: QWeight  # [R + 2N, Di]
    w_dt: torch.Tensor  # [Di, R] fp32 (fused into the scan)
    dt_b: torch.Tensor  # [Di] fp32
    A: torch.Tensor  # [Di, N] fp32 = -exp(A_log)
    D: torch.Tensor  # [Di] fp32
    w_out: QWeight  # [H, Di]


class MambaState:
    """Recurrent cache: conv windows [L, slots, KC-1, Di] and SSM states [L, slots, Di, N] (fp32)."""

    def __init__(self, cfg: MambaConfig, num_slots: int, device):
        self.num_blocks = num_slots
        self.conv = torch.zeros((cfg.n_layers, num_slots, cfg.d_conv - 1, cfg.d_inner), dtype=torch.float32,
                                device=device)
        self.ssm = torch.zeros((cfg.n_layers, num_slots, cfg.d_inner, cfg.d_state), dtype=torch.float32,
                               device=device)

    def layer(self, i: int):
        return self.conv[i], self.ssm[i]

    def nbytes(self) -> int:
        return (self.conv.numel() + self.ssm.numel()) * 4


class MambaWorkspace:
    def __init__(self, cfg: MambaConfig, max_tokens: int, max_seqs: int, device):
        dev = torch.device(device)
        T, H, Di = max_tokens, cfg.hidden, cfg.d_inner
        self.max_tokens, self.max_seqs = T, max_seqs
        self.h = torch.empty((T, H), dtype=torch.float32, device=dev)
        self.x16 = torch.empty((T, max(H, Di)), dtype=ACT_DTYPE, device=dev)
        self.xz = torch.empty((T, 2 * Di), dtype=torch.float32, device=dev)
        self.xc = torch.empty((T, Di), dtype=torch.float32, device=dev)
        self.dbc = torch.empty((T, cfg.dt_rank + 2 * cfg.d_state), dtype=torch.float32, device=dev)
        self.y16 = torch.empty((T, Di), dtype=ACT_DTYPE, device=dev)
        self.hs = torch.empty((max_seqs, H), dtype=torch.float32, device=dev)
        self.logits = torch.empty((max_seqs, cfg.vocab), dtype=torch.float32, device=dev)


class MambaModel:
    recurrent = True

    def __init__(self, cfg: MambaConfig, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.layers: list[MambaLayer] = []
        self.tok_embd: QWeight | None = None
        self.lm_head: QWeight | None = None
        self.out_norm: torch.Tensor | None = None
        self.tp_size, self.n_kv, self.n_heads = 1, 1, 1
        self.last_hidden = None
        self.slot_div = 1

    # ------------------------------------------------------------------ engine hooks
    def make_state_cache(self, num_slots: int, block_size: int) -> MambaState:
        """One state slot per engine cache block; a token's flat KV slot // block_size is its state slot."""
        self.slot_div = block_size
        return MambaState(self.cfg, num_slots, self.device)

    def make_workspace(self, max_tokens: int, max_seqs: int) -> MambaWorkspace:
        return MambaWorkspace(self.cfg, max_tokens, max_seqs, self.device)

    def state_bytes_per_seq(self) -> int:
        c = self.cfg
        return c.n_layers * c.d_inner * (c.d_conv - 1 + c.d_state) * 4

    def weight_bytes(self) -> int:
        n = sum(w.nbytes() for L in self.layers for w in (L.w_in, L.w_x, L.w_out))
        n += self.lm_head.nbytes() + (0 if self.tok_embd is self.lm_head else self.tok_embd.nbytes())
        return n

    # ------------------------------------------------------------------ loading
    @classmethod
    def load(cls, cfg: MambaConfig, get_tensor, device="cpu") -> "MambaModel":
        """`get_tensor(gguf_name) -> (raw, qtype, ggml_shape) | None` (formats/gguf conventions;
        llama.cpp mamba tensor names)."""
        m = cls(cfg, device)
        dev = m.device

        def f32(name, shape=None):
            t = get_tensor(name)
            if t is None:
                return None
            raw, qt, shp = t
            from ..ops.quant import dequantize
            a = dequantize(raw, qt, tuple(int(s) for s in shp))
            a = np.asarray(a, np.float32).reshape(shape if shape is not None else tuple(reversed([int(s) for s in shp])))
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

        def qw(name):
            raw, qt, shp = get_tensor(name)
            K_, N_ = int(shp[0]), int(shp[1])
            return QWeight.from_ggml(np.asarray(raw).view(np.uint8).reshape(N_, -1), qt, N_, K_, dev, name,
                                     dense_dtype=ACT_DTYPE)

        Di, R, NS, KC = cfg.d_inner, cfg.dt_rank, cfg.d_state, cfg.d_conv
        for i in range(cfg.n_layers):
            p = f"blk.{i}."
            cb = f32(p + "ssm_conv1d.bias", (Di,))
            m.layers.append(MambaLayer(
                norm=f32(p + "attn_norm.weight", (cfg.hidden,)),
                w_in=qw(p + "ssm_in.weight"),
                conv_w=f32(p + "ssm_conv1d.weight", (Di, KC)),
                conv_b=cb if cb is not None else torch.zeros(Di, device=dev),
                w_x=qw(p + "ssm_x.weight"),
                w_dt=f32(p + "ssm_dt.weight", (Di, R)),
                dt_b=f32(p + "ssm_dt.bias", (Di,)),
                A=f32(p + "ssm_a", (Di, NS)),
                D=f32(p + "ssm_d", (Di,)),
                w_out=qw(p + "ssm_out.weight"),
            ))
        m.tok_embd = qw("token_embd.weight")
        m.out_norm = f32("output_norm.weight", (cfg.hidden,))
        m.lm_head = qw("output.weight") if get_tensor("output.weight") is not None else m.tok_embd
        cfg.tie_embeddings = m.lm_head is m.tok_embd
        return m

    # ------------------------------------------------------------------ forward
    def embed(self, tokens: torch.Tensor, out: torch.Tensor):
        E = self.tok_embd
        if E.device.type == "cpu":
            out.copy_(E.dense_f32()[tokens.long()])
        elif not E.is_quant:
            K.gather_rows(E.data, tokens, out, 1.0)
        else:
            from .. import _native as N
            N.kcall("mxk_dequant_rows", int(E.qtype), E.data.data_ptr(), N.ptr(E.dplane), tokens.data_ptr(),
                    tokens.numel(), E.K, None, out.data_ptr(), out.stride(0), N.stream_ptr())
        return out

    def forward(self, fb, state: MambaState, ws: MambaWorkspace) -> torch.Tensor:
        cfg = self.cfg
        T, H, Di = fb.T, cfg.hidden, cfg.d_inner
        eps = cfg.rms_eps
        h = ws.h[:T]
        self.embed(fb.tokens, h)
        if fb.embed_rows:
            for r0, e in fb.embed_rows:
                h[r0:r0 + e.shape[0]].copy_(e)
        x16, xz, xc, dbc, y16 = ws.x16[:T, :H], ws.xz[:T], ws.xc[:T], ws.dbc[:T], ws.y16[:T]
        seg = _Segments(fb, T, self.slot_div)
        for li, L in enumerate(self.layers):
            conv_st, ssm_st = state.layer(li)
            K.rmsnorm(h, L.norm, eps, out_bf16=x16)
            qmatmul(L.w_in, x16, EPI_F32, xz)
            xc16 = ws.x16[:T, :Di]
            ssm_conv(xz, L.conv_w, L.conv_b, conv_st, seg, xc, xc16)
            qmatmul(L.w_x, xc16, EPI_F32, dbc)
            ssm_scan(xc, dbc, L.w_dt, L.dt_b, L.A, L.D, xz, ssm_st, seg, y16)
            qmatmul(L.w_out, y16, EPI_ADD_F32, h)
        S = fb.logits_idx.numel()
        hs = ws.hs[:S]
        K.select_rows(h, fb.logits_idx, hs)
        if fb.want_hidden or fb.keep_hidden:
            hn = hs * torch.rsqrt(hs.pow(2).mean(-1, keepdim=True) + eps) * self.out_norm
            if fb.want_hidden:
                return hn
            self.last_hidden = hn
        xbs = ws.x16[:S, :H]
        K.rmsnorm(hs, self.out_norm, eps, out_bf16=xbs)
        logits = ws.logits[:S]
        qmatmul(self.lm_head, xbs, EPI_F32, logits)
        return logits


class _Segments:
    """Ragged-batch layout shared by the SSM kernels of one step (see ssm.hip)."""

    def __init__(self, fb, T: int, slot_div: int):
        self.n_dec = fb.n_decode
        self.pf_cu = fb.pf_cu_q
        self.n_pf = 0 if fb.pf_cu_q is None else int(fb.pf_cu_q.numel()) - 1
        self.slots, self.positions = fb.slots, fb.positions
        self.slot_div = slot_div
        self.T = T

    def host_segments(self):
        """[(row0, len)] on the host (CPU reference path)."""
        out = [(i, 1) for i in range(self.n_dec)]
        if self.n_pf:
            cu = self.pf_cu.tolist()
            out += [(self.n_dec + cu[k], cu[k + 1] - cu[k]) for k in range(self.n_pf)]
        return out


def _seg_state(seg: _Segments, row0: int):
    slot = int(seg.slots[row0])
    if slot < 0:
        return None, True
    return slot // seg.slot_div, int(seg.positions[row0]) == 0


def ssm_conv(xz: torch.Tensor, w: torch.Tensor, b: torch.Tensor, conv_state: torch.Tensor, seg: _Segments,
             xc: torch.Tensor, xc16: torch.Tensor):
    """xc = silu(causal depthwise conv(x = xz[:, :Di]) + b), window carried in conv_state [slots, KC-1, Di]."""
    Di, KC = w.shape
    if xz.is_cuda:
        from .. import _native as N
        N.ensure_act(xc16.dtype)
        N.kcall("mxk_ssm_conv", xz.data_ptr(), xz.stride(0), w.data_ptr(), b.data_ptr(), conv_state.data_ptr(), KC,
                seg.slots.data_ptr(), seg.positions.data_ptr(), seg.slot_div, seg.n_dec, N.ptr(seg.pf_cu), seg.n_pf,
                xc.data_ptr(), xc16.data_ptr(), xc16.stride(0), Di, N.stream_ptr())
        return xc
    for row0, n in seg.host_segments():
        si, reset = _seg_state(seg, row0)
        prev = torch.zeros(KC - 1, Di) if (reset or si is None) else conv_state[si].clone()
        x = torch.cat([prev, xz[row0:row0 + n, :Di]], 0)  # [KC-1+n, Di]
        y = sum(w[:, k] * x[k:k + n] for k in range(KC)) + b
        y = y * torch.sigmoid(y)
        xc[row0:row0 + n] = y
        xc16[row0:row0 + n] = y.to(xc16.dtype)
        if si is not None:
            conv_state[si] = x[-(KC - 1):]
    return xc


def ssm_scan(xc, dbc, w_dt, dt_b, A, D, xz, ssm_state, seg: _Segments, y16):
    """Selective scan with fused dt_proj/softplus, D skip and SiLU(z) gate; y16 [T, Di] act16."""
    Di, R = w_dt.shape
    NS = A.shape[1]
    if xc.is_cuda:
        from .. import _native as N
        N.ensure_act(y16.dtype)
        N.kcall("mxk_ssm_scan", xc.data_ptr(), dbc.data_ptr(), dbc.stride(0), w_dt.data_ptr(), dt_b.data_ptr(),
                A.data_ptr(), D.data_ptr(), xz.data_ptr(), xz.stride(0), ssm_state.data_ptr(), seg.slots.data_ptr(),
                seg.positions.data_ptr(), seg.slot_div, seg.n_dec, N.ptr(seg.pf_cu), seg.n_pf, y16.data_ptr(),
                y16.stride(0), Di, R, NS, N.stream_ptr())
        return y16
    for row0, n in seg.host_segments():
        si, reset = _seg_state(seg, row0)
        h = torch.zeros(Di, NS) if (reset or si is None) else ssm_state[si].clone()
        for t in range(row0, row0 + n):
            dt = torch.nn.functional.softplus(dbc[t, :R] @ w_dt.t() + dt_b)
            Bt, Ct = dbc[t, R:R + NS], dbc[t, R + NS:R + 2 * NS]
            x = xc[t]
            h = torch.exp(dt[:, None] * A) * h + (dt * x)[:, None] * Bt[None, :]
            z = xz[t, Di:]
            y16[t] = ((h @ Ct + D * x) * (z * torch.sigmoid(z))).to(y16.dtype)
        if si is not None:
            ssm_state[si] = h
    return y16


# ------------------------------------------------------------------------------------------------
# checkpoint sources


def hf_mamba_source(model_dir: str):
    """(MambaConfig, get_tensor) for a transformers MambaForCausalLM directory (safetensors), exposing
    the tensors under llama.cpp's GGUF names (F32 ggml layouts)."""
    from safetensors.numpy import load_file
    with open(os.path.join(model_dir, "config.json")) as f:
        cfg = MambaConfig.from_hf(json.load(f), os.path.basename(model_dir.rstrip("/")))
    tensors = {}
    for fn in sorted(os.listdir(model_dir)):
        if fn.endswith(".safetensors"):
            tensors.update(load_file(os.path.join(model_dir, fn)))
    tensors = {k.removeprefix("backbone."): v for k, v in tensors.items()}
    names = {"embeddings.weight": "token_embd.weight", "embedding.weight": "token_embd.weight",
             "norm_f.weight": "output_norm.weight", "lm_head.weight": "output.weight"}
    sub = {"norm.weight": "attn_norm.weight", "mixer.in_proj.weight": "ssm_in.weight",
           "mixer.conv1d.weight": "ssm_conv1d.weight", "mixer.conv1d.bias": "ssm_conv1d.bias",
           "mixer.x_proj.weight": "ssm_x.weight", "mixer.dt_proj.weight": "ssm_dt.weight",
           "mixer.dt_proj.bias": "ssm_dt.bias", "mixer.A_log": "ssm_a", "mixer.D": "ssm_d",
           "mixer.out_proj.weight": "ssm_out.weight"}
    g = {}
    for k, v in tensors.items():
        if k in names:
            g[names[k]] = v
        elif k.startswith("layers."):
            _, i, rest = k.split(".", 2)
            if rest in sub:
                if rest == "mixer.A_log":
                    v = -np.exp(v.astype(np.float32))
                elif rest == "mixer.conv1d.weight":
                    v = v.reshape(v.shape[0], -1)
                g[f"blk.{i}.{sub[rest]}"] = v
    if cfg.tie_embeddings:
        g.pop("output.weight", None)

    def get_tensor(name):
        a = g.get(name)
        if a is None:
            return None
        a = np.ascontiguousarray(a.astype(np.float32))
        return a, QType.F32, tuple(reversed(a.shape))
    return cfg, get_tensor


def synthetic_mamba_source(cfg: MambaConfig, seed: int = 0, qtype: str = "Q8_0"):
    """Random-init Mamba weights (HF init statistics: dt bias = inv-softplus of U[1e-3, 1e-1],
    A = -[1..N]); the big projections in a real quantised block format when K allows it."""
    from ..ops.quant import random_quantized
    rng = np.random.default_rng(seed)
    H, Di, R, NS, KC = cfg.hidden, cfg.d_inner, cfg.dt_rank, cfg.d_state, cfg.d_conv
    qt = {"Q8_0": QType.Q8_0, "Q4_K": QType.Q4_K, "F16": QType.F16}[qtype]

    def mat(N_, K_, std=0.02):
        if K_ % 256 == 0 and qt != QType.F16:
            return random_quantized(rng, qt, N_, K_, std), qt, (K_, N_)
        a = (rng.standard_normal((N_, K_)) * std).astype(np.float32)
        return a, QType.F32, (K_, N_)

    def vec(a):
        a = np.ascontiguousarray(np.asarray(a, np.float32))
        return a, QType.F32, tuple(reversed(a.shape))
    plan = {"token_embd.weight": lambda: mat(cfg.vocab, H, 0.02), "output_norm.weight": lambda: vec(np.ones(H))}
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        dt = np.exp(rng.uniform(math.log(1e-3), math.log(1e-1), Di))
        plan.update({
            p + "attn_norm.weight": lambda: vec(np.ones(H)),
            p + "ssm_in.weight": (lambda: mat(2 * Di, H)),
            p + "ssm_conv1d.weight": (lambda: vec(rng.standard_normal((Di, KC)) * 0.3)),
            p + "ssm_conv1d.bias": (lambda: vec(rng.standard_normal(Di) * 0.1)),
            p + "ssm_x.weight": (lambda: mat(R + 2 * NS, Di, 0.05)),
            p + "ssm_dt.weight": (lambda: vec(rng.uniform(-1, 1, (Di, R)) * R ** -0.5)),
            p + "ssm_dt.bias": (lambda dt=dt: vec(dt + np.log(-np.expm1(-dt)))),
            p + "ssm_a": (lambda: vec(-np.tile(np.arange(1, NS + 1, dtype=np.float32), (Di, 1)))),
            p + "ssm_d": (lambda: vec(np.ones(Di))),
            p + "ssm_out.weight": (lambda: mat(H, Di, 0.02 / math.sqrt(2 * cfg.n_layers))),
        })
    cache = {}

    def get_tensor(name):
        if name not in plan:
            return None
        if name not in cache:
            cache[name] = plan[name]()
        return cache[name]
    return get_tensor
