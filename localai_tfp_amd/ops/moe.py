"""Mixture-of-experts FFN (Mixtral, Qwen2-MoE, Qwen3-MoE GGUF layouts).

Parity target: llama.cpp's build_moe_ffn as the reference's llama-cpp backend runs it (router
softmax, top-k, optional weight renormalisation, ggml_mul_mat_id over the stacked
`ffn_{gate,up,down}_exps` tensors, optional shared expert with a sigmoid gate for Qwen2-MoE).

GPU path (all device-side, hipGraph-capturable):
    moe_router (moe.hip: the router GEMV, one expert per wave with its fp32 row requested whole, 8 tokens per
    workgroup from LDS; for <= 8 rows it also computes the FFN RMSNorm) -> moe_route (softmax + top-k, one wave per
    token; in-launch variants are opt-in: profiles/r6_fence_free_handoffs.md) -> then, with the expert stacks in the
    t32 layout (models/llama.py finalize_layout;
    16-row-interleaved gate|up per expert):
      * decode (P = T k pairs <= GEMV_MAX_PAIRS): qmv_moe (qmv.hip) — one workgroup per (pair, 32 columns of its
        expert), q8 activations, gate|up SwiGLU into [P, F]; then qmv_moe_down — one workgroup per (token, 32
        columns of H) walks the token's k experts and adds the routing-weighted sum into h (the combine fused: no
        [P, H] buffer, one writer per output);
      * larger batches: moe_sort (counting sort of the pairs by expert, per-expert tile prefix) -> grouped qmm2
        (qmm2_impl.h Q2Group: 32- / 64-row MFMA tiles per expert, A rows gathered through the sort) for gate|up
        SwiGLU and down, the down epilogue adding each sorted row times its routing weight into the token's
        residual row (fp32 atomics; MX_MOE_GROUPED_COMBINE=0: [P, H] buffer + moe_combine in fixed order).
    Expert stacks that do not fit the t32 layout (a row count
    per expert or K that is not whole 32-row groups / 256-k super-blocks) keep the row layout and the qgemm16
    grouped kernel.
CPU path: the same math with dequantised fp32 expert weights (numerics oracle).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import _native as N
from . import core as K
from .linear import ACT_DTYPE, EPI_F32, EPI_SWIGLU, QWeight, qmatmul

E16_F32, E16_ADD_F32, E16_SWIGLU = 0, 2, 3
MOE_T32 = (12, 13, 14, 8)  # Q4_K, Q5_K, Q6_K, Q8_0: block formats with grouped t32 kernels (qmv_moe, qmm2 grouped)
GEMV_MAX_PAIRS = 64  # token-expert pairs up to which the grouped decode GEMV runs (above: the grouped qmm2 GEMM)


@dataclass
class MoEWeights:
    router: torch.Tensor  # fp32 [E, H]
    gate: QWeight | None  # [E*F, H] stacked (CPU / non-interleavable)
    up: QWeight | None
    gate_up: QWeight | None  # [E*2F, H], gate|up interleaved in 16-row groups per expert (GPU)
    down: QWeight  # [E*H, F] stacked
    n_expert: int
    n_used: int
    ffn: int  # per-expert F
    renorm: bool
    sh_gate_up: QWeight | None = None  # shared expert (Qwen2-MoE)
    sh_gate: QWeight | None = None
    sh_up: QWeight | None = None
    sh_down: QWeight | None = None
    sh_inp: torch.Tensor | None = None  # fp32 [H] sigmoid gate of the shared expert
    e0: int = 0  # expert parallelism: this rank holds experts [e0, e0 + n_local) of the n_expert
    n_local: int = 0  # 0 = all
    t32: bool = False  # gate_up / down re-laid in the t32 layout (grouped qmv / qmm2 kernels)

    def nbytes(self) -> int:
        n = self.router.numel() * 4
        for w in (self.gate, self.up, self.gate_up, self.down, self.sh_gate_up, self.sh_gate, self.sh_up,
                  self.sh_down):
            if w is not None:
                n += w.nbytes()
        return n

    def to_t32(self) -> bool:
        """Re-lay gate|up and down (and the shared expert) out in the t32 layout when every expert's rows are whole
        32-row groups and K whole 256-k super-blocks of a format the grouped kernels decode; returns self.t32."""
        El = self.n_local or self.n_expert
        gu, d = self.gate_up, self.down
        if (not self.t32 and gu is not None and gu.is_quant and d.is_quant and gu.data.is_cuda
                and (2 * self.ffn) % 32 == 0 and d.N % (32 * El) == 0 and gu.K % 256 == 0 and d.K % 256 == 0
                and ACT_DTYPE == torch.float16 and int(gu.qtype) in MOE_T32 and int(d.qtype) in MOE_T32):
            self.t32 = gu.to_t32() and d.to_t32()
        for w in (self.sh_gate_up, self.sh_down, self.sh_gate, self.sh_up):
            if isinstance(w, QWeight):
                w.to_t32()
        return self.t32

    def build_bf16_cache(self):
        for w in (self.sh_gate_up, self.sh_down):
            if w is not None:
                w.build_bf16_cache()


def route_ref(logits: torch.Tensor, k: int, renorm: bool):
    p = torch.softmax(logits.float(), -1)
    w, ids = torch.topk(p, k, -1)  # ties -> lower index (torch.topk is stable on CPU for equal values)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return ids.int(), w


_TICKETS: dict = {}
# top-k in the router launch (last workgroup of a token block, after a device-scope fence): off by default — the
# fence writes back the L2 on gfx950 and at c64 the fused router took 48 us / layer against 15 + 7 us for two launches
# (profiles/r6_moe_qwen3_30b.md)
ROUTE_FUSE = __import__("os").environ.get("MX_MOE_ROUTE_FUSE", "0") == "1"
# FFN RMSNorm inside the router launch for batches of at most one router token block (8 rows): c1 352 vs 339 tok/s;
# above, every expert-block workgroup would redo its tokens' norm (c64 7,531 vs 7,668 unfused)
NORM_FUSE = __import__("os").environ.get("MX_MOE_NORM_FUSE", "1") != "0"
NORM_FUSE_MAX_T = 8
# routing inside the single-workgroup counting sort for grouped batches of at most this many tokens: opt-in
# (MX_MOE_ROUTE_SORT=1) — one workgroup routing 64 tokens is a serial tail, c64 7,032 vs 7,552 tok/s with two launches
ROUTE_SORT = __import__("os").environ.get("MX_MOE_ROUTE_SORT", "0") == "1"
ROUTE_SORT_MAX_T = 64
# grouped (sorted) path: the down projection adds routing-weighted rows straight into the residual (fp32 atomics: the
# k rows of a token come from different experts' tiles, so the sum order is not fixed) instead of a [P, H] buffer + a
# combine launch; MX_MOE_GROUPED_COMBINE=0 keeps the deterministic combine
GROUPED_COMBINE_FUSE = __import__("os").environ.get("MX_MOE_GROUPED_COMBINE", "1") != "0"


def _router_tickets(dev, n: int) -> torch.Tensor:
    """Per-device zeroed ints for the router's last-workgroup routing (the kernel leaves them zeroed, so one buffer
    serves every layer and graph replay). Allocated outside capture by the first (warm-up) forward of a size."""
    t = _TICKETS.get(dev)
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 8192), dtype=torch.int32, device=dev)  # 64k tokens: never regrown under capture
        _TICKETS[dev] = t
    return t


def _grouped_wm(P: int, E: int) -> int:
    avg = P / max(1, min(E, P))
    return 1 if avg <= 16 else 2 if avg <= 40 else 4


def moe_ffn(W: MoEWeights, x: torch.Tensor, h: torch.Tensor, norm: tuple | None = None) -> torch.Tensor:
    """h [T, H] fp32 += MoE(x); x is the normed hidden state in 16-bit (GPU) or fp32 (CPU). norm = (src fp32 [T, H],
    gamma, eps): x is then the OUTPUT buffer of src's RMSNorm — on the GPU fast path the router kernel computes it
    (no separate norm launch), otherwise the norm kernel runs first."""
    T = x.shape[0]
    if T == 0:
        return h
    E, k, F = W.n_expert, W.n_used, W.ffn
    H = h.shape[1]
    if not x.is_cuda:
        if norm is not None:
            K.rmsnorm(norm[0], norm[1], norm[2], out_bf16=x)
        return _moe_ref(W, x.float(), h)
    ids = torch.empty(T, k, dtype=torch.int32, device=x.device)
    wts = torch.empty(T, k, dtype=torch.float32, device=x.device)
    st = N.stream_ptr()
    fast = (x.dtype in (torch.float16, torch.bfloat16) and H % 256 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and W.router.is_contiguous() and E <= 512)
    El = W.n_local or E
    # decode-sized grouped batches: the routing runs inside the sort's single workgroup (moe_route_sort)
    route_in_sort = (fast and W.t32 and El == E and ROUTE_SORT and GEMV_MAX_PAIRS < T * k and T <= ROUTE_SORT_MAX_T)
    fuse_norm = (fast and NORM_FUSE and T <= NORM_FUSE_MAX_T and norm is not None and norm[0].dtype == torch.float32 and norm[0].stride(1) == 1
                 and norm[0].stride(0) % 4 == 0 and norm[1].dtype == torch.float32 and norm[1].is_contiguous())
    if norm is not None and not fuse_norm:
        K.rmsnorm(norm[0], norm[1], norm[2], out_bf16=x)
    if fast:
        N.ensure_act(x.dtype)
        logits = torch.empty(T, E, dtype=torch.float32, device=x.device)
        tk = _router_tickets(x.device, (T + 7) // 8) if (ROUTE_FUSE and not route_in_sort) else None
        hs, g, eps = norm if fuse_norm else (None, None, 0.0)
        N.kcall("mxk_moe_router", x.data_ptr(), x.stride(0), W.router.data_ptr(), T, H, E, k, int(W.renorm),
                None if route_in_sort else ids.data_ptr(), wts.data_ptr(), logits.data_ptr(), N.ptr(tk), N.ptr(hs),
                hs.stride(0) if fuse_norm else 0, N.ptr(g), float(eps), st)
    else:
        logits = x.float() @ W.router.t()
        N.kcall("mxk_moe_route", logits.data_ptr(), logits.stride(0), T, E, k, int(W.renorm), ids.data_ptr(),
                wts.data_ptr(), st)
    if W.t32:
        _experts_t32(W, x, h, ids, wts, El, logits if route_in_sort else None)
        if W.sh_down is not None:
            _shared(W, x, h)
        return h
    y_zero = False
    if El != E:
        # expert parallelism: pairs routed to other ranks' experts go to a null bucket El (sorted last,
        # never computed) with weight 0; the grouped GEMMs run over the El local experts only
        loc = ids - W.e0
        off_rank = (loc < 0) | (loc >= El)
        ids = torch.where(off_rank, torch.full_like(loc, El), loc)
        wts = wts.masked_fill(off_rank, 0.0)
        y_zero = True
    P = T * k
    wm = _grouped_wm(P, E)
    Eb = El + (1 if El != E else 0)  # sort buckets (+ the null bucket)
    off = torch.empty(Eb + 1, dtype=torch.int32, device=x.device)
    tiles = torch.empty(Eb + 1, dtype=torch.int32, device=x.device)
    stok = torch.empty(P, dtype=torch.int32, device=x.device)
    inv = torch.empty(P, dtype=torch.int32, device=x.device)
    N.kcall("mxk_moe_sort", ids.data_ptr(), P, k, Eb, 16 * wm, off.data_ptr(), tiles.data_ptr(), stok.data_ptr(),
            inv.data_ptr(), None, None, st)
    E = El
    act = torch.empty(P, F, dtype=x.dtype, device=x.device)
    N.ensure_act(x.dtype)
    gu = W.gate_up
    N.kcall("mxk_moe_qgemm16", int(gu.qtype), E16_SWIGLU, wm, x.data_ptr(), x.stride(0), stok.data_ptr(),
            gu.data.data_ptr(), N.ptr(gu.dplane), off.data_ptr(), tiles.data_ptr(), E, P, 2 * F, gu.K,
            act.data_ptr(), act.stride(0), st)
    y = (torch.zeros if y_zero else torch.empty)(P, H, dtype=torch.float32, device=x.device)
    d = W.down
    N.kcall("mxk_moe_qgemm16", int(d.qtype), E16_F32, wm, act.data_ptr(), act.stride(0), None, d.data.data_ptr(),
            N.ptr(d.dplane), off.data_ptr(), tiles.data_ptr(), E, P, H, d.K, y.data_ptr(), y.stride(0), st)
    N.kcall("mxk_moe_combine", y.data_ptr(), y.stride(0), inv.data_ptr(), wts.data_ptr(), T, k, H, h.data_ptr(),
            h.stride(0), 1, st)
    if W.sh_down is not None:
        _shared(W, x, h)
    return h


def _experts_t32(W: MoEWeights, x: torch.Tensor, h: torch.Tensor, ids: torch.Tensor, wts: torch.Tensor, El: int,
                 logits: torch.Tensor | None = None):
    """Routed experts on the t32 stacks: grouped decode GEMV (small P) or grouped qmm2 (sorted pairs). logits: the
    routing is still to do and runs inside the sort launch (moe_route_sort)."""
    T, k, F, E = x.shape[0], W.n_used, W.ffn, W.n_expert
    H = h.shape[1]
    P = T * k
    st = N.stream_ptr()
    gu, d = W.gate_up, W.down
    N.ensure_act(x.dtype)
    act = torch.empty(P, F, dtype=x.dtype, device=x.device)
    if P <= GEMV_MAX_PAIRS:
        N.kcall("mxk_qmv_moe", int(gu.qtype), E16_SWIGLU, gu.data.data_ptr(), 2 * F, gu.K, ids.data_ptr(), P, W.e0,
                El, x.data_ptr(), x.stride(0), k, act.data_ptr(), act.stride(0), st)
        if k * d.K * 5 // 4 <= 64 * 1024 and h.stride(1) == 1:
            # down + combine in one launch: h[t] += sum_j w_tj (act_tj . W_e(tj)) (off-rank pairs contribute nothing)
            N.kcall("mxk_qmv_moe_down", int(d.qtype), d.data.data_ptr(), H, d.K, ids.data_ptr(), wts.data_ptr(), T, k,
                    W.e0, El, act.data_ptr(), act.stride(0), h.data_ptr(), h.stride(0), st)
            return
        y = (torch.zeros if El != E else torch.empty)(P, H, dtype=torch.float32, device=x.device)
        N.kcall("mxk_qmv_moe", int(d.qtype), E16_F32, d.data.data_ptr(), H, d.K, ids.data_ptr(), P, W.e0, El,
                act.data_ptr(), act.stride(0), 1, y.data_ptr(), y.stride(0), st)
        N.kcall("mxk_moe_combine", y.data_ptr(), y.stride(0), None, wts.data_ptr(), T, k, H, h.data_ptr(),
                h.stride(0), 1, st)
        return
    if El != E:  # expert parallelism: other ranks' pairs go to a null bucket El, sorted last, never computed
        loc = ids - W.e0
        off_rank = (loc < 0) | (loc >= El)
        ids = torch.where(off_rank, torch.full_like(loc, El), loc)
    wm = 1 if P <= 32 * El else 2
    Eb = El + (1 if El != E else 0)
    off = torch.empty(Eb + 1, dtype=torch.int32, device=x.device)
    tiles = torch.empty(Eb + 1, dtype=torch.int32, device=x.device)
    stok = torch.empty(P, dtype=torch.int32, device=x.device)
    inv = torch.empty(P, dtype=torch.int32, device=x.device)
    fuse = GROUPED_COMBINE_FUSE and h.stride(1) == 1
    swt = torch.empty(P, dtype=torch.float32, device=x.device) if fuse else None
    if logits is not None:
        N.kcall("mxk_moe_route_sort", logits.data_ptr(), logits.stride(0), T, E, k, int(W.renorm), ids.data_ptr(),
                wts.data_ptr(), 32 * wm, off.data_ptr(), tiles.data_ptr(), stok.data_ptr(), inv.data_ptr(), N.ptr(swt),
                st)
    else:
        N.kcall("mxk_moe_sort", ids.data_ptr(), P, k, Eb, 32 * wm, off.data_ptr(), tiles.data_ptr(), stok.data_ptr(),
                inv.data_ptr(), wts.data_ptr(), N.ptr(swt), st)
    N.kcall("mxk_qmm2_grouped", int(gu.qtype), E16_SWIGLU, wm, x.data_ptr(), x.stride(0), stok.data_ptr(),
            gu.data.data_ptr(), P, El, 2 * F, gu.K, tiles.data_ptr(), off.data_ptr(), act.data_ptr(), act.stride(0),
            None, None, st)
    if fuse:
        # down + combine: each sorted row's output, scaled by its routing weight, added into its token's residual row
        N.kcall("mxk_qmm2_grouped", int(d.qtype), E16_ADD_F32, wm, act.data_ptr(), act.stride(0), None,
                d.data.data_ptr(), P, El, H, d.K, tiles.data_ptr(), off.data_ptr(), h.data_ptr(), h.stride(0),
                stok.data_ptr(), swt.data_ptr(), st)
        return
    # rows of pairs routed to another rank's experts stay zero (weight 0 in the combine)
    y = (torch.zeros if El != E else torch.empty)(P, H, dtype=torch.float32, device=x.device)
    N.kcall("mxk_qmm2_grouped", int(d.qtype), E16_F32, wm, act.data_ptr(), act.stride(0), None, d.data.data_ptr(), P,
            El, H, d.K, tiles.data_ptr(), off.data_ptr(), y.data_ptr(), y.stride(0), None, None, st)
    N.kcall("mxk_moe_combine", y.data_ptr(), y.stride(0), inv.data_ptr(), wts.data_ptr(), T, k, H, h.data_ptr(),
            h.stride(0), 1, st)


def _shared(W: MoEWeights, x: torch.Tensor, h: torch.Tensor):
    T = x.shape[0]
    Fs = W.sh_down.K
    act = torch.empty(T, Fs, dtype=x.dtype, device=x.device)
    if W.sh_gate_up is not None:
        qmatmul(W.sh_gate_up, x, EPI_SWIGLU, act)
    else:
        g = torch.empty(T, Fs, dtype=x.dtype, device=x.device)
        u = torch.empty(T, Fs, dtype=x.dtype, device=x.device)
        qmatmul(W.sh_gate, x, 1, g)
        qmatmul(W.sh_up, x, 1, u)
        act.copy_(torch.nn.functional.silu(g.float()) * u.float())
    ys = torch.zeros(T, h.shape[1], dtype=torch.float32, device=x.device)
    qmatmul(W.sh_down, act, EPI_F32, ys, out_zeroed=True)
    if W.sh_inp is not None:
        ys.mul_(torch.sigmoid(x.float() @ W.sh_inp)[:, None])
    h.add_(ys)


def _moe_ref(W: MoEWeights, x: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    E, k, F = W.n_expert, W.n_used, W.ffn
    H = h.shape[1]
    ids, wts = route_ref(x @ W.router.t(), k, W.renorm)
    El = W.n_local or E
    g = W.gate.dense_f32().view(El, F, -1)
    u = W.up.dense_f32().view(El, F, -1)
    d = W.down.dense_f32().view(El, H, F)
    out = torch.zeros_like(h)
    for e in range(El):
        tok, slot = (ids == W.e0 + e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        xe = x[tok]
        a = torch.nn.functional.silu(xe @ g[e].t()) * (xe @ u[e].t())
        out.index_add_(0, tok, (a @ d[e].t()) * wts[tok, slot][:, None])
    h.add_(out)
    if W.sh_down is not None:
        gs, us = W.sh_gate.dense_f32(), W.sh_up.dense_f32()
        ys = (torch.nn.functional.silu(x @ gs.t()) * (x @ us.t())) @ W.sh_down.dense_f32().t()
        if W.sh_inp is not None:
            ys = ys * torch.sigmoid(x @ W.sh_inp)[:, None]
        h.add_(ys)
    return h


__all__ = ["MoEWeights", "moe_ffn", "route_ref", "ACT_DTYPE"]
