"""Device ops: each function runs the HIP kernel on CUDA (ROCm) tensors and an fp32 PyTorch
reference on CPU tensors. The CPU path is the numerics oracle for tests (HIP vs plain fp32) and
the plumbing path the engine uses when no GPU is present; on a GPU box the native library is
mandatory (``_native.kernels`` raises when it is missing).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import _native as N

# ------------------------------------------------------------------------------------------------
# norms


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, *, out_bf16: torch.Tensor | None = None,
            out_q8: tuple | None = None, residual_bf16: torch.Tensor | None = None):
    """y = x / rms(x) * w for fp32 rows x [M, H]; optionally x += residual_bf16 first (written back).
    Writes bf16 rows and/or q8 blocks (xq int8 [M, H], xds fp32 [M, H/32, 2])."""
    M, H = x.shape
    if M == 0:
        return
    if not x.is_cuda:
        if residual_bf16 is not None:
            x.add_(residual_bf16.float())
        y = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w
        if out_bf16 is not None:
            out_bf16.copy_(y)
        if out_q8 is not None:
            _quant_q8_ref(y, *out_q8)
        return
    xq, xds = out_q8 if out_q8 is not None else (None, None)
    if out_bf16 is not None:
        N.ensure_act(out_bf16.dtype)
    N.kcall("mxk_rmsnorm", x.data_ptr(), x.stride(0), N.ptr(residual_bf16),
            residual_bf16.stride(0) if residual_bf16 is not None else 0,
            x.data_ptr() if residual_bf16 is not None else None, w.data_ptr(), N.ptr(out_bf16),
            out_bf16.stride(0) if out_bf16 is not None else 0, N.ptr(xq), N.ptr(xds), M, H, float(eps),
            N.stream_ptr())


def rmsnorm_add(y: torch.Tensor, w: torch.Tensor, eps: float, h: torch.Tensor):
    """h += y / rms(y) * w (fp32 rows [M, H]; Gemma's post-attention / post-FFN norm)."""
    M, H = y.shape
    if M == 0:
        return h
    if not y.is_cuda:
        h.add_(y * torch.rsqrt(y.pow(2).mean(-1, keepdim=True) + eps) * w)
        return h
    N.kcall("mxk_rmsnorm_add", y.data_ptr(), y.stride(0), w.data_ptr(), h.data_ptr(), h.stride(0), M, H,
            float(eps), N.stream_ptr())
    return h


def _quant_q8_ref(y: torch.Tensor, xq: torch.Tensor, xds: torch.Tensor):
    M, K = y.shape
    b = y.float().reshape(M, K // 32, 32)
    d = b.abs().amax(-1) / 127.0
    idd = torch.where(d > 0, 1.0 / d.clamp_min(1e-30), torch.zeros_like(d))
    q = torch.round(b * idd[..., None]).clamp(-127, 127)
    xq.copy_(q.reshape(M, K).to(torch.int8))
    ds = xds.view(M, K // 32, 2)
    ds[..., 0] = d
    ds[..., 1] = d * q.sum(-1)


def quant_q8(x: torch.Tensor, xq: torch.Tensor, xds: torch.Tensor):
    M, K = x.shape
    if M == 0:
        return
    if not x.is_cuda:
        return _quant_q8_ref(x, xq, xds)
    N.ensure_act(x.dtype)
    N.kcall("mxk_quant_q8", x.data_ptr(), x.stride(0), xq.data_ptr(), xds.data_ptr(), M, K, N.stream_ptr())


def layernorm(x: torch.Tensor, g: torch.Tensor | None, b: torch.Tensor | None, eps: float,
              out: torch.Tensor, residual: torch.Tensor | None = None, xsum: torch.Tensor | None = None):
    """fp32 x [M, H] (+ residual) -> layernorm -> out (bf16 or fp32)."""
    M, H = x.shape
    if M == 0:
        return out
    if not x.is_cuda:
        v = x + residual if residual is not None else x
        if xsum is not None:
            xsum.copy_(v)
        out.copy_(F.layer_norm(v, (H,), g, b, eps))
        return out
    ob = out if out.dtype in (torch.bfloat16, torch.float16) else None
    of = out if out.dtype == torch.float32 else None
    if ob is not None:
        N.ensure_act(ob.dtype)
    N.kcall("mxk_layernorm", x.data_ptr(), x.stride(0), N.ptr(residual), residual.stride(0) if residual is not None else 0,
            N.ptr(xsum), N.ptr(g), N.ptr(b), N.ptr(ob), N.ptr(of), out.stride(0), M, H, float(eps), N.stream_ptr())
    return out


def groupnorm_nhwc(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, groups: int, eps: float, silu: bool,
                   out: torch.Tensor | None = None):
    """x fp32 [N, H, W, C] (channels-last)."""
    n, h, w, c = x.shape
    out = torch.empty_like(x) if out is None else out
    if not x.is_cuda:
        y = F.group_norm(x.permute(0, 3, 1, 2), groups, g, b, eps)
        if silu:
            y = F.silu(y)
        out.copy_(y.permute(0, 2, 3, 1))
        return out
    N.kcall("mxk_groupnorm_nhwc", x.data_ptr(), out.data_ptr(), g.data_ptr(), b.data_ptr(), n, h * w, c, groups,
            float(eps), int(silu), N.stream_ptr())
    return out


def layernorm_mod(x: torch.Tensor, scale: torch.Tensor | None, shift: torch.Tensor | None, rows_per_b: int,
                  out: torch.Tensor, eps: float = 1e-6):
    """adaLN: out = LN(x) * (1 + scale[b]) + shift[b], b = row // rows_per_b (diffusion.hip).
    x fp32 [M, H]; scale/shift fp32 [B, >=H] row views (any row stride); out act16 [M, H]."""
    M, H = x.shape
    if M == 0:
        return out
    if not x.is_cuda:
        y = F.layer_norm(x, (H,), eps=eps).view(-1, rows_per_b, H)
        if scale is not None:
            y = y * (1 + scale[:, None, :H])
        if shift is not None:
            y = y + shift[:, None, :H]
        out.copy_(y.reshape(M, H))
        return out
    N.ensure_act(out.dtype)
    ld = (scale if scale is not None else shift).stride(0) if (scale is not None or shift is not None) else 0
    if scale is not None and shift is not None and scale.stride(0) != shift.stride(0):
        raise ValueError("layernorm_mod: scale/shift must share a row stride")
    N.kcall("mxk_layernorm_mod", x.data_ptr(), x.stride(0), N.ptr(scale), N.ptr(shift), ld, rows_per_b,
            out.data_ptr(), out.stride(0), M, H, float(eps), N.stream_ptr())
    return out


def gate_add(x: torch.Tensor, y: torch.Tensor, gate: torch.Tensor | None, rows_per_b: int):
    """x (fp32 [M, H]) += gate[b] * y (act16 [M, H]); gate fp32 [B, >=H] row view or None (= 1)."""
    M, H = x.shape
    if M == 0:
        return x
    if not x.is_cuda:
        yy = y.float().view(-1, rows_per_b, H)
        if gate is not None:
            yy = yy * gate[:, None, :H]
        x.add_(yy.reshape(M, H))
        return x
    N.ensure_act(y.dtype)
    N.kcall("mxk_gate_add", x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), N.ptr(gate),
            gate.stride(0) if gate is not None else 0, rows_per_b, M, H, N.stream_ptr())
    return x


_GN_WS: dict = {}


def groupnorm16(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int, eps: float, silu: bool,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """GroupNorm (+SiLU) over an NCHW-shaped, channels_last 16-bit tensor (diffusion.hip); CPU: fp32."""
    n, c, h, w = x.shape
    if not x.is_cuda:
        y = F.group_norm(x.float(), groups, gamma, beta, eps)
        y = F.silu(y) if silu else y
        y = y.to(x.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    if out is None:
        out = torch.empty_like(x, memory_format=torch.channels_last)
    key = (x.device, n * groups)
    ws = _GN_WS.get(key)
    if ws is None:
        ws = _GN_WS[key] = torch.empty(n * groups * 2, dtype=torch.float64, device=x.device)
    N.ensure_act(x.dtype)
    N.kcall("mxk_groupnorm16", x.data_ptr(), out.data_ptr(), gamma.data_ptr(), beta.data_ptr(), n, h * w, c, groups,
            float(eps), int(silu), ws.data_ptr(), N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------------
# rotary embeddings


def rope_inv_freq(rot_dim: int, base: float = 10000.0, scale: float = 1.0, scaling: str = "none",
                  orig_ctx: int = 0, ext_factor: float = -1.0, beta_fast: float = 32.0, beta_slow: float = 1.0,
                  llama3: dict | None = None, freq_factors=None):
    """inv_freq table [rot_dim/2] and attention magnitude factor for the rope_kv kernel.
    Supports none/linear scaling, llama3.1 frequency smoothing, YaRN ramp (ext_factor) and
    per-frequency factors (GGUF rope_freqs)."""
    i = torch.arange(0, rot_dim, 2, dtype=torch.float64)
    inv = 1.0 / (base ** (i / rot_dim))
    attn_factor = 1.0
    if freq_factors is not None:
        inv = inv / torch.as_tensor(freq_factors, dtype=torch.float64)[: inv.numel()]
    if llama3:
        factor = llama3.get("factor", 8.0)
        lo, hi = llama3.get("low_freq_factor", 1.0), llama3.get("high_freq_factor", 4.0)
        old = llama3.get("original_max_position_embeddings", 8192)
        wl = 2 * math.pi / inv
        lo_wl, hi_wl = old / lo, old / hi
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    elif scaling == "linear" and scale not in (0.0, 1.0):
        inv = inv * scale
    elif scaling == "yarn" and scale not in (0.0, 1.0):
        # scale = freq_scale (= 1/factor) as in llama.cpp
        factor = 1.0 / scale
        orig = orig_ctx or 4096

        def corr_dim(nrot):
            return rot_dim * math.log(orig / (nrot * 2 * math.pi)) / (2 * math.log(base))

        low = max(math.floor(corr_dim(beta_fast)), 0)
        high = min(math.ceil(corr_dim(beta_slow)), rot_dim - 1)
        ramp = ((i / 2 - low) / max(high - low, 1e-3)).clamp(0, 1)
        ext = 1.0 if ext_factor < 0 else ext_factor
        mask = (1 - ramp) * ext
        inv = inv / factor * (1 - mask) + inv * mask
        attn_factor = 0.1 * math.log(factor) + 1.0
    return inv.float(), float(attn_factor)


def rope_kv(qkv: torch.Tensor, bias: torch.Tensor | None, positions: torch.Tensor, slots: torch.Tensor,
            inv_freq: torch.Tensor, attn_factor: float, Hq: int, Hkv: int, D: int, rot_dim: int, neox: bool,
            q_out: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_size: int,
            qk_norm: tuple | None = None, zero_after: bool = False):
    """qkv fp32 [T, (Hq+2Hkv)*D] -> q_out bf16 [T, Hq, D]; K/V scattered into the paged cache
    [num_blocks, Hkv, block_size, D] at `slots` (flat block*bs+offset; -1 skips). zero_after (GPU):
    the consumed qkv rows are left zeroed, ready for the next split-K accumulation into them."""
    T = qkv.shape[0]
    if T == 0:
        return
    if not qkv.is_cuda:
        x = qkv.float()
        if bias is not None:
            x = x + bias
        q = x[:, : Hq * D].reshape(T, Hq, D)
        k = x[:, Hq * D:(Hq + Hkv) * D].reshape(T, Hkv, D)
        v = x[:, (Hq + Hkv) * D:].reshape(T, Hkv, D)
        if qk_norm is not None:
            qn, kn, eps = qk_norm
            q = q * torch.rsqrt(q.pow(2).mean(-1, keepdim=True) + eps) * qn
            k = k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True) + eps) * kn
        ang = positions.double()[:, None] * inv_freq.double()[None, :]
        cos = (torch.cos(ang) * attn_factor).float()
        sin = (torch.sin(ang) * attn_factor).float()

        def rot(t):
            t = t.clone()
            r = t[..., :rot_dim]
            if neox:
                a, b = r[..., : rot_dim // 2], r[..., rot_dim // 2:]
                c, s = cos[:, None, :], sin[:, None, :]
                t[..., :rot_dim] = torch.cat([a * c - b * s, a * s + b * c], -1)
            else:
                a, b = r[..., 0::2], r[..., 1::2]
                c, s = cos[:, None, :], sin[:, None, :]
                out = torch.empty_like(r)
                out[..., 0::2] = a * c - b * s
                out[..., 1::2] = a * s + b * c
                t[..., :rot_dim] = out
            return t

        q_out.copy_(rot(q).to(q_out.dtype))
        kr = rot(k)
        kvf = kv_format(k_cache)
        if kvf >= 2:  # the kernel stages bf16 rows before quantising them: same rounding here
            from .kvq import quantize_rows
            kq = torch.from_numpy(quantize_rows(kr.to(torch.bfloat16).float().reshape(-1, D), kvf)).view(T, Hkv, -1)
            vq = torch.from_numpy(quantize_rows(v.to(torch.bfloat16).float().reshape(-1, D), kvf)).view(T, Hkv, -1)
        for t in range(T):
            s = int(slots[t])
            if s < 0:
                continue
            blk, off = divmod(s, block_size)
            if kvf >= 2:
                k_cache[blk, :, off, :] = kq[t]
                v_cache[blk, :, off, :] = vq[t]
            else:
                k_cache[blk, :, off, :] = _to_cache(kr[t], k_cache.dtype)
                v_cache[blk, :, off, :] = _to_cache(v[t], v_cache.dtype)
        return
    kvf = kv_format(k_cache)
    if kvf >= 2:
        # block-quantised cache: the rotated K and V rows go to a bf16 staging buffer [T, Hkv, D] (identity slots,
        # block size 1), then kvq.hip quantises them into their paged slots (one extra launch per layer)
        ks = torch.empty(T, Hkv, D, dtype=torch.bfloat16, device=qkv.device)
        vs = torch.empty_like(ks)
        ident = torch.arange(T, dtype=torch.int32, device=qkv.device)
        N.kcall("mxk_rope_kv", qkv.data_ptr(), N.ptr(bias), positions.data_ptr(), ident.data_ptr(),
                inv_freq.data_ptr(), float(attn_factor), T, Hq, Hkv, D, rot_dim, int(neox), q_out.data_ptr(),
                ks.data_ptr(), vs.data_ptr(), 1, N.ptr(qk_norm[0]) if qk_norm else None,
                N.ptr(qk_norm[1]) if qk_norm else None, float(qk_norm[2]) if qk_norm else 0.0, int(zero_after), 0,
                N.stream_ptr())
        N.kcall("mxk_kvq_append", kvf, ks.data_ptr(), vs.data_ptr(), slots.data_ptr(), T, Hkv, D, block_size,
                k_cache.data_ptr(), v_cache.data_ptr(), N.stream_ptr())
        return
    N.kcall("mxk_rope_kv", qkv.data_ptr(), N.ptr(bias), positions.data_ptr(), slots.data_ptr(), inv_freq.data_ptr(),
            float(attn_factor), T, Hq, Hkv, D, rot_dim, int(neox), q_out.data_ptr(), k_cache.data_ptr(),
            v_cache.data_ptr(), block_size, N.ptr(qk_norm[0]) if qk_norm else None,
            N.ptr(qk_norm[1]) if qk_norm else None, float(qk_norm[2]) if qk_norm else 0.0, int(zero_after),
            int(is_fp8(k_cache)), N.stream_ptr())


from .kvq import kv_format  # noqa: E402  (0 bf16, 1 fp8, 2.. llama.cpp block formats)

FP8_KV = torch.float8_e4m3fn  # OCP e4m3: the gfx950 hardware conversion format
FP8_MAX = 448.0


def is_fp8(t: torch.Tensor) -> bool:
    return t.dtype == FP8_KV


def _to_cache(x: torch.Tensor, dtype) -> torch.Tensor:
    """Cast for a KV-cache store; fp8 saturates to +-448 like the kernel (torch's cast gives NaN)."""
    if dtype == FP8_KV:
        x = x.clamp(-FP8_MAX, FP8_MAX)
    return x.to(dtype)


# ------------------------------------------------------------------------------------------------
# attention


def _attn_ref_one(q, k_cache, v_cache, table, ctx: int, qpos0: int, scale: float, block_size: int,
                  window: int = 0, softcap: float = 0.0):
    """q [t, Hq, D] for query positions qpos0..qpos0+t-1 of one sequence; causal over ctx keys
    (sliding `window` > 0: keys with qpos - kpos < window; `softcap` > 0: tanh score capping)."""
    t, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    nb = (ctx + block_size - 1) // block_size
    blocks = table[:nb].long()
    if kv_format(k_cache) >= 2:  # block-quantised rows: dequantise the blocks this sequence reads
        from .kvq import dequant_cache
        kvf = kv_format(k_cache)
        kb, vb = dequant_cache(k_cache[blocks], kvf, D), dequant_cache(v_cache[blocks], kvf, D)
    else:
        kb, vb = k_cache[blocks], v_cache[blocks]
    k = kb.permute(1, 0, 2, 3).reshape(Hkv, nb * block_size, D)[:, :ctx].float()
    v = vb.permute(1, 0, 2, 3).reshape(Hkv, nb * block_size, D)[:, :ctx].float()
    G = Hq // Hkv
    k = k.repeat_interleave(G, 0)
    v = v.repeat_interleave(G, 0)
    s = torch.einsum("thd,hkd->htk", q.float(), k) * scale
    if softcap > 0:
        s = softcap * torch.tanh(s / softcap)
    qp = torch.arange(qpos0, qpos0 + t)[:, None]
    kp = torch.arange(ctx)[None, :]
    bad = kp > qp
    if window > 0:
        bad = bad | (kp <= qp - window)
    s = s.masked_fill(bad[None], float("-inf"))
    p = torch.softmax(s, -1)
    return torch.einsum("htk,hkd->thd", p, v)


ATTN_DECODE_IMPL = __import__("os").environ.get("MX_ATTN_DECODE", "mfma")
# in-kernel split-K merge (last-arriving workgroup): measured slower on MI355X at batch 1 and 2.3x slower at
# 128 sequences (profiles/r2_attn_decode_fused_merge_negative.md: the device-scope fences serialise the
# workgroups); kept as an opt-in for experiments, the separate reduce launch is the default
FUSED_DECODE_MERGE = __import__("os").environ.get("MX_ATTN_FUSED_MERGE", "0") == "1"


def attn_decode(q: torch.Tensor, k_cache, v_cache, block_tables: torch.Tensor, seq_lens: torch.Tensor,
                scale: float, out: torch.Tensor, part_size: int = 256, n_parts: int | None = None,
                workspace: tuple | None = None, max_seq_len: int | None = None, window: int = 0,
                softcap: float = 0.0, impl: str | None = None):
    """q bf16 [B, Hq, D] (one query token per sequence, at position seq_len-1).
    impl: "mfma" (QK^T / PV on the matrix cores, head dims 64/128, <= 16 q heads per kv head) or
    "valu" (any shape); default MX_ATTN_DECODE (mfma)."""
    B, Hq, D = q.shape
    if B == 0:
        return out
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    if not q.is_cuda:
        for b in range(B):
            L = int(seq_lens[b])
            out[b] = _attn_ref_one(q[b:b + 1], k_cache, v_cache, block_tables[b], L, L - 1, scale, bs, window,
                                   softcap)[0].to(out.dtype)
        return out
    if n_parts is None:
        ml = max_seq_len if max_seq_len is not None else int(seq_lens.max())
        n_parts = max(1, -(-ml // part_size))
    cnt = None
    if n_parts > 1:
        if workspace is None:
            ml_t = torch.empty((B * Hq * n_parts, 2), dtype=torch.float32, device=q.device)
            po = torch.empty((B * Hq * n_parts, D), dtype=torch.float32, device=q.device)
            cnt = torch.zeros(B * Hkv, dtype=torch.int32, device=q.device)
        else:
            ml_t, po = workspace[:2]
            cnt = workspace[2] if len(workspace) > 2 else None
            if ml_t.numel() < B * Hq * n_parts * 2 or po.numel() < B * Hq * n_parts * D:
                raise ValueError(f"attn_decode: workspace holds {ml_t.numel() // 2} partial rows, "
                                 f"needs {B * Hq * n_parts} (B {B} x Hq {Hq} x {n_parts} partitions)")
    else:
        ml_t = po = None
    N.ensure_act(out.dtype)
    mfma = (impl or ATTN_DECODE_IMPL) == "mfma" and D in (64, 128) and Hq // Hkv <= 16
    if kv_format(k_cache) >= 2 and not mfma:
        raise ValueError(f"block-quantised KV caches need the MFMA decode kernel (head dim 64 / 128, <= 16 q heads per "
                         f"kv head); got D {D}, {Hq // Hkv} q heads per kv head")
    args = [q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
            block_tables.stride(0), seq_lens.data_ptr(), B, Hq, Hkv, D, bs, float(scale), int(window), float(softcap),
            part_size, n_parts, out.data_ptr(), out.stride(0), N.ptr(ml_t), N.ptr(po), kv_format(k_cache)]
    if mfma:
        # partition merge inside the attention kernel (zeroed per-(seq, kv head) counters), else a reduce launch
        if cnt is not None and (cnt.numel() < B * Hkv or not FUSED_DECODE_MERGE):
            cnt = None
        N.kcall("mxk_attn_decode_mfma", *args, N.ptr(cnt), N.stream_ptr())
    else:
        N.kcall("mxk_attn_decode", *args, N.stream_ptr())
    return out


def prefill_tiles(q_lens, rows_per_tile: int):
    seqs, q0s = [], []
    for s, ql in enumerate(q_lens):
        for q0 in range(0, int(ql), rows_per_tile):
            seqs.append(s)
            q0s.append(q0)
    return seqs, q0s


ATTN_VMODE = int(__import__("os").environ.get("MX_ATTN_VMODE", "0"))


def attn_prefill(q: torch.Tensor, k_cache, v_cache, block_tables: torch.Tensor, cu_q: torch.Tensor,
                 ctx_lens: torch.Tensor, scale: float, out: torch.Tensor, q_lens_host=None, ctx_lens_host=None,
                 vmode: int | None = None, window: int = 0, softcap: float = 0.0, tiles=None):
    """q bf16 [T, Hq, D] for S sequences (cu_q [S+1]); keys 0..ctx_len-1 from the paged cache.
    tiles: optional device (seq, q0) int32 tile lists (prefill_tiles(), padded with seq -1) prepared
    once per step by the engine — no host lists needed, so the launch is hipGraph-capturable."""
    T, Hq, D = q.shape
    if T == 0:
        return out
    if tiles is not None and q.is_cuda:
        Hkv, bs = k_cache.shape[1], k_cache.shape[2]
        N.ensure_act(out.dtype)
        N.kcall("mxk_attn_prefill", q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
                block_tables.stride(0), tiles[0].data_ptr(), tiles[1].data_ptr(), int(tiles[0].numel()),
                cu_q.data_ptr(), ctx_lens.data_ptr(), Hq, Hkv, D, bs, float(scale), int(window), float(softcap),
                out.data_ptr(), ATTN_VMODE if vmode is None else int(vmode), kv_format(k_cache), N.stream_ptr())
        return out
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    cu = cu_q.tolist() if q_lens_host is None else None
    if q_lens_host is None:
        q_lens_host = [cu[i + 1] - cu[i] for i in range(len(cu) - 1)]
    if ctx_lens_host is None:
        ctx_lens_host = ctx_lens.tolist()
    if not q.is_cuda:
        off = 0
        for s, ql in enumerate(q_lens_host):
            ctx = int(ctx_lens_host[s])
            out[off:off + ql] = _attn_ref_one(q[off:off + ql], k_cache, v_cache, block_tables[s], ctx, ctx - ql,
                                              scale, bs, window, softcap).to(out.dtype)
            off += ql
        return out
    rows = N.kernels().mxk_attn_prefill_rows(Hq, Hkv)
    seqs, q0s = prefill_tiles(q_lens_host, rows)
    tiles = torch.tensor([seqs, q0s], dtype=torch.int32).to(q.device, non_blocking=True)
    N.ensure_act(out.dtype)
    N.kcall("mxk_attn_prefill", q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
            block_tables.stride(0), tiles[0].data_ptr(), tiles[1].data_ptr(), len(seqs), cu_q.data_ptr(),
            ctx_lens.data_ptr(), Hq, Hkv, D, bs, float(scale), int(window), float(softcap), out.data_ptr(),
            ATTN_VMODE if vmode is None else int(vmode), kv_format(k_cache), N.stream_ptr())
    return out


def attn_dense(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: torch.Tensor, B: int, Sq: int, Sk: int,
               Hq: int, Hkv: int, D: int, scale: float, causal: bool = False,
               qlen: torch.Tensor | None = None, klen: torch.Tensor | None = None, kv_rows: int = 0,
               rbias: torch.Tensor | None = None):
    """Flash attention over dense token-major 16-bit tensors (attention_dense.hip).

    q/out: [B*Sq, >= Hq*D] (row stride = .stride(0)); k/v: [B*kv_rows, >= Hkv*D] of which the first
    Sk rows per batch are read (kv_rows = 0 -> Sk; a fixed-capacity KV cache passes its capacity).
    Head dims other than 64/128/512 are zero-padded to the next supported size (exact: padded dims add
    0 to q.k and produce 0 output columns that are dropped). klen/qlen: optional int32 [B] valid
    lengths (padding). rbias: optional fp32 [Hq, Sq + Sk - 1] additive bias by key-minus-query offset
    (index j - i + Sq - 1; T5's relative position bias), added to the scaled logits."""
    if B == 0 or Sq == 0:
        return out
    R = kv_rows or Sk
    if not q.is_cuda:
        qf = q[:, :Hq * D].float().view(B, Sq, Hq, D).transpose(1, 2)
        kf = k[:B * R, :Hkv * D].float().view(B, R, Hkv, D)[:, :Sk].transpose(1, 2)
        vf = v[:B * R, :Hkv * D].float().view(B, R, Hkv, D)[:, :Sk].transpose(1, 2)
        if Hq != Hkv:
            kf = kf.repeat_interleave(Hq // Hkv, 1)
            vf = vf.repeat_interleave(Hq // Hkv, 1)
        s = torch.einsum("bhqd,bhkd->bhqk", qf, kf) * scale
        kp = torch.arange(Sk)
        if rbias is not None:
            off = kp[None, :] - torch.arange(Sq)[:, None] + Sq - 1
            s = s + rbias.float().cpu()[:, off][None]
        mask = torch.zeros(B, 1, Sq, Sk, dtype=torch.bool)
        if causal:
            mask |= (kp[None, :] > (torch.arange(Sq)[:, None] + (Sk - Sq)))[None, None]
        if klen is not None:
            mask |= (kp[None, None, None, :] >= klen.view(B, 1, 1, 1).cpu())
        s = s.masked_fill(mask, float("-inf"))
        p = torch.softmax(s, -1).nan_to_num(0.0)
        o = torch.einsum("bhqk,bhkd->bqhd", p, vf).reshape(B * Sq, Hq * D)
        if qlen is not None:
            for b in range(B):
                o[b * Sq + int(qlen[b]):(b + 1) * Sq] = 0
        out[:, :Hq * D].copy_(o)
        return out
    Dp = 64 if D <= 64 else 128 if D <= 128 else 512 if D <= 512 else 0
    if not Dp:
        raise ValueError(f"attn_dense: head dim {D} > 512")
    if Dp != D:
        def pad(t, H):
            x = t[:, :H * D].reshape(t.shape[0], H, D)
            return torch.nn.functional.pad(x, (0, Dp - D)).reshape(t.shape[0], H * Dp)
        qp, kp_, vp = pad(q, Hq), pad(k[:B * R], Hkv), pad(v[:B * R], Hkv)
        op = torch.empty((out.shape[0], Hq * Dp), dtype=out.dtype, device=out.device)
        attn_dense(qp, kp_, vp, op, B, Sq, Sk, Hq, Hkv, Dp, scale, causal, qlen, klen, R, rbias)
        out[:, :Hq * D].copy_(op.view(-1, Hq, Dp)[..., :D].reshape(-1, Hq * D))
        return out
    if not (q.dtype == k.dtype == v.dtype == out.dtype):
        raise ValueError("attn_dense: q/k/v/out must share one 16-bit dtype")
    if rbias is not None and (rbias.dtype != torch.float32 or not rbias.is_contiguous() or
                              tuple(rbias.shape) != (Hq, Sq + Sk - 1)):
        raise ValueError(f"attn_dense: rbias must be contiguous fp32 [{Hq}, {Sq + Sk - 1}]")
    N.ensure_act(out.dtype)
    N.kcall("mxk_attn_dense", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0),
            out.data_ptr(), out.stride(0), B, Sq, Sk, Hq, Hkv, D, N.ptr(qlen), N.ptr(klen), int(causal),
            float(scale), int(R), N.ptr(rbias), Sq + Sk - 1, N.stream_ptr())
    return out


# ------------------------------------------------------------------------------------------------
# activations / misc


def glu(gate: torch.Tensor, up: torch.Tensor, out: torch.Tensor, act: str = "silu"):
    a = {"silu": 0, "gelu": 1, "gelu_tanh": 1, "gelu_erf": 2}[act]
    if not gate.is_cuda:
        g = gate.float()
        y = F.silu(g) if a == 0 else F.gelu(g, approximate="tanh" if a == 1 else "none")
        out.copy_(y * up.float())
        return out
    M, Fd = gate.shape
    N.ensure_act(out.dtype)
    N.kcall("mxk_glu", a, gate.data_ptr(), up.data_ptr(), gate.stride(0), out.data_ptr(), out.stride(0), M, Fd,
            N.stream_ptr())
    return out


def gather_rows(table: torch.Tensor, ids: torch.Tensor, out: torch.Tensor, scale: float = 1.0):
    """dense embedding gather -> fp32 rows"""
    if not table.is_cuda:
        out.copy_(table[ids.long()].float() * scale)
        return out
    dt = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[table.dtype]
    N.kcall("mxk_gather_rows", table.data_ptr(), dt, ids.data_ptr(), ids.numel(), table.shape[1], float(scale),
            out.data_ptr(), N.stream_ptr())
    return out


def select_rows(x: torch.Tensor, idx: torch.Tensor, out: torch.Tensor):
    if not x.is_cuda:
        out.copy_(x[idx.long()])
        return out
    N.kcall("mxk_select_rows_f32", x.data_ptr(), x.stride(0), idx.data_ptr(), idx.numel(), x.shape[1], out.data_ptr(),
            out.stride(0), N.stream_ptr())
    return out


def cast_act(x: torch.Tensor, out: torch.Tensor):
    """fp32 -> 16-bit activation (bf16 or f16, by out.dtype)."""
    return cast_bf16(x, out)


def cast_bf16(x: torch.Tensor, out: torch.Tensor):
    if not x.is_cuda:
        out.copy_(x)
        return out
    N.ensure_act(out.dtype)
    N.kcall("mxk_cast_f32_bf16", x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), x.shape[0], x.shape[1],
            N.stream_ptr())
    return out


def wavenet_gate(x: torch.Tensor, H: int) -> torch.Tensor:
    """tanh(x[:, :H]) * sigmoid(x[:, H:]) for x [B, 2H, T] fp32 (audio.hip wavenet_gate)."""
    if not x.is_cuda:
        return torch.tanh(x[:, :H]) * torch.sigmoid(x[:, H:])
    x = x.contiguous().float()
    B, _, T = x.shape
    out = torch.empty(B, H, T, device=x.device, dtype=torch.float32)
    N.kcall("mxk_wavenet_gate", x.data_ptr(), out.data_ptr(), B, H, T, N.stream_ptr())
    return out
