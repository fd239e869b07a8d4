"""Quantised linear layers: GPU weight container + M-dependent kernel dispatch.

``QWeight`` owns one [N, K] projection in a GPU-native layout (ops/quant.py). ``qmatmul`` picks:

* M <= 4 and q8 activations available  -> ``mxk_qgemv``   (int8 dot4, HBM-bound decode)
* otherwise                             -> ``mxk_qgemm_mfma`` (dequant-to-bf16 MFMA), with the
  workgroup shape (WM x 16 rows, WN x 16 cols per wave) and split-K chosen so the grid covers the
  256 CUs: split-K partials go through fp32 atomics into either the residual stream (o_proj,
  down_proj: EPI_ADD_F32) or a zeroed fp32 buffer (QKV).
* dense (F16/BF16/F32 or non-native quant types densified at load) -> hipBLASLt via torch.matmul.

On CPU tensors everything runs as an fp32 PyTorch reference (dequantised weights), which is the
numerics oracle for the HIP kernels.
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch

from .. import _native as N
from ..formats.gguf import QType
from . import autotune as _AT
from . import quant as Q

log = logging.getLogger("localai_tfp_amd.ops")

EPI_F32, EPI_BF16, EPI_ADD_F32, EPI_SWIGLU, EPI_GEGLU = 0, 1, 2, 3, 4
GLU_EPIS = (EPI_SWIGLU, EPI_GEGLU)  # gated-FFN epilogues over 16-row interleaved gate|up weights
EPI_ACT = EPI_BF16  # "16-bit activation out" (bf16 or f16 by the output tensor's dtype)
CU_COUNT = 256
_os = __import__("os")
# 16-bit activation format of the model graphs: f16 by default (packed-f16 dequant GEMM, qgemm16.hip);
# MX_ACT=bf16 selects the bf16 kernels.
ACT_DTYPE = torch.bfloat16 if _os.environ.get("MX_ACT", "f16").lower() == "bf16" else torch.float16
# rows at or above this go through the dense 16-bit weight cache (hipBLASLt) when it is enabled;
# below it the quantised MFMA kernels (decode batches) — tuned with tools/bench_qgemm.py.
BF16_CACHE_MIN_M = int(_os.environ.get("MX_BF16_CACHE_MIN_M", "0")) or None


class QWeight:
    """A [N, K] weight. ``qtype`` is a ggml QType for native quant layouts, or "dense"."""

    def __init__(self, N_: int, K: int, qtype, data: torch.Tensor, dplane: torch.Tensor | None = None,
                 raw_ggml: np.ndarray | None = None, raw_qtype: int | None = None, name: str = ""):
        self.N, self.K = int(N_), int(K)
        self.qtype = qtype
        self.data = data
        self.dplane = dplane
        self.name = name
        self._raw = raw_ggml  # kept only for CPU reference dequantisation
        self._raw_qtype = raw_qtype
        self._dense_f32: torch.Tensor | None = None
        self.bf16_cache: torch.Tensor | None = None
        self.layout = "ggml"  # "ggml" (GPU-native block rows) | "t32" (tiled, ops/quant.py tile32)
        self.src_qtype = raw_qtype  # block format of the checkpoint (Q4_0 etc. run as Q8_0: see Q8_EXACT)

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_ggml(cls, raw: np.ndarray, qtype: int, N_: int, K: int, device="cpu", name: str = "",
                  dense_dtype=torch.bfloat16, t32: bool = False):
        """t32: the caller re-lays the weight out with to_t32() (or ensure_kernel_layout()) before use, so
        formats whose kernels exist only in the t32 layout (Q5_K, and Q4_0/Q4_1/Q5_0/Q5_1 as MX4F/MX5F) stay
        in their own bit width; otherwise those run on the Q8_0 kernels."""
        qt = raw_qtype_in = QType(qtype)
        dev = torch.device(device)
        if dev.type == "cpu":
            # CPU: keep the ggml bytes, dequantise lazily for the reference path
            return cls(N_, K, int(qt) if qt in Q.GPU_NATIVE else "dense",
                       torch.empty(0), None, np.asarray(raw), int(qt), name)
        t32_only_ok = t32 and N_ % 32 == 0 and ACT_DTYPE == torch.float16
        if qt in Q.Q32_FAMILY and t32_only_ok and K % 256 == 0:
            raw, qt = Q.to_mxf(raw, qt, N_, K)  # exact: 4/5-bit codes + f16 scale/offset per 32
        if qt in Q.T32_ONLY and not t32_only_ok and K % 256 == 0:
            raw, qt = Q.to_q8_0(raw, qt, N_, K), QType.Q8_0  # no t32 tiling possible: Q8_0 kernels
        if qt in (*Q.Q8_EXACT, *Q.Q8_REQUANT) and qt not in Q.T32_ONLY and K % 256 == 0:
            # no dedicated layout for this block format: carried on the Q8_0 kernels, never densified
            raw, qt = Q.to_q8_0(raw, qt, N_, K), QType.Q8_0
        if qt in Q.GPU_NATIVE and K % 256 == 0:
            data, dpl = Q.repack_for_gpu(raw, qt, N_, K)
            t = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
            d = torch.from_numpy(np.ascontiguousarray(dpl).view(np.int16)).to(dev) if dpl is not None else None
            w = cls(N_, K, int(qt), t, d, None, int(qt), name)
            w.src_qtype = int(QType(raw_qtype_in))
            return w
        if qt not in (QType.F32, QType.F16, QType.BF16):
            log.warning("%s: %s weight with K=%d densified to 16 bits (no quantised kernel layout for it)",
                        name, qt.name, K)
        dense = Q.dequantize(raw, qt, (K, N_))
        t = torch.from_numpy(dense).to(dev, dense_dtype)
        return cls(N_, K, "dense", t, None, None, int(qt), name)

    @classmethod
    def dense(cls, w: torch.Tensor, name: str = ""):
        return cls(w.shape[0], w.shape[1], "dense", w.contiguous(), None, None, None, name)

    @property
    def is_quant(self) -> bool:
        return self.qtype != "dense"

    @property
    def device(self):
        return self.data.device if self.data.numel() else torch.device("cpu")

    def nbytes(self) -> int:
        n = self.data.numel() * self.data.element_size()
        if self.dplane is not None:
            n += self.dplane.numel() * 2
        return n

    # ---------------------------------------------------------------- reference / caches
    def dense_f32(self) -> torch.Tensor:
        """fp32 [N, K] (CPU reference or debugging)."""
        if self._dense_f32 is not None:
            return self._dense_f32
        if self._raw is not None:
            w = torch.from_numpy(Q.dequantize(self._raw, self._raw_qtype, (self.K, self.N)).copy())
        elif self.qtype == "dense":
            w = self.data.float()
        else:
            w = self.dequant_gpu(torch.float32)
        if w.device.type == "cpu":
            self._dense_f32 = w
        return w

    def dequant_gpu(self, dtype=torch.bfloat16, rows: torch.Tensor | None = None) -> torch.Tensor:
        assert self.is_quant and self.data.is_cuda
        n = self.N if rows is None else rows.numel()
        out = torch.empty((n, self.K), dtype=dtype, device=self.data.device)
        ob = out if dtype in (torch.bfloat16, torch.float16) else None
        of = out if dtype == torch.float32 else None
        if ob is not None:
            N.ensure_act(dtype)
        if self.layout == "t32":
            N.kcall("mxk_dequant_t32", int(self.qtype), self.data.data_ptr(), N.ptr(rows), n, self.K, N.ptr(ob),
                    N.ptr(of), self.K, N.stream_ptr())
            return out
        N.kcall("mxk_dequant_rows", int(self.qtype), self.data.data_ptr(), N.ptr(self.dplane),
                N.ptr(rows), n, self.K, N.ptr(ob), N.ptr(of), self.K, N.stream_ptr())
        return out

    def to_t32(self) -> bool:
        """Re-lay the GPU copy out in the t32 tiled layout (qmm / qmv kernels). In place; returns False
        (layout unchanged) when the weight does not qualify (CPU, dense, N % 32, K % 256, bf16 mode)."""
        if (self.layout == "t32" or not self.is_quant or not self.data.is_cuda or self.N % 32 or self.K % 256
                or ACT_DTYPE != torch.float16 or int(self.qtype) not in (int(q) for q in Q.T32_UNIT)):
            return self.layout == "t32"
        self.data = Q.tile32(self.data, self.dplane, int(self.qtype), self.N, self.K)
        self.dplane = None
        self.layout = "t32"
        return True

    def ensure_kernel_layout(self) -> bool:
        """A block format that only has t32 kernels (Q5_K) but stayed in the row layout (an expert stack, a
        weight that never went through to_t32) is re-laid onto the Q8_0 kernels. Returns True if changed."""
        if not self.is_quant or not self.data.is_cuda or self.layout != "ggml" or \
                int(self.qtype) not in (int(q) for q in Q.T32_ONLY):
            return False
        raw = self.data.cpu().numpy()
        q8 = Q.to_q8_0(raw, int(self.qtype), self.N, self.K)
        data, dpl = Q.repack_for_gpu(q8, QType.Q8_0, self.N, self.K)
        dev = self.data.device
        self.data = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
        self.dplane = torch.from_numpy(np.ascontiguousarray(dpl).view(np.int16)).to(dev)
        self.qtype = int(QType.Q8_0)
        log.info("%s: Q5_K weight outside the t32 layout carried on the Q8_0 kernels", self.name)
        return True

    def build_bf16_cache(self, dtype=None):
        """Optional dense 16-bit (ACT_DTYPE) copy for large-M prefill through hipBLASLt (288 GB HBM
        makes the 2 B/param copy affordable; engine config `prefill_bf16_cache`)."""
        if self.is_quant and self.data.is_cuda and self.bf16_cache is None:
            self.bf16_cache = self.dequant_gpu(dtype or ACT_DTYPE)
        return self.bf16_cache


def concat_rows(ws: list[QWeight], name: str = "") -> QWeight | None:
    """Fuse projections sharing K and qtype along N (e.g. Q|K|V). None if not fusable."""
    if not ws or any(w.qtype != ws[0].qtype or w.K != ws[0].K or w.layout != "ggml" for w in ws):
        return None
    if ws[0].device.type == "cpu":
        if any(w._raw is None for w in ws):
            return None
        raw = np.concatenate([np.asarray(w._raw).reshape(w.N, -1) for w in ws], 0)
        return QWeight(sum(w.N for w in ws), ws[0].K, ws[0].qtype, torch.empty(0), None, raw,
                       ws[0]._raw_qtype, name)
    data = torch.cat([w.data for w in ws], 0)
    dpl = torch.cat([w.dplane for w in ws], 0) if ws[0].dplane is not None else None
    return QWeight(sum(w.N for w in ws), ws[0].K, ws[0].qtype, data, dpl, None, ws[0]._raw_qtype, name)


def interleave_gate_up(gate: QWeight, up: QWeight, name: str = "") -> QWeight | None:
    """Gate/up rows interleaved in 16-row groups for the fused SwiGLU epilogue."""
    if gate.qtype != up.qtype or gate.K != up.K or gate.N != up.N or gate.N % 16 or gate.layout != "ggml":
        return None
    if gate.device.type == "cpu":
        if gate._raw is None:
            return None
        raw = Q.interleave_rows16(np.asarray(gate._raw).reshape(gate.N, -1), np.asarray(up._raw).reshape(up.N, -1))
        return QWeight(2 * gate.N, gate.K, gate.qtype, torch.empty(0), None, raw, gate._raw_qtype, name)

    def il(a, b):
        g = a.shape[0] // 16
        return torch.stack([a.reshape(g, 16, -1), b.reshape(g, 16, -1)], 1).reshape(2 * a.shape[0], -1)

    data = il(gate.data, up.data)
    dpl = il(gate.dplane, up.dplane) if gate.dplane is not None else None
    return QWeight(2 * gate.N, gate.K, gate.qtype, data, dpl, None, gate._raw_qtype, name)


# ------------------------------------------------------------------------------------------------
def _mfma_shape(M: int, N_: int, nblk: int, can_split: bool, qtype: int):
    if M <= 16:
        wm = 1
    elif M <= 32:
        wm = 2
    elif M <= 64:
        wm = 4
    else:
        wm = 8
    wn = 2
    cols = -(-N_ // (64 * wn))
    mt = -(-M // (16 * wm))
    splits = 1
    if can_split:
        target = 2 * CU_COUNT
        while cols * mt * splits < target and splits * 2 <= nblk // 2:
            splits *= 2
    return wm, wn, splits


def qmatmul(W: QWeight, x: torch.Tensor | None, epi: int, out: torch.Tensor, *, xq: torch.Tensor | None = None,
            xds: torch.Tensor | None = None, out_zeroed: bool = False, fuse: "NormFuse | None" = None):
    """out (+)= x @ W^T with the given epilogue.

    x:   bf16 [M, K] (MFMA / dense path) — may be None when (xq, xds) given and M <= 4
    epi: EPI_F32 (store fp32) | EPI_BF16 | EPI_ADD_F32 (out += ; fp32) | EPI_SWIGLU / EPI_GEGLU
         (silu- / gelu-gated, 16-bit [M, N/2])
    out_zeroed: for EPI_F32, caller guarantees `out` is zero so split-K may accumulate atomically.
    fuse: the RMSNorm split across this GEMM and its neighbour (NormFuse; only where norm_fusable() said so).
    """
    M = (x if x is not None else xq).shape[0]
    if M == 0:
        return out
    dev = (x if x is not None else xq).device
    if dev.type == "cpu":
        return _qmatmul_ref(W, x if x is not None else _deq_q8(xq, xds), epi, out)
    if not W.is_quant:
        y = torch.matmul(x, W.data.t()) if x.dtype == W.data.dtype else torch.matmul(x.to(W.data.dtype), W.data.t())
        return _apply_epi_dense(y, epi, out)
    if W.layout == "t32":
        return _qmatmul_t32(W, x, epi, out, xq, xds, M, out_zeroed, fuse)
    if fuse is not None:
        raise ValueError("qmatmul: norm fusion needs t32 weights")
    if M <= 4 and xq is not None:
        if epi in (EPI_BF16, *GLU_EPIS):
            N.ensure_act(out.dtype)
        N.kcall("mxk_qgemv", int(W.qtype), epi, xq.data_ptr(), xds.data_ptr(), W.data.data_ptr(), N.ptr(W.dplane),
                M, W.N, W.K, out.data_ptr(), out.stride(0), N.stream_ptr())
        return out
    if x is None:
        raise ValueError("qmatmul: MFMA path needs 16-bit activations")
    can_split = epi == EPI_ADD_F32 or (epi == EPI_F32 and out_zeroed)
    if W.bf16_cache is not None and M >= dense_min_m(x.dtype, epi, can_split) and W.bf16_cache.dtype == x.dtype:
        return _dense_cached(W, x, epi, out, M)
    nblk = W.K // 256
    f16 = x.dtype == torch.float16
    if f16 and M >= Q32_MIN_M:
        wm, wn, splits = _mfma32_shape(M, W.N, nblk, can_split)
        e = EPI_ADD_F32 if (epi == EPI_F32 and splits > 1) else epi
        if e in (EPI_BF16, *GLU_EPIS) and out.dtype != x.dtype:
            raise ValueError(f"qmatmul: {out.dtype} output with {x.dtype} activations")
        if e in (EPI_BF16, *GLU_EPIS):
            N.ensure_act(out.dtype)
        N.kcall("mxk_qgemm32", int(W.qtype), e, wm, wn, x.data_ptr(), x.stride(0), W.data.data_ptr(), N.ptr(W.dplane),
                M, W.N, W.K, splits, out.data_ptr(), out.stride(0), N.stream_ptr())
        return out
    wm, wn, splits = (_mfma16_shape if f16 else _mfma_shape)(M, W.N, nblk, can_split, int(W.qtype))
    e = epi
    if epi == EPI_F32 and splits > 1:
        e = EPI_ADD_F32
    if e in (EPI_BF16, *GLU_EPIS) and out.dtype != x.dtype:
        raise ValueError(f"qmatmul: {out.dtype} output with {x.dtype} activations")
    N.kcall("mxk_qgemm16" if f16 else "mxk_qgemm_mfma", int(W.qtype), e, wm, wn, x.data_ptr(), x.stride(0),
            W.data.data_ptr(), N.ptr(W.dplane), M, W.N, W.K, splits, out.data_ptr(), out.stride(0), N.stream_ptr())
    return out


def _dense_cached(W: QWeight, x, epi: int, out, M: int):
    """hipBLASLt on the dense 16-bit weight copy (only where it measured faster than qmm)."""
    wt = W.bf16_cache.t()
    if epi in (EPI_ADD_F32, EPI_F32) and out.is_contiguous() and _fp32_out_ok(x.dtype):
        # hipBLASLt 16-bit x 16-bit -> fp32 with the residual add fused as beta = 1
        if epi == EPI_ADD_F32:
            torch.addmm(out, x, wt, out_dtype=torch.float32, out=out)
        else:
            torch.mm(x, wt, out_dtype=torch.float32, out=out)
        return out
    y = torch.matmul(x, wt)
    if epi in GLU_EPIS:
        N.ensure_act(out.dtype)
        N.kcall("mxk_swiglu_il16", y.data_ptr(), y.stride(0), out.data_ptr(), out.stride(0), M, W.N // 2,
                int(epi == EPI_GEGLU), N.stream_ptr())
        return out
    return _apply_epi_dense(y, epi, out)


# Row chunking of wide K-quant GEMMs (M > ROW_CHUNK): every launch holds at most ROW_CHUNK rows. The qmm tiles hold
# 128 or 256 rows with one workgroup per CU, so M = 384 as one launch runs two row tiles per column panel — 448
# workgroups, 1.75 waves over 256 CUs, 512 rows of MFMA work (profiles/r4_engine_c128_kernels.md: gate_up 199 us at
# M = 384 against 74 us at M = 256 and 42 us at M = 128); 256 + 128 as two launches fills the chip twice instead.
ROW_CHUNK = int(os.environ.get("MX_ROW_CHUNK", "0"))


def row_chunks(M: int, chunk: int | None = None) -> list[tuple[int, int]]:
    """[(r0, r1)] row ranges of at most `chunk` rows (ROW_CHUNK; 0 = one launch)."""
    c = ROW_CHUNK if chunk is None else chunk
    if c <= 0 or M <= c:
        return [(0, M)]
    return [(r, min(r + c, M)) for r in range(0, M, c)]


def run_plan(plan: tuple, W: QWeight, x: torch.Tensor, epi: int, out: torch.Tensor, out_zeroed: bool,
             fuse: "NormFuse | None" = None):
    """Launch one GEMM plan (ops/autotune.py): ("q3", wm, splits) | ("q2", wm, ks, wn, splits) | ("rows", chunk)."""
    M = x.shape[0]
    kind = plan[0]
    if fuse is not None and kind != "q2":
        raise ValueError(f"norm fusion needs a qmm2 plan, not {plan}")
    if kind == "rows":
        for r0, r1 in row_chunks(M, plan[1]):
            _qmatmul_t32(W, x[r0:r1], epi, out[r0:r1], None, None, r1 - r0, out_zeroed)
        return out
    splits = plan[-1]
    e = EPI_ADD_F32 if (epi == EPI_F32 and splits > 1) else epi
    if e in (EPI_BF16, *GLU_EPIS):
        if out.dtype != x.dtype:
            raise ValueError(f"qmatmul: {out.dtype} output with {x.dtype} activations")
        N.ensure_act(out.dtype)
    if kind == "q3":
        N.kcall("mxk_qmm3", int(W.qtype), e, plan[1], x.data_ptr(), x.stride(0), W.data.data_ptr(), M, W.N, W.K,
                splits, out.data_ptr(), out.stride(0), N.stream_ptr())
    elif kind == "q2" and fuse is not None and fuse.mode & 4:
        f = fuse
        slots, rot, bias, qo, kc, vc, n_off, D, hq, hkv, bsz = f.rope
        N.kcall("mxk_qmm2_rope", int(W.qtype), e, plan[1], plan[2], plan[3], x.data_ptr(), x.stride(0),
                W.data.data_ptr(), M, W.N, W.K, splits, out.data_ptr(), out.stride(0), f.mode, N.ptr(f.ss_in),
                1.0 / W.K, f.eps, N.ptr(f.tick), slots.data_ptr(), rot.data_ptr(), N.ptr(bias), qo.data_ptr(),
                kc.data_ptr(), vc.data_ptr(), int(n_off), int(D).bit_length() - 1, int(hq), int(hkv), int(bsz),
                N.stream_ptr())
    elif kind == "q2" and fuse is not None:
        f = fuse
        N.kcall("mxk_qmm2_fused", int(W.qtype), e, plan[1], plan[2], plan[3], x.data_ptr(), x.stride(0),
                W.data.data_ptr(), M, W.N, W.K, splits, out.data_ptr(), out.stride(0), f.mode, N.ptr(f.ss_out),
                N.ptr(f.ss_zero), N.ptr(f.gamma), N.ptr(f.xn), f.xn.stride(0) if f.xn is not None else 0,
                N.ptr(f.tick), N.ptr(f.ss_in), 1.0 / W.K, f.eps, N.stream_ptr())
    elif kind == "q2":
        N.kcall("mxk_qmm2", int(W.qtype), e, plan[1], plan[2], plan[3], x.data_ptr(), x.stride(0), W.data.data_ptr(),
                M, W.N, W.K, splits, out.data_ptr(), out.stride(0), N.stream_ptr())
    else:
        raise ValueError(f"unknown GEMM plan {plan}")
    return out


def _t32_plan(W: QWeight, M: int, epi: int, out_zeroed: bool, dtype=torch.float16):
    """The plan _qmatmul_t32 runs for an M-row f16 GEMM on t32 weights, or None where it takes the dense copy."""
    can_split = epi == EPI_ADD_F32 or (epi == EPI_F32 and out_zeroed)
    if W.bf16_cache is not None and M >= dense_min_m(dtype, epi, can_split) and W.bf16_cache.dtype == dtype:
        return None
    forced = QMM2 or QMM3 or QMM2_FORCE is not None or QMM3_FORCE is not None
    plan = _AT.lookup(W.N, W.K, int(W.qtype), epi, can_split, M) if (_AT.TUNED and not forced) else None
    if plan is None:
        if len(row_chunks(M)) > 1:
            plan = ("rows", ROW_CHUNK)
        else:
            plan = _gemm_pick(M, W.N, W.K, int(W.qtype), can_split)
    return plan


class NormFuse:
    """The RMSNorm between two K-quant GEMMs, split across them (qmm2_impl.h Q2Fuse): the producer (the residual-add
    o_proj / down GEMM, mode 1) writes xn = f16(h * gamma) and the rows' sums of squares into ss_out as its output
    blocks become final, and re-zeroes ss_zero; the consumer (qkv / gate|up, mode 2) scales its rows by
    rsqrt(ss_in / K + eps). ss buffers: [rows, 32] fp32 (one 128-byte line per row), tick: zeroed int32 counters."""
    __slots__ = ("mode", "ss_out", "ss_zero", "gamma", "xn", "tick", "ss_in", "eps", "rope")

    def __init__(self, mode: int, *, ss_out=None, ss_zero=None, gamma=None, xn=None, tick=None, ss_in=None,
                 eps: float = 0.0, rope: tuple | None = None):
        self.mode, self.ss_out, self.ss_zero, self.gamma, self.xn = mode, ss_out, ss_zero, gamma, xn
        self.tick, self.ss_in, self.eps = tick, ss_in, float(eps)
        # mode bit 4 (the q|k|v GEMM): RoPE + paged KV append in the epilogue, rope = (slots, rot = the step's
        # [T, D / 2, 2] (cos, sin) x attn_factor table, bias or None, q_out bf16 [T, Hq * D], k_cache, v_cache, column
        # offset, D, Hq, Hkv, block_size)
        self.rope = rope


NORM_FUSE = os.environ.get("MX_NORM_FUSE", "0") != "0"
ROPE_FUSE = os.environ.get("MX_ROPE_FUSE", "0") != "0"
_NORM_FUSE_QT = None


def norm_fusable(W, M: int, epi: int, out_zeroed: bool = False, rope: bool = False) -> bool:
    """True where an M-row GEMM on W runs a qmm2 plan whose fused-RMSNorm instance exists (Q4_K / Q5_K / Q6_K / Q8_0
    t32 weights, M > 4, f16 activations; fp32 / residual-add / SwiGLU epilogues)."""
    global _NORM_FUSE_QT
    if _NORM_FUSE_QT is None:
        _NORM_FUSE_QT = {int(QType.Q4_K), int(QType.Q5_K), int(QType.Q6_K), int(QType.Q8_0)}
    if (not (ROPE_FUSE if rope else NORM_FUSE) or not isinstance(W, QWeight) or W.layout != "t32" or M <= 4 or int(W.qtype) not in _NORM_FUSE_QT
            or epi not in (EPI_F32, EPI_ADD_F32, EPI_SWIGLU) or W.data.device.type != "cuda"):
        return False
    plan = _t32_plan(W, M, epi, out_zeroed)
    return plan is not None and plan[0] == "q2"


def _qmatmul_t32(W: QWeight, x, epi: int, out, xq, xds, M: int, out_zeroed: bool, fuse: "NormFuse | None" = None):
    """t32 tiled weights: qmv (q8 activations, M <= 4) or qmm2 / qmm3 (f16 activations, any M; tuned plan)."""
    if fuse is not None:
        if x is None or x.dtype != torch.float16:
            raise ValueError("qmatmul: norm fusion needs f16 activations")
        plan = _t32_plan(W, M, epi, out_zeroed)
        if plan is None:
            raise ValueError("qmatmul: norm fusion on a dense-copy GEMM")
        return run_plan(plan, W, x, epi, out, out_zeroed, fuse)
    if M <= 4 and xq is not None:
        if epi in (EPI_BF16, *GLU_EPIS):
            N.ensure_act(out.dtype)
        ks = 1
        if epi == EPI_ADD_F32 or (epi == EPI_F32 and out_zeroed):
            # narrow outputs (o_proj / down / qkv: N/32 groups < CUs): split K over workgroups, fp32 atomics
            units = W.K // Q.T32_UNIT[QType(int(W.qtype))][1]
            while (W.N // 32) * ks < 2 * CU_COUNT and units // (ks * 2) >= 2:
                ks *= 2
        N.kcall("mxk_qmv", int(W.qtype), EPI_ADD_F32 if ks > 1 else epi, xq.data_ptr(), xds.data_ptr(),
                W.data.data_ptr(), M, W.N, W.K, ks, out.data_ptr(), out.stride(0), N.stream_ptr())
        return out
    if x is None or x.dtype != torch.float16:
        raise ValueError("qmatmul: t32 weights need f16 activations (or q8 activations with M <= 4)")
    plan = _t32_plan(W, M, epi, out_zeroed, x.dtype)
    if plan is None:
        return _dense_cached(W, x, epi, out, M)
    return run_plan(plan, W, x, epi, out, out_zeroed)


QMV_FUSE = os.environ.get("MX_QMV_FUSE", "1") != "0"


QMV1_NORM_KS1 = os.environ.get("MX_QMV1_NORM_KS1", "1") != "0"


def qmv_fusable(W, M: int, epi: int, out_zeroed: bool = False, norm: bool = False) -> int:
    """K-split count of the fused-input decode GEMV for this weight / batch, or 0 if it does not apply
    (not t32, M > 4, or the per-workgroup LDS slice of the q8 activations would exceed 64 KB)."""
    if not QMV_FUSE or not isinstance(W, QWeight) or W.layout != "t32" or not 0 < M <= 4 or W.data.device.type != "cuda":
        return 0
    ks = 1
    elem = 64 if int(W.qtype) == int(QType.Q8_0) else 256
    if norm and M == 1 and W.K in (4096, 8192) and QMV1_NORM_KS1:
        return 1  # unsplit: the batch-1 qmv1 kernel reads the row once, ahead of the weights (qmv.hip)
    if epi == EPI_ADD_F32 or (epi == EPI_F32 and out_zeroed):
        units = W.K // elem
        while (W.N // 32) * ks < 2 * CU_COUNT and units // (ks * 2) >= 2:
            ks *= 2
    mm = 1 if M == 1 else 2 if M == 2 else 4
    sl = -(-(W.K // elem) // ks) * elem
    return 0 if mm * (sl + sl // 4) > 64 * 1024 else ks


def qmv_fused(W: QWeight, x: torch.Tensor, epi: int, out: torch.Tensor, *, norm: torch.Tensor | None = None,
              eps: float = 0.0, out_zeroed: bool = False) -> bool:
    """Decode GEMV (M <= 4, t32 weights) with the q8 quantisation of `x` — and with `norm`, the RMSNorm
    x / rms(x) * norm of the fp32 residual rows `x` — fused into the GEMV prologue (qmv.hip mxk_qmv_x).
    Returns False (nothing launched) where the fused kernel does not apply; the caller then runs
    rmsnorm / quant_q8 + qmatmul."""
    M = x.shape[0]
    ks = qmv_fusable(W, M, epi, out_zeroed, norm is not None)
    if (not ks or not x.is_cuda or x.stride(-1) != 1
            or (norm is None and x.dtype not in (torch.float16, torch.bfloat16))
            or (norm is not None and x.dtype != torch.float32)):
        return False
    if epi in (EPI_BF16, *GLU_EPIS):
        if norm is None and out.dtype != x.dtype:
            return False
        N.ensure_act(out.dtype)
    elif norm is None:
        N.ensure_act(x.dtype)
    N.kcall("mxk_qmv_x", int(W.qtype), EPI_ADD_F32 if ks > 1 else epi, 2 if norm is not None else 1, x.data_ptr(),
            x.stride(0), N.ptr(norm), float(eps), W.data.data_ptr(), M, W.N, W.K, ks, out.data_ptr(), out.stride(0),
            N.stream_ptr())
    return True


QMV_ROPE_QTYPES = (int(QType.Q4_K), int(QType.Q5_K), int(QType.Q6_K), int(QType.Q3_K), int(QType.Q2_K))
QMV_ROPE_FUSE = os.environ.get("MX_QMV_ROPE", "1") != "0"


def qmv_rope_ok(W, x: torch.Tensor, q_out: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, D: int,
                n_off: int) -> bool:
    """Does mxk_qmv1_rope apply to this qkv part? Callers fusing several parts check EVERY part first, so a
    model whose parts mix block formats (q|k Q4_K, v Q8_0 / MX4F) takes the unfused path for all of them."""
    return not (not QMV_ROPE_FUSE or not isinstance(W, QWeight) or W.layout != "t32"
                or int(W.qtype) not in QMV_ROPE_QTYPES or W.K not in (4096, 8192) or x.shape[0] != 1 or not x.is_cuda
                or x.dtype != torch.float32 or not x.is_contiguous() or k_cache.dtype != torch.bfloat16
                or v_cache.dtype != torch.bfloat16 or q_out.dtype != torch.bfloat16 or D not in (64, 128) or n_off % 32)


# off by default: the ticket / fence / atomic chain cost more than the extra workgroups bought at batch 1 (8B c1
# 469 vs 529 tok/s, 70B TP8 shard unchanged; gpurun_out/k12)
QMV_ROPE_SPLIT = os.environ.get("MX_QMV_ROPE_SPLIT", "0") == "1"


def qmv_rope_split(W: QWeight) -> int:
    """K-split of the batch-1 qkv GEMV: narrow parts (1024-6144 columns = 32-192 column groups) spread over the CUs,
    keeping at least two 256-element units per workgroup; the last workgroup of a column group runs the epilogue."""
    if not QMV_ROPE_SPLIT:
        return 1
    groups, units = W.N // 32, W.K // 256
    ks = 1
    while groups * ks < CU_COUNT and units % (ks * 2) == 0 and units // (ks * 2) >= 2:
        ks *= 2
    return ks


def qmv_rope_fused(W: QWeight, x: torch.Tensor, norm: torch.Tensor, eps: float, n_off: int, positions, slots,
                   inv_freq: torch.Tensor, bias, attn_factor: float, Hq: int, Hkv: int, D: int, q_out: torch.Tensor,
                   k_cache: torch.Tensor, v_cache: torch.Tensor, block_size: int, sk=None) -> bool:
    """Batch-1 qkv part: RMSNorm -> q8 -> GEMV -> (+bias) -> RoPE (adjacent pairs, whole head) -> q_out or the
    paged K/V caches at slots[0], one launch (qmv.hip mxk_qmv1_rope). sk = (fp32 workspace >= N, int32 tickets
    >= N / 32), both zeroed: the GEMV splits K over several workgroups per column group. False: not applicable,
    nothing launched."""
    if not qmv_rope_ok(W, x, q_out, k_cache, v_cache, D, n_off):
        return False
    ks = qmv_rope_split(W) if sk is not None and sk[0].numel() >= W.N and sk[1].numel() >= W.N // 32 else 1
    N.kcall("mxk_qmv1_rope", int(W.qtype), x.data_ptr(), norm.data_ptr(), float(eps), W.data.data_ptr(), W.N, W.K,
            n_off, positions.data_ptr(), slots.data_ptr(), inv_freq.data_ptr(), N.ptr(bias), float(attn_factor), Hq,
            Hkv, D, q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_size, ks,
            sk[0].data_ptr() if ks > 1 else 0, sk[1].data_ptr() if ks > 1 else 0, N.stream_ptr())
    return True


def dense_min_m(dtype, epi: int = EPI_ADD_F32, can_split: bool = True) -> int:
    """Smallest M routed to the dense weight cache (hipBLASLt). From tools/bench_qgemm.py +
    tools/tune_qgemm16.py on MI355X (Llama-3-8B shapes): the bf16 dequant-MFMA kernel loses to the
    dense path from M=128; the packed-f16 kernel with split-K wins for the residual-accumulating /
    split-able projections up to M=256 (qkv 19.6 vs 20.5 us, o_proj 15.4 vs 19.6, down 42 vs 58.5 at
    M=128) but loses the SwiGLU gate|up (no split-K) from M~96 and the LM head from M~48."""
    if BF16_CACHE_MIN_M:
        return BF16_CACHE_MIN_M
    if dtype != torch.float16:
        return 128
    if epi in GLU_EPIS:
        return DENSE_MIN_M_SWIGLU
    if not can_split:
        return DENSE_MIN_M_NOSPLIT
    return DENSE_MIN_M_SPLIT


# From tools/tune_qmm.py on MI355X (profiles/r2_qmm_tune.jsonl): qmm on t32 weights beats the dense copy
# below these M; above, hipBLASLt on 2 B/weight still wins for the layer projections (not the LM head,
# which never gets a dense copy).
DENSE_MIN_M_SWIGLU = int(os.environ.get("MX_DENSE_MIN_M_SWIGLU", "96"))
DENSE_MIN_M_NOSPLIT = int(os.environ.get("MX_DENSE_MIN_M_NOSPLIT", "96"))
DENSE_MIN_M_SPLIT = int(os.environ.get("MX_DENSE_MIN_M_SPLIT", "192"))


Q32_MIN_M = int(os.environ.get("MX_Q32_MIN_M", "48"))
Q32_FORCE: tuple | None = None  # (wm, wn, splits) override for tuning (tools/tune_qgemm32.py)


# qmm2.hip: second-generation quantised GEMM (wave tile = all BM rows x one 32-column group, super-block
# unrolled k loop, 4-slot LDS-DMA ring) for the Q4_K_M formats. (wm, ks): BM = 32 wm rows, ks = 1 (4 waves)
# or 2 (8 waves splitting each k-tile's k-steps); 128 columns per workgroup; K split in whole super-blocks.
QMM2 = os.environ.get("MX_QMM2", "0") != "0"
QMM2_FORCE: tuple | None = None  # (wm, ks, wn, splits) override (tests, tools/prof_qmm.py)
# compiled (wm, ks, wn): wm 32-row MFMA blocks x wn 32-column groups per wave, ks 1 / 2 waves per SIMD
QMM2_CONFIGS = ((2, 1, 1), (2, 2, 1), (4, 1, 1), (4, 2, 1), (8, 1, 1), (1, 2, 2), (2, 1, 2), (2, 2, 2), (4, 1, 2),
                # 192- / 224-row tiles (M = 384 / 448 as two row tiles)
                (6, 1, 1), (6, 2, 1), (3, 2, 2), (7, 1, 1),
                # ks | 8: the 8-slot LDS ring (64-row tiles)
                (2, 9, 1), (2, 10, 1), (1, 10, 2),
                # ks 17: wide tiles, 8 column groups (256 columns) per 8-wave workgroup — half the A staging per flop
                (2, 17, 1), (4, 17, 1), (6, 17, 1), (3, 17, 2), (7, 17, 1),
                # ks | 32: 6-slot LDS-DMA ring for the 128-row tiles, offered to the tuner with MX_QMM2_R6=1: five stages
                # in flight instead of three changed nothing at M = 128-256 (gate_up M=128 42.1 vs 41.9 us,
                # profiles/r6_qmm2_ring6.md) — the DMA latency is not what bounds the decode tiles
                *(((4, 33, 1), (4, 34, 1), (2, 34, 2), (2, 33, 2)) if os.environ.get("MX_QMM2_R6", "0") == "1" else ()))
# ks 18: 4-wave wide tiles, each wave 64 columns x 32 wm rows (one wave per SIMD); compiled and tested
# (test_qmm2[*-18-*]), offered to the tuner with MX_QMM2_WIDE4=1
if os.environ.get("MX_QMM2_WIDE4", "0") == "1":
    QMM2_CONFIGS = QMM2_CONFIGS + ((2, 18, 2), (4, 18, 2), (6, 18, 2))
# every t32 block format runs on qmm2 / qmm3 (qmm2_fmt.h decoders)
QMM2_QTYPES = (int(QType.Q4_K), int(QType.Q6_K), int(QType.Q3_K), int(QType.Q2_K), int(QType.Q5_K), int(QType.Q8_0),
               int(QType.MX4F), int(QType.MX5F))
QMM2_MIN_M = int(os.environ.get("MX_QMM2_MIN_M", "16"))


def _split_for(tiles: int, K: int, can_split: bool) -> int:
    splits = 1
    if can_split:
        nsb = K // 256
        while tiles * splits < (3 * CU_COUNT) // 4 and nsb // (splits * 2) >= 2:
            splits *= 2
    return splits


def _gemm_pick(M: int, N_: int, K: int, qtype: int, can_split: bool):
    """Untuned fallback plan ("q3", wm, splits) | ("q2", wm, ks, wn, splits) for a t32 GEMM — shapes the load-time
    autotuner (ops/autotune.py) did not time. The rule follows the tuned Llama-3-8B table
    (profiles/r5_gemm_autotune.md): 64-row 8-wave qmm2 tiles for the narrow projections, 128-row tiles for the
    wide ones, qmm3 for the gated FFN at 129-256 rows."""
    if QMM3 and M >= QMM3_MIN_M:  # explicit overrides (tests, tuning)
        return ("q3", *_qmm3_shape(M, N_, K, can_split))
    if QMM2 and M >= QMM2_MIN_M:
        return ("q2", *_qmm2_shape(M, N_, K, can_split))
    nct = -(-N_ // 128)
    wide = N_ >= 16384
    if M <= 64 or (not wide and K < 8192 and M <= 256):
        return ("q2", 2, 2, 1, _split_for(-(-M // 64) * nct, K, can_split))
    if wide and 128 < M <= 256:
        return ("q3", 4, 1)
    if not wide and M > 256 and K < 8192:
        return ("q2", 4, 2, 1, 1)
    return ("q2", 4, 2, 1, _split_for(-(-M // 128) * nct, K, can_split))


# qmm3.hip: warp-specialised (4 DMA / dequant waves + 4 MFMA waves per workgroup), BM = 64 wm rows
QMM3 = os.environ.get("MX_QMM3", "0") != "0"
QMM3_FORCE: tuple | None = None  # (wm, splits) override for tuning
QMM3_MIN_M = int(os.environ.get("MX_QMM3_MIN_M", "64"))


def _qmm3_shape(M: int, N_: int, K: int, can_split: bool):
    """(wm, splits) for qmm3: the smallest row tile (64 / 128 / 256 rows) covering M, then K splits as qmm2."""
    if QMM3_FORCE is not None:
        wm, splits = QMM3_FORCE
        return wm, (splits if can_split else 1)
    wm = 1 if M <= 64 else 2 if M <= 128 else 4
    tiles = -(-M // (64 * wm)) * -(-N_ // 128)
    splits = 1
    if can_split:
        nsb = K // 256
        while tiles * splits < (3 * CU_COUNT) // 4 and nsb // (splits * 2) >= 2:
            splits *= 2
    return wm, splits


def _qmm2_shape(M: int, N_: int, K: int, can_split: bool):
    """(wm, ks, wn, splits) for qmm2: the smallest row tile covering M (up to 256 rows per workgroup), then K
    splits (split-able outputs only) until ~3/4 of the CUs hold a workgroup, >= 2 super-blocks per split."""
    if QMM2_FORCE is not None:
        wm, ks, wn, splits = QMM2_FORCE
        return wm, ks, wn, (splits if can_split else 1)
    if M <= 64:
        wm, ks, wn = 1, 2, 2
    elif M <= 128:
        wm, ks, wn = 2, 2, 2
    else:
        wm, ks, wn = 4, 1, 2
    tiles = -(-M // (32 * wm * wn)) * -(-N_ // 128)
    splits = 1
    if can_split:
        nsb = K // 256
        while tiles * splits < (3 * CU_COUNT) // 4 and nsb // (splits * 2) >= 2:
            splits *= 2
    return wm, ks, wn, splits


def _mfma32_shape(M: int, N_: int, nblk: int, can_split: bool):
    """qgemm32 tile / split-K choice: 32*wm-row tiles, 128 columns per workgroup, K splits (fp32
    atomics) only for split-able outputs until the grid covers the CUs."""
    if Q32_FORCE is not None:
        wm, wn, splits = Q32_FORCE
        return wm, wn, (splits if can_split else 1)
    wm = 1 if M <= 32 else 2 if M <= 64 else 4
    wn = 1
    cols = -(-N_ // (128 * wn))
    mt = -(-M // (32 * wm))
    splits = 1
    if can_split:
        while cols * mt * splits < CU_COUNT and splits * 2 <= max(1, nblk // 4):
            splits *= 2
    return wm, wn, splits


def _mfma16_shape(M: int, N_: int, nblk: int, can_split: bool, qtype: int):
    """qgemm16 tile / split-K choice (tools/tune_qgemm16.py): 64-row tiles (WM=4, 2 waves/SIMD);
    split-able outputs take WN=1 (64 columns per workgroup) and 2-8 K splits — fp32 atomics are
    cheap at few splits but their count scales with M x N x splits."""
    wm = 1 if M <= 16 else 2 if M <= 32 else 4
    if not can_split:
        return wm, 2, 1
    wn = 1 if wm == 4 else 2
    if M <= 64:
        splits = 8 if nblk >= 32 else 4
    elif M <= 128:
        splits = 4 if nblk >= 32 else 2
    else:
        splits = 2
    splits = max(1, min(splits, nblk // 2))
    return wm, wn, splits


_FP32_OUT: dict = {}


def _fp32_out_ok(dtype=torch.bfloat16) -> bool:
    """Does this torch build expose mm/addmm with out_dtype=float32 for 16-bit inputs (ROCm)?"""
    if dtype not in _FP32_OUT:
        try:
            a = torch.ones(16, 32, dtype=dtype, device="cuda")
            b = torch.ones(32, 16, dtype=dtype, device="cuda")
            o = torch.ones(16, 16, dtype=torch.float32, device="cuda")
            torch.addmm(o, a, b, out_dtype=torch.float32, out=o)
            o2 = torch.empty(16, 16, dtype=torch.float32, device="cuda")
            torch.mm(a, b, out_dtype=torch.float32, out=o2)
            _FP32_OUT[dtype] = bool(torch.allclose(o, torch.full_like(o, 33.0))) and \
                bool(torch.allclose(o2, torch.full_like(o2, 32.0)))
        except Exception:
            _FP32_OUT[dtype] = False
    return _FP32_OUT[dtype]


def _apply_epi_dense(y: torch.Tensor, epi: int, out: torch.Tensor):
    if epi == EPI_F32:
        out.copy_(y)
    elif epi == EPI_BF16:
        out.copy_(y)
    elif epi == EPI_ADD_F32:
        out.add_(y.float())
    else:
        yf = y.float()
        Nn = yf.shape[1]
        g = Nn // 32
        v = yf.reshape(-1, g, 2, 16)
        gate, up = v[:, :, 0, :].reshape(-1, Nn // 2), v[:, :, 1, :].reshape(-1, Nn // 2)
        act = torch.nn.functional.silu(gate) if epi == EPI_SWIGLU else \
            torch.nn.functional.gelu(gate, approximate="tanh")
        out.copy_(act * up)
    return out


def glu_interleaved(y: torch.Tensor, epi: int, out: torch.Tensor) -> torch.Tensor:
    """Gated activation of pre-activation rows in the fused gate|up layout (16-row groups: interleave_gate_up):
    y [M, 2F] -> out [M, F] = act(gate) * up (the qmm GLU epilogue as its own step)."""
    if y.is_cuda:
        N.ensure_act(out.dtype)
        N.kcall("mxk_swiglu_il16", y.data_ptr(), y.stride(0), out.data_ptr(), out.stride(0), y.shape[0],
                y.shape[1] // 2, int(epi == EPI_GEGLU), N.stream_ptr())
        return out
    return _apply_epi_dense(y.float(), epi, out)


def _qmatmul_ref(W: QWeight, x: torch.Tensor, epi: int, out: torch.Tensor):
    y = x.float() @ W.dense_f32().t()
    return _apply_epi_dense(y, epi, out)


def _deq_q8(xq: torch.Tensor, xds: torch.Tensor) -> torch.Tensor:
    M, K = xq.shape
    d = xds.reshape(M, K // 32, 2)[:, :, 0]
    return (xq.float().reshape(M, K // 32, 32) * d[:, :, None]).reshape(M, K)
