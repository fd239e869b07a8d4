"""GGML block formats: reference (de)quantisers and the MI355X repacking used by the HIP kernels.

* ``dequantize(raw, qtype, shape)`` — exact numpy reference for every block type llama.cpp models
  ship with (Q4_0/Q4_1/Q5_0/Q5_1/Q8_0/Q2_K/Q3_K/Q4_K/Q5_K/Q6_K, F16/BF16/F32). It is the CPU oracle
  the kernel tests compare against and the fallback used to densify types the GPU GEMMs do not
  consume natively.
* ``quantize_q4_k / quantize_q6_k / quantize_q8_0`` — simple (min/max, not llama.cpp's iterative
  search) quantisers, only used to build synthetic GGUF checkpoints for tests and ``bench.py``.
* ``repack_for_gpu`` — converts on-disk blocks to the layouts csrc/kernels/qgemm.hip reads:
    Q4_K: unchanged 144-byte blocks (already 16 B aligned; lane group g reads bytes 32g..32g+31);
    Q6_K: 208-byte aligned blocks [ql 128 | qh 64 | scales 16] + separate fp16 d plane, with the
          quarter-block g owning contiguous ql/qh/scale bytes (lossless permutation);
    Q8_0: int8 plane [N, K] + fp16 d plane [N, K/32].
"""
from __future__ import annotations

import numpy as np

from ..formats.gguf import BLOCK, QType

# --------------------------------------------------------------------------------------------
# helpers


def _f16(b: np.ndarray) -> np.ndarray:
    """[nb, 2] uint8 -> [nb] float32"""
    return np.ascontiguousarray(b).view(np.float16).astype(np.float32).reshape(-1)


def _blocks(raw: np.ndarray, qtype: QType) -> np.ndarray:
    be, bb = BLOCK[qtype]
    raw = np.ascontiguousarray(raw).reshape(-1)
    return raw.reshape(-1, bb)


def q4k_scale_min(scales: np.ndarray):
    """scales: [nb, 12] uint8 -> (sc [nb, 8], m [nb, 8]) as float32."""
    s = scales.astype(np.int32)
    sc = np.empty((s.shape[0], 8), np.int32)
    mn = np.empty((s.shape[0], 8), np.int32)
    sc[:, :4] = s[:, 0:4] & 63
    mn[:, :4] = s[:, 4:8] & 63
    sc[:, 4:] = (s[:, 8:12] & 0xF) | ((s[:, 0:4] >> 6) << 4)
    mn[:, 4:] = (s[:, 8:12] >> 4) | ((s[:, 4:8] >> 6) << 4)
    return sc.astype(np.float32), mn.astype(np.float32)


def _pack_q4k_scales(sc: np.ndarray, mn: np.ndarray) -> np.ndarray:
    sc = sc.astype(np.uint8)
    mn = mn.astype(np.uint8)
    out = np.zeros((sc.shape[0], 12), np.uint8)
    out[:, 0:4] = sc[:, 0:4] | ((sc[:, 4:8] >> 4) << 6)
    out[:, 4:8] = mn[:, 0:4] | ((mn[:, 4:8] >> 4) << 6)
    out[:, 8:12] = (sc[:, 4:8] & 0xF) | ((mn[:, 4:8] & 0xF) << 4)
    return out


# --------------------------------------------------------------------------------------------
# dequantisers (return float32 [n_elements])


def dq_q4_0(raw):
    b = _blocks(raw, QType.Q4_0)
    d = _f16(b[:, 0:2].copy())
    qs = b[:, 2:18]
    lo = (qs & 0xF).astype(np.int8) - 8
    hi = (qs >> 4).astype(np.int8) - 8
    return (np.concatenate([lo, hi], 1).astype(np.float32) * d[:, None]).reshape(-1)


def dq_q4_1(raw):
    b = _blocks(raw, QType.Q4_1)
    d = _f16(b[:, 0:2].copy())
    m = _f16(b[:, 2:4].copy())
    qs = b[:, 4:20]
    q = np.concatenate([qs & 0xF, qs >> 4], 1).astype(np.float32)
    return (q * d[:, None] + m[:, None]).reshape(-1)


def _q5_high(qh_bytes):
    qh = qh_bytes.copy().view(np.uint32).reshape(-1, 1)
    bits = (qh >> np.arange(32, dtype=np.uint32)) & 1
    return bits.astype(np.uint8)  # [nb, 32]


def dq_q5_0(raw):
    b = _blocks(raw, QType.Q5_0)
    d = _f16(b[:, 0:2].copy())
    hb = _q5_high(b[:, 2:6])
    qs = b[:, 6:22]
    lo = (qs & 0xF) | (hb[:, :16] << 4)
    hi = (qs >> 4) | (hb[:, 16:] << 4)
    q = np.concatenate([lo, hi], 1).astype(np.float32) - 16
    return (q * d[:, None]).reshape(-1)


def dq_q5_1(raw):
    b = _blocks(raw, QType.Q5_1)
    d = _f16(b[:, 0:2].copy())
    m = _f16(b[:, 2:4].copy())
    hb = _q5_high(b[:, 4:8])
    qs = b[:, 8:24]
    lo = (qs & 0xF) | (hb[:, :16] << 4)
    hi = (qs >> 4) | (hb[:, 16:] << 4)
    q = np.concatenate([lo, hi], 1).astype(np.float32)
    return (q * d[:, None] + m[:, None]).reshape(-1)


def dq_q8_0(raw):
    b = _blocks(raw, QType.Q8_0)
    d = _f16(b[:, 0:2].copy())
    q = b[:, 2:34].view(np.int8).astype(np.float32)
    return (q * d[:, None]).reshape(-1)


def dq_q2_k(raw):
    b = _blocks(raw, QType.Q2_K)
    scales = b[:, 0:16]
    qs = b[:, 16:80]
    d = _f16(b[:, 80:82].copy())
    dmin = _f16(b[:, 82:84].copy())
    out = np.empty((b.shape[0], 256), np.float32)
    for n in range(2):
        q = qs[:, 32 * n:32 * n + 32]
        for j in range(4):
            vals = (q >> (2 * j)) & 3
            for half in range(2):
                isx = 8 * n + 2 * j + half
                sc = scales[:, isx]
                dl = d * (sc & 0xF)
                ml = dmin * (sc >> 4)
                e0 = 128 * n + 32 * j + 16 * half
                out[:, e0:e0 + 16] = dl[:, None] * vals[:, 16 * half:16 * half + 16] - ml[:, None]
    return out.reshape(-1)


def dq_q3_k(raw):
    b = _blocks(raw, QType.Q3_K)
    hmask = b[:, 0:32]
    qs = b[:, 32:96]
    sc_raw = b[:, 96:108].astype(np.uint32)
    d = _f16(b[:, 108:110].copy())
    # unpack 16 6-bit scales (llama.cpp kmask1/kmask2 trick)
    aux = sc_raw.reshape(-1, 3, 4)
    w = aux[:, :, 0] | (aux[:, :, 1] << 8) | (aux[:, :, 2] << 16) | (aux[:, :, 3] << 24)
    a0, a1, a2 = w[:, 0], w[:, 1], w[:, 2]
    km1, km2 = np.uint32(0x03030303), np.uint32(0x0f0f0f0f)
    t = a2
    r = [(a0 & km2) | (((t >> 0) & km1) << 4), (a1 & km2) | (((t >> 2) & km1) << 4),
         ((a0 >> 4) & km2) | (((t >> 4) & km1) << 4), ((a1 >> 4) & km2) | (((t >> 6) & km1) << 4)]
    sc = np.stack(r, 1).astype(np.uint32).view(np.uint8).reshape(-1, 16).view(np.int8).astype(np.float32) - 32
    out = np.empty((b.shape[0], 256), np.float32)
    m = 1
    isx = 0
    for n in range(2):
        q = qs[:, 32 * n:32 * n + 32]
        for j in range(4):
            for half in range(2):
                l0 = 16 * half
                vals = ((q[:, l0:l0 + 16] >> (2 * j)) & 3).astype(np.int32)
                hm = (hmask[:, l0:l0 + 16] & m) != 0
                vals = vals - np.where(hm, 0, 4)
                e0 = 128 * n + 32 * j + l0
                out[:, e0:e0 + 16] = (d * sc[:, isx])[:, None] * vals
                isx += 1
            m <<= 1
    return out.reshape(-1)


def dq_q4_k(raw):
    b = _blocks(raw, QType.Q4_K)
    d = _f16(b[:, 0:2].copy())
    dmin = _f16(b[:, 2:4].copy())
    sc, mn = q4k_scale_min(b[:, 4:16])
    qs = b[:, 16:144]
    out = np.empty((b.shape[0], 256), np.float32)
    for c in range(4):
        q = qs[:, 32 * c:32 * c + 32]
        out[:, 64 * c:64 * c + 32] = (d * sc[:, 2 * c])[:, None] * (q & 0xF) - (dmin * mn[:, 2 * c])[:, None]
        out[:, 64 * c + 32:64 * c + 64] = (d * sc[:, 2 * c + 1])[:, None] * (q >> 4) - (dmin * mn[:, 2 * c + 1])[:, None]
    return out.reshape(-1)


def dq_q5_k(raw):
    b = _blocks(raw, QType.Q5_K)
    d = _f16(b[:, 0:2].copy())
    dmin = _f16(b[:, 2:4].copy())
    sc, mn = q4k_scale_min(b[:, 4:16])
    qh = b[:, 16:48]
    qs = b[:, 48:176]
    out = np.empty((b.shape[0], 256), np.float32)
    for c in range(4):
        q = qs[:, 32 * c:32 * c + 32]
        h0 = ((qh >> (2 * c)) & 1) << 4
        h1 = ((qh >> (2 * c + 1)) & 1) << 4
        out[:, 64 * c:64 * c + 32] = (d * sc[:, 2 * c])[:, None] * ((q & 0xF) | h0) - (dmin * mn[:, 2 * c])[:, None]
        out[:, 64 * c + 32:64 * c + 64] = (d * sc[:, 2 * c + 1])[:, None] * ((q >> 4) | h1) - (dmin * mn[:, 2 * c + 1])[:, None]
    return out.reshape(-1)


def q6k_codes(raw) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """ggml Q6_K blocks -> (q [nb, 256] in 0..63, scales [nb, 16] int8, d [nb] f32)."""
    b = _blocks(raw, QType.Q6_K)
    ql = b[:, 0:128].astype(np.int32)
    qh = b[:, 128:192].astype(np.int32)
    sc = b[:, 192:208].view(np.int8)
    d = _f16(b[:, 208:210].copy())
    q = np.empty((b.shape[0], 256), np.int32)
    for n in range(2):
        l = ql[:, 64 * n:64 * n + 64]
        h = qh[:, 32 * n:32 * n + 32]
        base = 128 * n
        q[:, base + 0:base + 32] = (l[:, 0:32] & 0xF) | (((h >> 0) & 3) << 4)
        q[:, base + 32:base + 64] = (l[:, 32:64] & 0xF) | (((h >> 2) & 3) << 4)
        q[:, base + 64:base + 96] = (l[:, 0:32] >> 4) | (((h >> 4) & 3) << 4)
        q[:, base + 96:base + 128] = (l[:, 32:64] >> 4) | (((h >> 6) & 3) << 4)
    return q, sc, d


def dq_q6_k(raw):
    q, sc, d = q6k_codes(raw)
    s = np.repeat(sc.astype(np.float32), 16, axis=1) * d[:, None]
    return ((q - 32).astype(np.float32) * s).reshape(-1)


# IQ4_NL / IQ4_XS: 4-bit indices into a fixed non-linear int8 codebook (ggml kvalues_iq4nl)
IQ4_KVALUES = np.array([-127, -104, -83, -65, -49, -35, -22, -10, 1, 13, 25, 38, 53, 69, 89, 113], np.int8)


def _iq4_codes(qs):
    """[nb, 16] packed nibbles -> [nb, 32] codebook values (low nibbles first, as ggml)."""
    return IQ4_KVALUES[np.concatenate([qs & 0xF, qs >> 4], 1)]


def dq_iq4_nl(raw):
    b = _blocks(raw, QType.IQ4_NL)
    d = _f16(b[:, 0:2].copy())
    return (_iq4_codes(b[:, 2:18]).astype(np.float32) * d[:, None]).reshape(-1)


def iq4_xs_scales(b):
    """[nb, 136] IQ4_XS blocks -> per-32 scales d * (ls - 32), float32 [nb, 8]."""
    d = _f16(b[:, 0:2].copy())
    sh = b[:, 2:4].copy().view(np.uint16).reshape(-1).astype(np.int32)
    sl = b[:, 4:8].astype(np.int32)
    ib = np.arange(8)
    ls = ((sl[:, ib // 2] >> (4 * (ib % 2))) & 0xF) | (((sh[:, None] >> (2 * ib)) & 3) << 4)
    return d[:, None] * (ls - 32).astype(np.float32)


def dq_iq4_xs(raw):
    b = _blocks(raw, QType.IQ4_XS)
    dl = iq4_xs_scales(b)
    codes = _iq4_codes(b[:, 8:136].reshape(-1, 16)).reshape(-1, 8, 32).astype(np.float32)
    return (codes * dl[:, :, None]).reshape(-1)


_DQ = {
    QType.IQ4_NL: dq_iq4_nl, QType.IQ4_XS: dq_iq4_xs,
    QType.Q4_0: dq_q4_0, QType.Q4_1: dq_q4_1, QType.Q5_0: dq_q5_0, QType.Q5_1: dq_q5_1,
    QType.Q8_0: dq_q8_0, QType.Q2_K: dq_q2_k, QType.Q3_K: dq_q3_k, QType.Q4_K: dq_q4_k,
    QType.Q5_K: dq_q5_k, QType.Q6_K: dq_q6_k,
}


# ---- MX4F / MX5F: the t32 kernels' layout for the 32-weight "scale (+ offset)" formats ----------------
# Row format per 256 weights (8 sub-blocks of 32), w = s_i * code + m_i exactly (Q4_0: m = -8 d; Q5_0: m = -16 d):
#   [0:16)  f16 s0..s3, m0..m3   [16:32) f16 s4..s7, m4..m7          (header halves: k-tiles 0-1 / 2-3)
#   MX4F: [32:160) codes in Q4_K order (byte 32 jq + b: low nibble = weight 64 jq + b, high = 64 jq + 32 + b)
#   MX5F: per 64-weight k-tile jq: [32 B low-nibble codes as above | 8 B high bits, bit u of the k-tile's
#         64-bit little-endian word = bit 4 of weight 64 jq + u]
Q32_FAMILY = (QType.Q4_0, QType.Q4_1, QType.Q5_0, QType.Q5_1)


def q32_parts(raw: np.ndarray, qtype: int):
    """ggml Q4_0/Q4_1/Q5_0/Q5_1 blocks -> (codes uint8 [nb, 32], s f16 [nb], m f16 [nb]), w = s * code + m."""
    q = QType(qtype)
    b = _blocks(raw, q)
    s = b[:, 0:2].copy().view(np.float16).reshape(-1)
    if q in (QType.Q4_1, QType.Q5_1):
        m = b[:, 2:4].copy().view(np.float16).reshape(-1)
        o = 4
    else:
        m = (s.astype(np.float32) * (-8.0 if q == QType.Q4_0 else -16.0)).astype(np.float16)  # exact (x 2^k)
        o = 2
    if q in (QType.Q4_0, QType.Q4_1):
        qs = b[:, o:o + 16]
        codes = np.concatenate([qs & 0xF, qs >> 4], 1)
    else:
        hb = _q5_high(b[:, o:o + 4])
        qs = b[:, o + 4:o + 20]
        codes = np.concatenate([(qs & 0xF) | (hb[:, :16] << 4), (qs >> 4) | (hb[:, 16:] << 4)], 1)
    return codes.astype(np.uint8), s, m


def to_mxf(raw: np.ndarray, qtype: int, n_rows: int, row_len: int) -> tuple[np.ndarray, QType]:
    """Q4_0/Q4_1 -> MX4F rows, Q5_0/Q5_1 -> MX5F rows (uint8 [n_rows, row_len / 256 * 160|192]); exact."""
    q = QType(qtype)
    codes, s, m = q32_parts(raw, q)
    nu = row_len // 256
    five = q in (QType.Q5_0, QType.Q5_1)
    c = codes.reshape(n_rows, nu, 8, 32)
    s8 = s.reshape(n_rows, nu, 2, 4)
    m8 = m.reshape(n_rows, nu, 2, 4)
    hdr = np.concatenate([s8, m8], 3).view(np.uint8).reshape(n_rows, nu, 32)
    lo = (c[:, :, 0::2] & 0xF) | ((c[:, :, 1::2] & 0xF) << 4)  # [n, nu, 4 k-tiles, 32 bytes]
    if not five:
        body = lo.reshape(n_rows, nu, 128)
    else:
        hb = ((c >> 4) & 1).reshape(n_rows, nu, 4, 64)
        qh8 = np.packbits(hb, axis=3, bitorder="little")  # [n, nu, 4, 8]
        body = np.concatenate([lo, qh8], 3).reshape(n_rows, nu, 160)
    out = np.concatenate([hdr, body], 2).astype(np.uint8)
    return out.reshape(n_rows, -1), (QType.MX5F if five else QType.MX4F)


def _dq_mxf(raw, five: bool):
    B = 192 if five else 160
    u = raw.reshape(-1, B)
    hdr = u[:, :32].copy().view(np.float16).astype(np.float32).reshape(-1, 2, 2, 4)  # [nu, half, s|m, 4]
    s = hdr[:, :, 0].reshape(-1, 8)
    m = hdr[:, :, 1].reshape(-1, 8)
    if five:
        body = u[:, 32:].reshape(-1, 4, 40)
        lo, qh8 = body[:, :, :32], body[:, :, 32:]
        hb = np.unpackbits(qh8, axis=2, bitorder="little").reshape(-1, 4, 2, 32)
    else:
        lo = u[:, 32:].reshape(-1, 4, 32)
        hb = np.zeros((u.shape[0], 4, 2, 32), np.uint8)
    codes = np.stack([lo & 0xF, lo >> 4], 2) | (hb << 4)  # [nu, 4, 2, 32] = sub-block 2 jq + i
    w = codes.reshape(-1, 8, 32).astype(np.float32) * s[:, :, None] + m[:, :, None]
    return w.reshape(-1)


_DQ[QType.MX4F] = lambda r: _dq_mxf(r, False)
_DQ[QType.MX5F] = lambda r: _dq_mxf(r, True)


def dequantize(raw: np.ndarray, qtype: int, shape) -> np.ndarray:
    """raw bytes (any shape) of a ggml tensor with ggml `shape` -> float32 numpy array of
    shape reversed(shape)."""
    q = QType(qtype)
    np_shape = tuple(reversed(tuple(shape)))
    raw = np.asarray(raw)
    if q == QType.F32:
        return raw.reshape(-1).view(np.float32).reshape(np_shape).astype(np.float32)
    if q == QType.F16:
        return raw.reshape(-1).view(np.float16).astype(np.float32).reshape(np_shape)
    if q == QType.BF16:
        u = raw.reshape(-1).view(np.uint16).astype(np.uint32) << 16
        return u.view(np.float32).reshape(np_shape)
    if q not in _DQ:
        raise NotImplementedError(f"dequantize {q.name}" + (": the IQ1/IQ2/IQ3 codebook grids are not built into this "
                                                           "framework; re-quantise the model to a K-quant or IQ4"
                                                           if q.name.startswith(("IQ", "TQ")) else ""))
    return _DQ[q](raw.reshape(-1).view(np.uint8)).reshape(np_shape)


# --------------------------------------------------------------------------------------------
# quantisers (synthetic checkpoints / tests)


def quantize_q8_0(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 32)
    amax = np.abs(x).max(1)
    d = amax / 127.0
    idd = np.where(d > 0, 1.0 / np.maximum(d, 1e-30), 0.0)
    q = np.clip(np.rint(x * idd[:, None]), -127, 127).astype(np.int8)
    out = np.empty((x.shape[0], 34), np.uint8)
    out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q.view(np.uint8)
    return out.reshape(-1)


def quantize_q4_0(x: np.ndarray) -> np.ndarray:
    """ggml quantize_row_q4_0: d = (signed max) / -8, codes x/d + 8.5 truncated into [0, 15]."""
    x = np.asarray(x, np.float32).reshape(-1, 32)
    idx = np.abs(x).argmax(1)
    mx = x[np.arange(x.shape[0]), idx]
    d = mx / -8.0
    idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1.0), 0.0).astype(np.float32)
    q = np.minimum(15, (x * idd[:, None] + 8.5).astype(np.int8)).astype(np.uint8)
    out = np.empty((x.shape[0], 18), np.uint8)
    out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q[:, :16] | (q[:, 16:] << 4)
    return out.reshape(-1)


def quantize_q4_k(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 8, 32)
    lo = np.minimum(x.min(2), 0.0)
    hi = x.max(2)
    scale = (hi - lo) / 15.0
    mins = -lo
    d = scale.max(1) / 63.0
    dmin = mins.max(1) / 63.0
    d16 = d.astype(np.float16).astype(np.float32)
    dm16 = dmin.astype(np.float16).astype(np.float32)
    sc = np.clip(np.rint(np.where(d16[:, None] > 0, scale / np.maximum(d16[:, None], 1e-30), 0)), 0, 63)
    mn = np.clip(np.rint(np.where(dm16[:, None] > 0, mins / np.maximum(dm16[:, None], 1e-30), 0)), 0, 63)
    eff_s = d16[:, None] * sc
    eff_m = dm16[:, None] * mn
    q = np.where(eff_s[:, :, None] > 0, np.rint((x + eff_m[:, :, None]) / np.maximum(eff_s[:, :, None], 1e-30)), 0)
    q = np.clip(q, 0, 15).astype(np.uint8).reshape(-1, 256)
    nb = q.shape[0]
    out = np.empty((nb, 144), np.uint8)
    out[:, 0:2] = d16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dm16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = _pack_q4k_scales(sc.astype(np.int32), mn.astype(np.int32))
    for c in range(4):
        out[:, 16 + 32 * c:16 + 32 * c + 32] = q[:, 64 * c:64 * c + 32] | (q[:, 64 * c + 32:64 * c + 64] << 4)
    return out.reshape(-1)


def quantize_q6_k(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 16, 16)
    amax = np.abs(x).max(2)
    scale = amax / 31.0
    d = np.abs(scale).max(1) / 127.0
    d16 = d.astype(np.float16).astype(np.float32)
    sc = np.clip(np.rint(np.where(d16[:, None] > 0, scale / np.maximum(d16[:, None], 1e-30), 0)), -128, 127)
    eff = d16[:, None] * sc
    q = np.where(eff[:, :, None] > 0, np.rint(x / np.maximum(eff[:, :, None], 1e-30)), 0)
    q = (np.clip(q, -32, 31) + 32).astype(np.int32).reshape(-1, 256)
    nb = q.shape[0]
    out = np.zeros((nb, 210), np.uint8)
    for n in range(2):
        b0 = 128 * n
        q1, q2, q3, q4 = (q[:, b0 + 32 * j:b0 + 32 * j + 32] for j in range(4))
        out[:, 64 * n:64 * n + 32] = ((q1 & 0xF) | ((q3 & 0xF) << 4)).astype(np.uint8)
        out[:, 64 * n + 32:64 * n + 64] = ((q2 & 0xF) | ((q4 & 0xF) << 4)).astype(np.uint8)
        out[:, 128 + 32 * n:128 + 32 * n + 32] = ((q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)).astype(np.uint8)
    out[:, 192:208] = sc.astype(np.int8).view(np.uint8)
    out[:, 208:210] = d16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    return out.reshape(-1)


def quantize_q5_k(x: np.ndarray) -> np.ndarray:
    """Q5_K: the Q4_K scheme with 5-bit codes (0..31) whose high bits go to qh (ggml block layout)."""
    x = np.asarray(x, np.float32).reshape(-1, 8, 32)
    lo = np.minimum(x.min(2), 0.0)
    hi = x.max(2)
    scale = (hi - lo) / 31.0
    mins = -lo
    d16 = (scale.max(1) / 63.0).astype(np.float16).astype(np.float32)
    dm16 = (mins.max(1) / 63.0).astype(np.float16).astype(np.float32)
    sc = np.clip(np.rint(np.where(d16[:, None] > 0, scale / np.maximum(d16[:, None], 1e-30), 0)), 0, 63)
    mn = np.clip(np.rint(np.where(dm16[:, None] > 0, mins / np.maximum(dm16[:, None], 1e-30), 0)), 0, 63)
    eff_s = d16[:, None] * sc
    eff_m = dm16[:, None] * mn
    q = np.where(eff_s[:, :, None] > 0, np.rint((x + eff_m[:, :, None]) / np.maximum(eff_s[:, :, None], 1e-30)), 0)
    q = np.clip(q, 0, 31).astype(np.uint8).reshape(-1, 256)
    nb = q.shape[0]
    out = np.zeros((nb, 176), np.uint8)
    out[:, 0:2] = d16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dm16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = _pack_q4k_scales(sc.astype(np.int32), mn.astype(np.int32))
    qh = np.zeros((nb, 32), np.uint8)
    for c in range(4):
        a, b_ = q[:, 64 * c:64 * c + 32], q[:, 64 * c + 32:64 * c + 64]
        out[:, 48 + 32 * c:48 + 32 * c + 32] = (a & 0xF) | ((b_ & 0xF) << 4)
        qh |= ((a >> 4) << (2 * c)).astype(np.uint8) | ((b_ >> 4) << (2 * c + 1)).astype(np.uint8)
    out[:, 16:48] = qh
    return out.reshape(-1)


QUANTIZERS = {QType.Q4_0: quantize_q4_0, QType.Q4_K: quantize_q4_k, QType.Q6_K: quantize_q6_k, QType.Q8_0: quantize_q8_0, QType.Q5_K: quantize_q5_k}


def _pack_q3k_scales(sc: np.ndarray) -> np.ndarray:
    """16 6-bit Q3_K scale codes per block -> the 12 packed bytes (inverse of dq_q3_k's kmask unpack)."""
    sc = sc.astype(np.uint32)
    lo = sc & 0xF
    hi = (sc >> 4) & 0x3
    out = np.zeros((sc.shape[0], 12), np.uint8)
    # bytes 0..7: low nibbles (scales 0..7 in the low nibble, 8..15 in the high nibble of the same byte)
    out[:, 0:8] = (lo[:, 0:8] | (lo[:, 8:16] << 4)).astype(np.uint8)
    # bytes 8..11: 2-bit high parts; byte 8 + i holds scales i, 4 + i, 8 + i, 12 + i at bits 0, 2, 4, 6
    for i in range(4):
        out[:, 8 + i] = (hi[:, i] | (hi[:, 4 + i] << 2) | (hi[:, 8 + i] << 4) | (hi[:, 12 + i] << 6)).astype(np.uint8)
    return out


def random_quantized(rng: np.random.Generator, qtype: int, n_rows: int, row_len: int, std: float = 0.02) -> np.ndarray:
    """Random-init blocks directly in the quantised domain (valid scales, uniform codes) with
    element std ~= `std`. Used for multi-GB synthetic checkpoints (quantising 8B fp32 weights
    would take minutes); same byte layout and bit width as a real checkpoint."""
    q = QType(qtype)
    nel = n_rows * row_len
    be, bb = BLOCK[q]
    nb = nel // be
    if q == QType.Q4_K:
        out = rng.integers(0, 256, size=(nb, 144), dtype=np.uint8)
        sc = rng.integers(40, 64, size=(nb, 8))
        mn = sc.copy()
        # value = d*sc*q - dmin*m with q uniform 0..15 (std 4.61): pick dmin = 7.5 d to centre
        d = np.full(nb, std / (52 * 4.61), np.float32)
        out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 2:4] = (d * 7.5).astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 4:16] = _pack_q4k_scales(sc, mn)
        return out.reshape(-1)
    if q == QType.Q5_K:
        out = rng.integers(0, 256, size=(nb, 176), dtype=np.uint8)
        sc = rng.integers(40, 64, size=(nb, 8))
        mn = sc.copy()
        d = np.full(nb, std / (52 * 9.23), np.float32)  # q uniform 0..31: std 9.23, centre dmin = 15.5 d
        out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 2:4] = (d * 15.5).astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 4:16] = _pack_q4k_scales(sc, mn)
        return out.reshape(-1)
    if q == QType.Q6_K:
        out = rng.integers(0, 256, size=(nb, 210), dtype=np.uint8)
        sc = rng.integers(40, 80, size=(nb, 16)).astype(np.int8)
        d = np.full(nb, std / (60 * 18.5), np.float32)  # q-32 uniform in [-32,31]: std 18.5
        out[:, 192:208] = sc.view(np.uint8)
        out[:, 208:210] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        return out.reshape(-1)
    if q == QType.Q3_K:  # value = d * (sc - 32) * (q - 4 + 4 h), code uniform in [-4, 3] (std 2.29)
        out = rng.integers(0, 256, size=(nb, 110), dtype=np.uint8)
        sc = rng.integers(40, 64, size=(nb, 16)).astype(np.uint32)  # 6-bit codes, (sc - 32) in [8, 31]
        out[:, 96:108] = _pack_q3k_scales(sc)
        d = np.full(nb, std / (20 * 2.29), np.float32)
        out[:, 108:110] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        return out.reshape(-1)
    if q == QType.Q2_K:  # value = d * (sc & 15) * q - dmin * (sc >> 4), q uniform in 0..3 (std 1.12)
        out = rng.integers(0, 256, size=(nb, 84), dtype=np.uint8)
        s4 = rng.integers(8, 16, size=(nb, 16)).astype(np.uint8)
        out[:, 0:16] = s4 | (s4 << 4)  # min code = scale code: centred around q = 1.5 with dmin = 1.5 d
        d = np.full(nb, std / (12 * 1.12), np.float32)
        out[:, 80:82] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 82:84] = (d * 1.5).astype(np.float16).view(np.uint8).reshape(-1, 2)
        return out.reshape(-1)
    if q == QType.Q8_0:
        out = rng.integers(0, 256, size=(nb, 34), dtype=np.uint8)
        d = np.full(nb, std / 73.6, np.float32)
        out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        return out.reshape(-1)
    if q in Q32_FAMILY:  # random codes, d per block around std / code-std, offsets centring the codes
        out = rng.integers(0, 256, size=(nb, bb), dtype=np.uint8)
        five = q in (QType.Q5_0, QType.Q5_1)
        cstd, centre = (9.23, 15.5) if five else (4.61, 7.5)
        d = (std / cstd) * rng.uniform(0.7, 1.3, nb).astype(np.float32)
        out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        if q in (QType.Q4_1, QType.Q5_1):
            out[:, 2:4] = (-d * centre * rng.uniform(0.9, 1.1, nb)).astype(np.float16).view(np.uint8).reshape(-1, 2)
        return out.reshape(-1)
    if q == QType.F32:
        return (rng.standard_normal(nel, dtype=np.float32) * std).view(np.uint8)
    if q == QType.F16:
        return (rng.standard_normal(nel, dtype=np.float32) * std).astype(np.float16).view(np.uint8)
    raise NotImplementedError(q.name)


# --------------------------------------------------------------------------------------------
# GPU layouts


def repack_q6_k(raw: np.ndarray, n_rows: int, row_len: int):
    """ggml Q6_K -> (blocks [n_rows, nblk*208] uint8, d [n_rows, nblk] fp16-as-uint16)."""
    q, sc, d = q6k_codes(raw)
    nb = q.shape[0]
    qg = q.reshape(nb, 4, 64)  # quarter g -> 64 elements
    lo = (qg & 0xF)
    hi = qg >> 4
    out = np.empty((nb, 208), np.uint8)
    ql = (lo[:, :, 0:32] | (lo[:, :, 32:64] << 4)).astype(np.uint8)  # [nb, 4, 32]
    out[:, 0:128] = ql.reshape(nb, 128)
    h4 = hi.reshape(nb, 4, 4, 16)  # [nb, g, s, i]
    qh = (h4[:, :, 0] | (h4[:, :, 1] << 2) | (h4[:, :, 2] << 4) | (h4[:, :, 3] << 6)).astype(np.uint8)
    out[:, 128:192] = qh.reshape(nb, 64)
    out[:, 192:208] = sc.view(np.uint8)
    dd = d.astype(np.float16).view(np.uint16)
    nblk = row_len // 256
    return out.reshape(n_rows, nblk * 208), dd.reshape(n_rows, nblk)


def repack_q8_0(raw: np.ndarray, n_rows: int, row_len: int):
    b = _blocks(raw, QType.Q8_0)
    d = b[:, 0:2].copy().view(np.uint16).reshape(n_rows, row_len // 32)
    qs = b[:, 2:34].reshape(n_rows, row_len)
    return np.ascontiguousarray(qs), np.ascontiguousarray(d)


GPU_NATIVE = (QType.Q4_K, QType.Q6_K, QType.Q8_0, QType.Q5_K, QType.MX4F, QType.MX5F, QType.Q3_K, QType.Q2_K)
# native only in the t32 tiled layout (qmv / qmm / qmm2 / qmm3 / dequant_t32 kernels); a weight of these formats
# that cannot be tiled (N % 32, expert stacks) is carried on the Q8_0 kernels instead (QWeight.ensure_kernel_layout;
# Q3_K exactly, Q2_K re-quantised)
T32_ONLY = (QType.Q5_K, QType.MX4F, QType.MX5F, QType.Q3_K, QType.Q2_K)

# Block formats without a dedicated kernel layout yet, carried on the Q8_0 kernels (qmm / qmv) instead of
# a dense 16-bit copy: the integer code of every weight is kept EXACTLY where the format is "scale x
# small int" per <= 32 weights (Q4_0, Q5_0, IQ4_NL; Q3_K's (sc-32)(q-4) fits int8 against the
# super-block d; IQ4_XS up to the f16 rounding of its per-32 scale); the offset formats (Q4_1, Q5_1,
# Q2_K, Q5_K) are re-quantised to 8 bits (error ~1/254 of the block max, well under their own).
Q8_EXACT = (QType.Q4_0, QType.Q5_0, QType.IQ4_NL, QType.IQ4_XS, QType.Q3_K)
Q8_REQUANT = (QType.Q4_1, QType.Q5_1, QType.Q2_K)


def to_q8_0(raw: np.ndarray, qtype: int, n_rows: int, row_len: int) -> np.ndarray:
    """ggml rows of another block format -> Q8_0 rows [n_rows, row_len/32 * 34] (see Q8_EXACT)."""
    q = QType(qtype)
    w = dequantize(raw, q, (row_len, n_rows)).reshape(-1, 32)
    if q in (QType.MX4F, QType.MX5F):  # exact where the block's offset is a code multiple (Q4_0 / Q5_0 origin)
        s = np.asarray(raw).reshape(-1, 192 if q == QType.MX5F else 160)[:, :32].copy().view(np.float16)
        d16 = s.reshape(-1, 2, 2, 4)[:, :, 0].reshape(-1)
        safe = np.where(d16.astype(np.float32) != 0, d16.astype(np.float32), 1.0)
        ci = np.rint(w / safe[:, None])
        out = np.empty((w.shape[0], 34), np.uint8)
        out[:, 0:2] = d16.view(np.uint8).reshape(-1, 2)
        out[:, 2:] = np.clip(ci, -127, 127).astype(np.int8).view(np.uint8)
        bad = (np.abs(ci).max(1) > 127) | (np.abs(ci * d16.astype(np.float32)[:, None] - w).max(1) > 0)
        if bad.any():
            out[bad] = quantize_q8_0(w[bad]).reshape(-1, 34)
        return out.reshape(n_rows, -1)
    if q not in Q8_EXACT:
        return quantize_q8_0(w).reshape(n_rows, -1)
    b = _blocks(np.asarray(raw).reshape(-1).view(np.uint8), q)
    if q in (QType.Q4_0, QType.Q5_0, QType.IQ4_NL):
        dd = _f16(b[:, 0:2].copy())                          # one block = 32 weights
    elif q == QType.Q3_K:
        dd = np.repeat(_f16(b[:, 108:110].copy()), 8)        # super-block d for its 8 x 32 weights
    else:  # IQ4_XS
        dd = iq4_xs_scales(b).reshape(-1)
    d16 = dd.astype(np.float16)
    safe = np.where(d16.astype(np.float32) != 0, d16.astype(np.float32), 1.0)
    ci = np.rint(w / safe[:, None])
    codes = np.clip(ci, -127, 127).astype(np.int8)
    out = np.empty((w.shape[0], 34), np.uint8)
    out[:, 0:2] = d16.view(np.uint8).reshape(-1, 2)
    out[:, 2:] = codes.view(np.uint8)
    over = np.abs(ci).max(1) > 127  # Q3_K's (-32)(-4) = 128 corner: that block re-quantised to 8 bits
    if over.any():
        out[over] = quantize_q8_0(w[over]).reshape(-1, 34)
    return out.reshape(n_rows, -1)


def repack_for_gpu(raw: np.ndarray, qtype: int, n_rows: int, row_len: int):
    """-> (data uint8 [n_rows, bytes_per_row], dplane uint16 [n_rows, x] or None)."""
    q = QType(qtype)
    if q in (QType.Q4_K, QType.Q5_K, QType.MX4F, QType.MX5F, QType.Q3_K, QType.Q2_K):
        return np.ascontiguousarray(np.asarray(raw).reshape(n_rows, -1)), None
    if q == QType.Q6_K:
        return repack_q6_k(raw, n_rows, row_len)
    if q == QType.Q8_0:
        return repack_q8_0(raw, n_rows, row_len)
    raise NotImplementedError(f"{q.name} has no native GPU layout")


T32_UNIT = {QType.Q4_K: (4608, 256), QType.Q6_K: (6784, 256), QType.Q8_0: (2176, 64), QType.Q5_K: (5632, 256),
            QType.MX4F: (5120, 256), QType.MX5F: (6144, 256), QType.Q3_K: (3584, 256), QType.Q2_K: (2688, 256)}


def tile32(data, dplane, qtype: int, n_rows: int, row_len: int):
    """GPU-native layout (see csrc/kernels/qmm.hip) -> "t32" tiled layout: columns (output rows)
    grouped 32 at a time, per (group, unit) the 32 columns' bytes stored together so every LDS-DMA /
    load wave-instruction of the qmm / qmv kernels reads contiguous memory. Works on torch tensors
    (the GPU copy, via reshapes/permutes) or numpy arrays. Returns uint8 [n_rows / 32, n_units * UNIT]."""
    import torch
    q = QType(qtype)
    if n_rows % 32 or row_len % 256 or q not in T32_UNIT:
        raise ValueError(f"t32 layout needs N % 32 == 0, K % 256 == 0 and Q4_K/Q6_K/Q8_0 (got {q.name} {n_rows}x{row_len})")
    t = data if isinstance(data, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(data))
    if t.dtype != torch.uint8:
        t = t.contiguous().view(torch.uint8)
    t = t.reshape(n_rows, -1)
    G = n_rows // 32
    if q == QType.Q4_K:
        nb = row_len // 256
        b = t.reshape(G, 32, nb, 144)
        hdr = b[..., :16].permute(0, 2, 1, 3).reshape(G, nb, 512)
        qs = b[..., 16:].reshape(G, 32, nb, 4, 2, 16).permute(0, 2, 3, 4, 1, 5).reshape(G, nb, 4096)
        out = torch.cat([hdr, qs], 2)
    elif q == QType.Q5_K:
        # ggml block {d, dmin, scales[12], qh[32], qs[128]} -> [hdr 32 x 16 B][qs as Q4_K][qh: 2 chunks x 32 x 16 B]
        nb = row_len // 256
        b = t.reshape(G, 32, nb, 176)
        hdr = b[..., :16].permute(0, 2, 1, 3).reshape(G, nb, 512)
        qh = b[..., 16:48].reshape(G, 32, nb, 2, 16).permute(0, 2, 3, 1, 4).reshape(G, nb, 1024)
        qs = b[..., 48:].reshape(G, 32, nb, 4, 2, 16).permute(0, 2, 3, 4, 1, 5).reshape(G, nb, 4096)
        out = torch.cat([hdr, qs, qh], 2)
    elif q in (QType.MX4F, QType.MX5F):
        # rows [hdr 32 | k-tile bodies] -> [hdr: 2 halves x 32 x 16 B][k-tile jq: 2 x (32 x 16 B codes) (+ 32 x 8 B qh8)]
        nb = row_len // 256
        kb = 40 if q == QType.MX5F else 32
        b = t.reshape(G, 32, nb, 32 + 4 * kb)
        hdr = b[..., :32].reshape(G, 32, nb, 2, 16).permute(0, 2, 3, 1, 4).reshape(G, nb, 1024)
        body = b[..., 32:].reshape(G, 32, nb, 4, kb)
        codes = body[..., :32].reshape(G, 32, nb, 4, 2, 16).permute(0, 2, 3, 4, 1, 5).reshape(G, nb, 4, 1024)
        if q == QType.MX5F:
            qh8 = body[..., 32:].permute(0, 2, 3, 1, 4).reshape(G, nb, 4, 256)
            codes = torch.cat([codes, qh8], 3)
        out = torch.cat([hdr, codes.reshape(G, nb, -1)], 2)
    elif q == QType.Q3_K:
        # ggml {hmask[32], qs[64], scales[12], d} -> [hdr: 32 x 16 B {scales[12], d, pad}]
        # [hmask: 2 chunks x 32 x 16 B][qs half n = 0, 1: 2 chunks x 32 x 16 B]
        nb = row_len // 256
        b = t.reshape(G, 32, nb, 110)
        hdr = torch.cat([b[..., 96:110], torch.zeros_like(b[..., 0:2])], 3).permute(0, 2, 1, 3).reshape(G, nb, 512)
        hm = b[..., 0:32].reshape(G, 32, nb, 2, 16).permute(0, 2, 3, 1, 4).reshape(G, nb, 1024)
        qs = b[..., 32:96].reshape(G, 32, nb, 2, 2, 16).permute(0, 2, 3, 4, 1, 5).reshape(G, nb, 2048)
        out = torch.cat([hdr, hm, qs], 2)
    elif q == QType.Q2_K:
        # ggml {scales[16], qs[64], d, dmin} -> [sc: 32 x 16 B][dd: 32 x 4 B {d, dmin}]
        # [qs half n = 0, 1: 2 chunks x 32 x 16 B]
        nb = row_len // 256
        b = t.reshape(G, 32, nb, 84)
        sc = b[..., 0:16].permute(0, 2, 1, 3).reshape(G, nb, 512)
        dd = b[..., 80:84].permute(0, 2, 1, 3).reshape(G, nb, 128)
        qs = b[..., 16:80].reshape(G, 32, nb, 2, 2, 16).permute(0, 2, 3, 4, 1, 5).reshape(G, nb, 2048)
        out = torch.cat([sc, dd, qs], 2)
    elif q == QType.Q6_K:
        nb = row_len // 256
        b = t.reshape(G, 32, nb, 208)
        ql = b[..., :128].reshape(G, 32, nb, 4, 2, 16)
        qh = b[..., 128:192].reshape(G, 32, nb, 4, 1, 16)
        quarters = torch.cat([ql, qh], 4).permute(0, 2, 3, 4, 1, 5).reshape(G, nb, 6144)
        sc = b[..., 192:208].permute(0, 2, 1, 3).reshape(G, nb, 512)
        d = dplane if isinstance(dplane, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(dplane))
        d = d.reshape(n_rows, nb).contiguous().view(torch.uint8).reshape(G, 32, nb, 2)
        d4 = torch.cat([d, torch.zeros_like(d)], 3).permute(0, 2, 1, 3).reshape(G, nb, 128)
        out = torch.cat([sc, d4, quarters], 2)
    else:
        nt = row_len // 64
        qs = t.reshape(G, 32, nt, 4, 16).permute(0, 2, 3, 1, 4).reshape(G, nt, 2048)
        d = dplane if isinstance(dplane, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(dplane))
        d = d.reshape(n_rows, nt * 2).contiguous().view(torch.uint8).reshape(G, 32, nt, 4).permute(0, 2, 1, 3)
        out = torch.cat([d.reshape(G, nt, 128), qs], 2)
    return out.reshape(G, -1).contiguous()


def interleave_rows16(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Interleave two [N, X] row matrices in 16-row groups: [a0..a15, b0..b15, a16..a31, ...].
    This is the gate/up layout the fused SwiGLU epilogue expects (N multiple of 16)."""
    n = a.shape[0]
    assert n % 16 == 0 and b.shape == a.shape
    out = np.empty((2 * n,) + a.shape[1:], a.dtype)
    g = n // 16
    out.reshape(g, 2, 16, *a.shape[1:])[:, 0] = a.reshape(g, 16, *a.shape[1:])
    out.reshape(g, 2, 16, *a.shape[1:])[:, 1] = b.reshape(g, 16, *a.shape[1:])
    return out
