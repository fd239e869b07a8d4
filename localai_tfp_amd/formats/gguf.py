"""GGUF v2/v3 reader and writer (zero-copy tensor views over an mmap).

The reference consumes GGUF through llama.cpp (`common_init_from_params`, reached from
backend/cpp/llama/grpc-server.cpp:509) and parses the header a second time in Go to guess
defaults (core/config/gguf.go:149-253). This module does both jobs for the MI355X worker: the
metadata dict drives :mod:`localai_tfp_amd.config.guesser`, and :meth:`GGUFReader.tensor` hands out
``numpy.memmap`` views that the loader repacks into the GPU weight layouts of ``ops/quant.py``.
The writer exists so tests and ``bench.py`` can produce synthetic random-init checkpoints of the
exact Llama-3 architectures named in BASELINE.json (there is no network to fetch real ones).
"""
from __future__ import annotations

import mmap
import struct
from dataclasses import dataclass, field
from enum import IntEnum
from pathlib import Path
from typing import Any, BinaryIO

import numpy as np

GGUF_MAGIC = 0x46554747  # b"GGUF" little-endian
DEFAULT_ALIGNMENT = 32


class GType(IntEnum):
    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


_SCALAR_FMT = {
    GType.UINT8: "<B", GType.INT8: "<b", GType.UINT16: "<H", GType.INT16: "<h",
    GType.UINT32: "<I", GType.INT32: "<i", GType.FLOAT32: "<f", GType.BOOL: "<?",
    GType.UINT64: "<Q", GType.INT64: "<q", GType.FLOAT64: "<d",
}
_NP_OF = {
    GType.UINT8: np.uint8, GType.INT8: np.int8, GType.UINT16: np.uint16, GType.INT16: np.int16,
    GType.UINT32: np.uint32, GType.INT32: np.int32, GType.FLOAT32: np.float32, GType.BOOL: np.bool_,
    GType.UINT64: np.uint64, GType.INT64: np.int64, GType.FLOAT64: np.float64,
}


class QType(IntEnum):
    """ggml tensor types (ggml.h numbering, as stored in GGUF)."""
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    IQ2_XXS = 16
    IQ2_XS = 17
    IQ3_XXS = 18
    IQ1_S = 19
    IQ4_NL = 20
    IQ3_S = 21
    IQ2_S = 22
    IQ4_XS = 23
    I8 = 24
    I16 = 25
    I32 = 26
    I64 = 27
    F64 = 28
    IQ1_M = 29
    BF16 = 30
    TQ1_0 = 34
    TQ2_0 = 35
    # this framework's GPU block layouts (never stored in a GGUF file): 4- / 5-bit codes with an f16 scale and
    # offset per 32 weights, w = s * code + m — Q4_0 / Q4_1 / Q5_0 / Q5_1 rows re-laid out exactly (ops/quant.py)
    MX4F = 240
    MX5F = 241


# (elements per block, bytes per block)
BLOCK = {
    QType.F32: (1, 4), QType.F16: (1, 2), QType.BF16: (1, 2), QType.F64: (1, 8),
    QType.I8: (1, 1), QType.I16: (1, 2), QType.I32: (1, 4), QType.I64: (1, 8),
    QType.Q4_0: (32, 18), QType.Q4_1: (32, 20), QType.Q5_0: (32, 22), QType.Q5_1: (32, 24),
    QType.Q8_0: (32, 34), QType.Q8_1: (32, 36),
    QType.Q2_K: (256, 84), QType.Q3_K: (256, 110), QType.Q4_K: (256, 144), QType.Q5_K: (256, 176),
    QType.Q6_K: (256, 210), QType.Q8_K: (256, 292),
    QType.IQ2_XXS: (256, 66), QType.IQ2_XS: (256, 74), QType.IQ3_XXS: (256, 98), QType.IQ1_S: (256, 50),
    QType.IQ4_NL: (32, 18), QType.IQ3_S: (256, 110), QType.IQ2_S: (256, 82), QType.IQ4_XS: (256, 136),
    QType.IQ1_M: (256, 56), QType.TQ1_0: (256, 54), QType.TQ2_0: (256, 66),
    QType.MX4F: (256, 160), QType.MX5F: (256, 192),
}

# GGUF file-type ids (general.file_type) for naming
FILE_TYPE_NAMES = {0: "F32", 1: "F16", 2: "Q4_0", 3: "Q4_1", 7: "Q8_0", 8: "Q5_0", 9: "Q5_1",
                   10: "Q2_K", 11: "Q3_K_S", 12: "Q3_K_M", 13: "Q3_K_L", 14: "Q4_K_S", 15: "Q4_K_M",
                   16: "Q5_K_S", 17: "Q5_K_M", 18: "Q6_K", 32: "BF16"}


def tensor_nbytes(qtype: int, shape) -> int:
    n = int(np.prod(shape)) if len(shape) else 1
    be, bb = BLOCK[QType(qtype)]
    if n % be:
        raise ValueError(f"{QType(qtype).name}: {n} elements not a multiple of block {be}")
    return n // be * bb


@dataclass
class TensorInfo:
    name: str
    shape: tuple  # ggml order: shape[0] = innermost (row length)
    qtype: int
    offset: int  # relative to data section
    nbytes: int = 0

    @property
    def rows(self) -> int:
        return int(np.prod(self.shape[1:])) if len(self.shape) > 1 else 1

    @property
    def row_len(self) -> int:
        return int(self.shape[0])


class GGUFReader:
    """Parses the header eagerly; tensor bytes are mmap views (no copy until the loader repacks)."""

    def __init__(self, path: str | Path):
        self.path = Path(path)
        self._f = open(self.path, "rb")
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        self.metadata: dict[str, Any] = {}
        self.tensors: dict[str, TensorInfo] = {}
        self._parse()

    # -- low level readers over the mmap --
    def _rd(self, fmt):
        v = struct.unpack_from(fmt, self._mm, self._p)
        self._p += struct.calcsize(fmt)
        return v[0]

    def _rd_str(self):
        n = self._rd("<Q")
        s = self._mm[self._p:self._p + n].decode("utf-8", errors="replace")
        self._p += n
        return s

    def _rd_val(self, t: int):
        t = GType(t)
        if t == GType.STRING:
            return self._rd_str()
        if t == GType.ARRAY:
            et = GType(self._rd("<I"))
            n = self._rd("<Q")
            if et == GType.STRING:
                return [self._rd_str() for _ in range(n)]
            if et == GType.ARRAY:
                return [self._rd_val(GType.ARRAY) for _ in range(n)]
            dt = np.dtype(_NP_OF[et]).newbyteorder("<")
            arr = np.frombuffer(self._mm, dtype=dt, count=n, offset=self._p).copy()
            self._p += n * dt.itemsize
            return arr
        return self._rd(_SCALAR_FMT[t])

    def _parse(self):
        self._p = 0
        magic = self._rd("<I")
        if magic != GGUF_MAGIC:
            raise ValueError(f"{self.path}: not a GGUF file (magic {magic:#x})")
        self.version = self._rd("<I")
        if self.version not in (2, 3):
            raise ValueError(f"unsupported GGUF version {self.version}")
        n_t = self._rd("<Q")
        n_kv = self._rd("<Q")
        for _ in range(n_kv):
            k = self._rd_str()
            t = self._rd("<I")
            self.metadata[k] = self._rd_val(t)
        infos = []
        for _ in range(n_t):
            name = self._rd_str()
            nd = self._rd("<I")
            shape = tuple(self._rd("<Q") for _ in range(nd))
            qt = self._rd("<I")
            off = self._rd("<Q")
            ti = TensorInfo(name, shape, qt, off)
            ti.nbytes = tensor_nbytes(qt, shape)
            infos.append(ti)
        align = int(self.metadata.get("general.alignment", DEFAULT_ALIGNMENT))
        self.alignment = align
        self.data_offset = (self._p + align - 1) // align * align
        for ti in infos:
            self.tensors[ti.name] = ti

    def tensor_bytes(self, name: str) -> np.ndarray:
        ti = self.tensors[name]
        return np.frombuffer(self._mm, dtype=np.uint8, count=ti.nbytes, offset=self.data_offset + ti.offset)

    def tensor(self, name: str) -> np.ndarray:
        """Dense tensors as typed arrays (numpy order = reversed ggml shape); quantised as raw bytes
        shaped [rows, bytes_per_row]."""
        ti = self.tensors[name]
        raw = self.tensor_bytes(name)
        shp = tuple(reversed(ti.shape))
        q = QType(ti.qtype)
        if q == QType.F32:
            return raw.view(np.float32).reshape(shp)
        if q == QType.F16:
            return raw.view(np.float16).reshape(shp)
        if q == QType.BF16:
            return raw.view(np.uint16).reshape(shp)
        if q in (QType.I8, QType.I16, QType.I32, QType.I64, QType.F64):
            dt = {QType.I8: np.int8, QType.I16: np.int16, QType.I32: np.int32, QType.I64: np.int64,
                  QType.F64: np.float64}[q]
            return raw.view(dt).reshape(shp)
        return raw.reshape(ti.rows, -1)

    def get(self, key: str, default=None):
        return self.metadata.get(key, default)

    @property
    def architecture(self) -> str:
        return str(self.metadata.get("general.architecture", "llama"))

    def arch_get(self, key: str, default=None):
        return self.metadata.get(f"{self.architecture}.{key}", default)

    def close(self):
        try:
            self._mm.close()
        except BufferError:
            pass  # numpy views still alive; the map is released when they are
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ------------------------------------------------------------------------------------------------
@dataclass
class _WTensor:
    name: str
    shape: tuple  # ggml order
    qtype: int
    data: Any  # bytes-like or callable returning bytes
    nbytes: int


@dataclass
class GGUFWriter:
    """Streaming GGUF v3 writer. Tensor payloads may be callables so multi-GB synthetic models are
    generated block by block without holding the whole file in memory."""

    path: str | Path
    metadata: dict = field(default_factory=dict)
    alignment: int = DEFAULT_ALIGNMENT
    _tensors: list = field(default_factory=list)
    _types: dict = field(default_factory=dict)

    def add(self, key: str, value, gtype: GType | None = None):
        self.metadata[key] = value
        if gtype is not None:
            self._types[key] = gtype

    def add_tensor(self, name: str, data, shape=None, qtype: int = QType.F32):
        """`data`: numpy array (dense; shape inferred) or bytes/callable with explicit ggml `shape`."""
        if isinstance(data, np.ndarray) and shape is None:
            shape = tuple(reversed(data.shape))
            qtype = {np.dtype(np.float32): QType.F32, np.dtype(np.float16): QType.F16,
                     np.dtype(np.int32): QType.I32}.get(data.dtype, qtype)
            payload = np.ascontiguousarray(data).tobytes()
        else:
            payload = data
        nb = tensor_nbytes(qtype, shape)
        self._tensors.append(_WTensor(name, tuple(int(s) for s in shape), int(qtype), payload, nb))

    @staticmethod
    def _guess_type(v):
        if isinstance(v, bool):
            return GType.BOOL
        if isinstance(v, int):
            return GType.INT64 if (v < -2**31 or v >= 2**31) else (GType.UINT32 if v >= 0 else GType.INT32)
        if isinstance(v, float):
            return GType.FLOAT32
        if isinstance(v, str):
            return GType.STRING
        if isinstance(v, (list, tuple, np.ndarray)):
            return GType.ARRAY
        raise TypeError(type(v))

    def _w_str(self, f: BinaryIO, s: str):
        b = s.encode("utf-8")
        f.write(struct.pack("<Q", len(b)))
        f.write(b)

    def _w_val(self, f, v, t: GType):
        if t == GType.STRING:
            self._w_str(f, v)
        elif t == GType.ARRAY:
            if isinstance(v, np.ndarray):
                et = {np.dtype(np.float32): GType.FLOAT32, np.dtype(np.int32): GType.INT32,
                      np.dtype(np.uint32): GType.UINT32, np.dtype(np.int64): GType.INT64,
                      np.dtype(np.uint8): GType.UINT8, np.dtype(np.int8): GType.INT8,
                      np.dtype(np.bool_): GType.BOOL, np.dtype(np.float64): GType.FLOAT64}[v.dtype]
                f.write(struct.pack("<IQ", et, len(v)))
                f.write(np.ascontiguousarray(v).astype(v.dtype.newbyteorder("<")).tobytes())
                return
            vals = list(v)
            et = self._guess_type(vals[0]) if vals else GType.INT32
            if et == GType.UINT32 and any(isinstance(x, int) and x < 0 for x in vals):
                et = GType.INT32
            f.write(struct.pack("<IQ", et, len(vals)))
            for x in vals:
                self._w_val(f, x, et)
        else:
            f.write(struct.pack(_SCALAR_FMT[t], v))

    def write(self):
        p = Path(self.path)
        with open(p, "wb") as f:
            f.write(struct.pack("<IIQQ", GGUF_MAGIC, 3, len(self._tensors), len(self.metadata) + 1))
            meta = dict(self.metadata)
            meta["general.alignment"] = self.alignment
            self._types.setdefault("general.alignment", GType.UINT32)
            # write the alignment key first (readers rely on it being present before data)
            for k, v in meta.items():
                self._w_str(f, k)
                t = self._types.get(k) or self._guess_type(v)
                f.write(struct.pack("<I", t))
                self._w_val(f, v, t)
            off = 0
            offsets = []
            for t in self._tensors:
                offsets.append(off)
                off += (t.nbytes + self.alignment - 1) // self.alignment * self.alignment
            for t, o in zip(self._tensors, offsets):
                self._w_str(f, t.name)
                f.write(struct.pack("<I", len(t.shape)))
                for s in t.shape:
                    f.write(struct.pack("<Q", s))
                f.write(struct.pack("<IQ", t.qtype, o))
            pos = f.tell()
            pad = (pos + self.alignment - 1) // self.alignment * self.alignment - pos
            f.write(b"\0" * pad)
            for t, o in zip(self._tensors, offsets):
                data = t.data() if callable(t.data) else t.data
                if isinstance(data, np.ndarray):
                    data = data.tobytes()
                if len(data) != t.nbytes:
                    raise ValueError(f"{t.name}: payload {len(data)} B != expected {t.nbytes} B")
                f.write(data)
                pad = (t.nbytes + self.alignment - 1) // self.alignment * self.alignment - t.nbytes
                f.write(b"\0" * pad)
        return p
