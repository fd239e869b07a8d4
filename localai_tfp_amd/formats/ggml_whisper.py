"""whisper.cpp's legacy ggml model container (`ggml-base.bin`, `ggml-base-q5_1.bin`, ...) — the
files the reference's whisper backend loads with `whisper.New(opts.ModelFile)`
(backend/go/transcribe/whisper/whisper.go:20-25).

Layout (little endian, no alignment padding):
  u32 magic 0x67676d6c
  i32 x 11 hparams: n_vocab n_audio_ctx n_audio_state n_audio_head n_audio_layer n_text_ctx
                    n_text_state n_text_head n_text_layer n_mels ftype
  i32 n_mel, i32 n_fft, f32[n_mel * n_fft] mel filterbank
  i32 n_tokens, n_tokens x (u32 len, bytes) vocabulary pieces in rank order
  tensors until EOF: i32 n_dims, i32 name_len, i32 ggml_type, i32[n_dims] ne (ne0 first),
                     name bytes, raw data
Tensor data stays memory-mapped; `tensor(name)` dequantises on demand (ops.quant.dequantize).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

from .gguf import BLOCK, QType

MAGIC = 0x67676D6C
HPARAMS = ("n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
           "n_text_state", "n_text_head", "n_text_layer", "n_mels", "ftype")


@dataclass
class TensorInfo:
    name: str
    qtype: int
    shape: tuple  # ggml order (ne0 first)
    offset: int
    nbytes: int


def _nbytes(qtype: int, shape) -> int:
    n = int(np.prod(shape)) if len(shape) else 1
    be, bb = BLOCK[QType(qtype)]
    return n // be * bb


class GGMLWhisperFile:
    def __init__(self, path: str):
        self.path = path
        self.mm = np.memmap(path, np.uint8, mode="r")
        buf = self.mm
        (magic,) = struct.unpack_from("<I", buf, 0)
        if magic != MAGIC:
            raise ValueError(f"{path}: not a ggml whisper model (magic {magic:#x})")
        off = 4
        vals = struct.unpack_from("<11i", buf, off)
        off += 44
        self.hparams = dict(zip(HPARAMS, vals))
        n_mel, n_fft = struct.unpack_from("<ii", buf, off)
        off += 8
        self.mel_filters = np.frombuffer(buf, np.float32, n_mel * n_fft, off).reshape(n_mel, n_fft).copy()
        off += 4 * n_mel * n_fft
        (n_tok,) = struct.unpack_from("<i", buf, off)
        off += 4
        self.vocab: list[bytes] = []
        for _ in range(n_tok):
            (ln,) = struct.unpack_from("<I", buf, off)
            off += 4
            self.vocab.append(bytes(buf[off:off + ln]))
            off += ln
        self.tensors: dict[str, TensorInfo] = {}
        size = len(buf)
        while off + 12 <= size:
            n_dims, name_len, ttype = struct.unpack_from("<iii", buf, off)
            off += 12
            shape = struct.unpack_from(f"<{n_dims}i", buf, off)
            off += 4 * n_dims
            name = bytes(buf[off:off + name_len]).decode()
            off += name_len
            nb = _nbytes(ttype, shape)
            self.tensors[name] = TensorInfo(name, ttype, tuple(shape), off, nb)
            off += nb

    def tensor(self, name: str) -> np.ndarray | None:
        from ..ops.quant import dequantize
        ti = self.tensors.get(name)
        if ti is None:
            return None
        a = dequantize(self.mm[ti.offset: ti.offset + ti.nbytes], ti.qtype, ti.shape)
        # 1-D parameters are sometimes stored as [n, 1] / [1, n]
        if name.endswith(".bias") or "ln" in name.rsplit(".", 2)[-2]:
            a = a.reshape(-1)
        return a


def write_ggml_whisper(path: str, hparams: dict, mel_filters: np.ndarray, vocab: list[bytes],
                       tensors: dict[str, np.ndarray], f16: bool = True):
    """Write a ggml whisper file (tests / synthetic checkpoints). 2-D+ weights as F16 when `f16`."""
    with open(path, "wb") as f:
        f.write(struct.pack("<I", MAGIC))
        f.write(struct.pack("<11i", *(int(hparams[k]) for k in HPARAMS)))
        f.write(struct.pack("<ii", *mel_filters.shape))
        f.write(np.ascontiguousarray(mel_filters, np.float32).tobytes())
        f.write(struct.pack("<i", len(vocab)))
        for p in vocab:
            f.write(struct.pack("<I", len(p)) + p)
        for name, a in tensors.items():
            a = np.asarray(a, np.float32)
            half = f16 and a.ndim >= 2 and "positional" not in name
            ne = tuple(reversed(a.shape))
            nm = name.encode()
            f.write(struct.pack("<iii", a.ndim, len(nm), 1 if half else 0))
            f.write(struct.pack(f"<{a.ndim}i", *ne))
            f.write(nm)
            f.write(np.ascontiguousarray(a, np.float16 if half else np.float32).tobytes())
