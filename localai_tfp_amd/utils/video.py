"""Video file writer for generated frames (the reference's diffusers `export_to_video`,
backend/python/diffusers/backend.py:340, which needs OpenCV / imageio — neither ships in this image).

* `.gif` / `.webp`: animated image through PIL;
* anything else (the gateway names its outputs `.mp4`): an ISO-BMFF MP4 with one Motion-JPEG video
  track (sample entry `jpeg`), written here box by box: ftyp, moov (mvhd, trak: tkhd, mdia: mdhd, hdlr,
  minf: vmhd, dinf/dref, stbl: stsd, stts, stsc, stsz, stco), mdat. ffmpeg / VLC / QuickTime decode it;
  no H.264 encoder is available offline.
"""
from __future__ import annotations

import io
import os
import struct


def _box(kind: bytes, *payload: bytes) -> bytes:
    body = b"".join(payload)
    return struct.pack(">I", 8 + len(body)) + kind + body


def _full(kind: bytes, version: int, flags: int, *payload: bytes) -> bytes:
    return _box(kind, struct.pack(">I", (version << 24) | flags), *payload)


_MATRIX = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def mp4_mjpeg(jpegs: list[bytes], width: int, height: int, fps: int) -> bytes:
    """MP4 bytes holding the JPEG frames at `fps` (timescale = fps, one tick per frame)."""
    fps = max(1, int(fps))
    n = len(jpegs)
    ftyp = _box(b"ftyp", b"isom", struct.pack(">I", 512), b"isomiso2mp41")
    mdat_payload = b"".join(jpegs)
    mvhd = _full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, fps, n), struct.pack(">IH", 0x10000, 0x100),
                 b"\0" * 10, _MATRIX, b"\0" * 24, struct.pack(">I", 2))
    tkhd = _full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, n), b"\0" * 8, struct.pack(">HHHH", 0, 0, 0, 0),
                 _MATRIX, struct.pack(">II", width << 16, height << 16))
    mdhd = _full(b"mdhd", 0, 0, struct.pack(">IIII", 0, 0, fps, n), struct.pack(">HH", 0x55C4, 0))
    hdlr = _full(b"hdlr", 0, 0, struct.pack(">I", 0), b"vide", b"\0" * 12, b"VideoHandler\0")
    vmhd = _full(b"vmhd", 0, 1, b"\0" * 8)
    dinf = _box(b"dinf", _full(b"dref", 0, 0, struct.pack(">I", 1), _full(b"url ", 0, 1)))
    name = b"Photo - JPEG"
    entry = _box(b"jpeg", b"\0" * 6, struct.pack(">H", 1), b"\0" * 16, struct.pack(">HH", width, height),
                 struct.pack(">II", 0x480000, 0x480000), struct.pack(">IH", 0, 1),
                 bytes([len(name)]) + name + b"\0" * (31 - len(name)), struct.pack(">Hh", 24, -1))
    stsd = _full(b"stsd", 0, 0, struct.pack(">I", 1), entry)
    stts = _full(b"stts", 0, 0, struct.pack(">III", 1, n, 1))
    stsc = _full(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, n, 1))
    stsz = _full(b"stsz", 0, 0, struct.pack(">II", 0, n), b"".join(struct.pack(">I", len(j)) for j in jpegs))

    def moov_with(offset: int) -> bytes:
        stco = _full(b"stco", 0, 0, struct.pack(">II", 1, offset))
        stbl = _box(b"stbl", stsd, stts, stsc, stsz, stco)
        minf = _box(b"minf", vmhd, dinf, stbl)
        trak = _box(b"trak", tkhd, _box(b"mdia", mdhd, hdlr, minf))
        return _box(b"moov", mvhd, trak)
    moov_len = len(moov_with(0))
    offset = len(ftyp) + moov_len + 8  # mdat payload after its 8-byte header
    return ftyp + moov_with(offset) + _box(b"mdat", mdat_payload)


def write_video(frames: list, path: str, fps: int = 7, quality: int = 90) -> str:
    """frames: PIL images (same size). Format from the extension (.gif / .webp, else MP4 Motion-JPEG)."""
    if not frames:
        raise ValueError("write_video: no frames")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    ext = os.path.splitext(path)[1].lower()
    fps = max(1, int(fps))
    if ext in (".gif", ".webp"):
        frames[0].save(path, save_all=True, append_images=frames[1:], duration=int(1000 / fps), loop=0)
        return path
    jpegs = []
    for f in frames:
        b = io.BytesIO()
        f.convert("RGB").save(b, format="JPEG", quality=quality)
        jpegs.append(b.getvalue())
    w, h = frames[0].size
    with open(path, "wb") as fh:
        fh.write(mp4_mjpeg(jpegs, w, h, fps))
    return path


def read_mp4_boxes(data: bytes, start: int = 0, end: int | None = None) -> list[tuple[bytes, int, int]]:
    """(type, payload offset, payload length) of the boxes in data[start:end] (tests / inspection)."""
    end = len(data) if end is None else end
    out = []
    i = start
    while i + 8 <= end:
        size, kind = struct.unpack(">I4s", data[i:i + 8])
        if size < 8:
            break
        out.append((kind, i + 8, size - 8))
        i += size
    return out
