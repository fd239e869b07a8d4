"""Audio I/O shared by the speech workers (whisper, VAD, TTS, sound generation).

The reference converts every upload with an ffmpeg subprocess to 16 kHz mono s16 WAV
(pkg/utils/ffmpeg.go:19-27) and decodes it with go-audio/wav (whisper.go:42-55). Here WAV in any
PCM / IEEE-float layout is parsed natively and resampled with a polyphase filter; other containers
(mp3, ogg, webm, ...) go through ffmpeg when it is installed, exactly like the reference.
"""
from __future__ import annotations

import math
import os
import shutil
import struct
import subprocess
import tempfile

import numpy as np

SAMPLE_RATE = 16000


def _parse_wav(data: bytes) -> tuple[np.ndarray, int]:
    if data[:4] not in (b"RIFF", b"RF64") or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file")
    off = 12
    fmt = None
    pcm = None
    while off + 8 <= len(data):
        cid, size = data[off:off + 4], struct.unpack_from("<I", data, off + 4)[0]
        body = data[off + 8: off + 8 + size]
        if cid == b"fmt ":
            tag, ch, rate, _, _, bits = struct.unpack_from("<HHIIHH", body, 0)
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: subformat GUID's first u16
                tag = struct.unpack_from("<H", body, 24)[0]
            fmt = (tag, ch, rate, bits)
        elif cid == b"data":
            pcm = body if size != 0xFFFFFFFF else data[off + 8:]
        off += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError("WAV without fmt/data chunk")
    tag, ch, rate, bits = fmt
    if tag == 3:
        x = np.frombuffer(pcm[: len(pcm) // (bits // 8) * (bits // 8)], "<f4" if bits == 32 else "<f8").astype(np.float32)
    elif tag == 1:
        if bits == 8:
            x = (np.frombuffer(pcm, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(pcm[: len(pcm) // 2 * 2], "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(pcm[: len(pcm) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = np.frombuffer(pcm[: len(pcm) // 4 * 4], "<i4").astype(np.float32) / float(1 << 31)
        else:
            raise ValueError(f"unsupported PCM width {bits}")
    else:
        raise ValueError(f"unsupported WAV format tag {tag}")
    x = x[: len(x) // ch * ch].reshape(-1, ch).mean(axis=1) if ch > 1 else x
    return np.ascontiguousarray(x, np.float32), rate


def resample(x: np.ndarray, sr: int, target: int = SAMPLE_RATE) -> np.ndarray:
    if sr == target or len(x) == 0:
        return x.astype(np.float32, copy=False)
    from scipy.signal import resample_poly
    g = math.gcd(sr, target)
    return resample_poly(x, target // g, sr // g).astype(np.float32)


def load_audio(path: str, sr: int = SAMPLE_RATE) -> np.ndarray:
    """Any audio file -> float32 mono PCM in [-1, 1] at `sr`."""
    with open(path, "rb") as f:
        data = f.read()
    try:
        x, rate = _parse_wav(data)
        return resample(x, rate, sr)
    except ValueError:
        pass
    ff = shutil.which("ffmpeg")
    if ff is None:
        raise ValueError(f"{os.path.basename(path)}: not a WAV file and ffmpeg is not installed")
    r = subprocess.run([ff, "-nostdin", "-i", path, "-f", "s16le", "-ac", "1", "-ar", str(sr), "-"],
                       capture_output=True, check=False)
    if r.returncode != 0:
        raise ValueError(f"ffmpeg failed: {r.stderr.decode(errors='replace')[-400:]}")
    return np.frombuffer(r.stdout, "<i2").astype(np.float32) / 32768.0


def wav_bytes(x: np.ndarray, sr: int = SAMPLE_RATE) -> bytes:
    """float32 mono -> 16-bit PCM WAV bytes."""
    pcm = (np.clip(np.asarray(x, np.float32), -1.0, 1.0) * 32767.0).astype("<i2").tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(pcm)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, sr, sr * 2, 2, 16)
    return hdr + b"data" + struct.pack("<I", len(pcm)) + pcm


def write_wav(path: str, x: np.ndarray, sr: int = SAMPLE_RATE) -> str:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d or None, suffix=".wav")
    with os.fdopen(fd, "wb") as f:
        f.write(wav_bytes(x, sr))
    os.replace(tmp, path)
    return path


def read_wav_bytes(data: bytes, sr: int = SAMPLE_RATE) -> np.ndarray:
    x, rate = _parse_wav(data)
    return resample(x, rate, sr)


__all__ = ["SAMPLE_RATE", "load_audio", "resample", "wav_bytes", "write_wav", "read_wav_bytes"]
