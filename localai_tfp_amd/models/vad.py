"""Silero voice-activity detector (v5, 16 kHz) — the reference's `silero-vad` backend
(backend/go/vad/silero/vad.go:17-57 over silero-vad-go speech.Detector + onnxruntime).

The reference runs the ONNX graph once per 512-sample window (32 ms), carrying the LSTM state and a
64-sample context between calls. Here a whole clip is one batched pass:

  1. windows  [T, 64 + 512]   context-prefixed windows built with one unfold (no Python loop)
  2. STFT     reflection pad -> frames [T*4, 256] @ basis^T [256, 258] -> |X| [T, 129, 4]
  3. encoder  4 x (conv1d k3 + ReLU) over all T windows at once (129->128->64->64->128 channels,
              strides 1,2,2,1 -> one 128-vector per window)
  4. gates    gx = enc @ W_ih^T + b_ih + b_hh for every window in one GEMM
  5. scan     csrc/kernels/audio.hip lstm_scan<128, HEAD>: the only sequential part; W_hh stays in
              VGPRs, the decoder head (ReLU -> 1x1 conv -> sigmoid) is fused, output = p(speech)
              per window.
  6. segments the speech.Detector.Detect state machine (threshold 0.5, negative threshold
              threshold-0.15, min-silence 0, speech-pad 0 as the reference configures it).

Weights: a silero v5 state dict (safetensors or a weights-only torch file) with the JIT module's
names (`_model.stft.forward_basis_buffer`, `_model.encoder.N.reparam_conv.*`,
`_model.decoder.rnn.*`, `_model.decoder.decoder.2.*`), or `synthetic:silero-vad` (exact DFT basis,
random encoder/LSTM). Each request starts from a zero state (the Go detector carries state across
Detect calls until Reset, which makes results depend on request order; per-request state is the
deterministic choice).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

SR = 16000
WINDOW = 512
CONTEXT = 64
N_FFT = 256
HOP = 128
HIDDEN = 128
ENC = [(129, 128, 1), (128, 64, 2), (64, 64, 2), (64, 128, 1)]  # (in, out, stride), kernel 3, pad 1


@dataclass
class VADParams:
    threshold: float = 0.5
    min_silence_ms: int = 0
    speech_pad_ms: int = 0


def dft_basis(n_fft: int = N_FFT) -> torch.Tensor:
    """[n_fft + 2, 1, n_fft] real/imag Fourier basis with a periodic Hann window (silero's STFT)."""
    n = torch.arange(n_fft, dtype=torch.float64)
    k = torch.arange(n_fft // 2 + 1, dtype=torch.float64)[:, None]
    win = 0.5 - 0.5 * torch.cos(2 * math.pi * n / n_fft)
    ang = 2 * math.pi * k * n / n_fft
    basis = torch.cat([torch.cos(ang) * win, -torch.sin(ang) * win], 0)
    return basis.float()[:, None, :]


def synthetic_state_dict(seed: int = 0) -> dict:
    g = torch.Generator().manual_seed(seed)
    sd = {"stft.forward_basis_buffer": dft_basis()}
    for i, (ci, co, _) in enumerate(ENC):
        sd[f"encoder.{i}.reparam_conv.weight"] = torch.randn(co, ci, 3, generator=g) / math.sqrt(3 * ci)
        sd[f"encoder.{i}.reparam_conv.bias"] = torch.randn(co, generator=g) * 0.05
    s = 1 / math.sqrt(HIDDEN)
    for n, shp in (("weight_ih", (4 * HIDDEN, HIDDEN)), ("weight_hh", (4 * HIDDEN, HIDDEN)),
                   ("bias_ih", (4 * HIDDEN,)), ("bias_hh", (4 * HIDDEN,))):
        sd[f"decoder.rnn.{n}"] = (torch.rand(*shp, generator=g) * 2 - 1) * s
    sd["decoder.decoder.2.weight"] = torch.randn(1, HIDDEN, 1, generator=g) * s
    sd["decoder.decoder.2.bias"] = torch.zeros(1)
    return sd


def onnx_state_dict(path) -> dict:
    """silero_vad.onnx (the gallery's file, backend/go/vad/silero/vad.go:15-54) -> state dict: the weight
    initializers are read with the protobuf-only ONNX reader (formats/onnx.py) — v5 keeps them inside
    the 16 kHz / 8 kHz If branches — and matched to this module's names by suffix and shape; the 16 kHz
    set wins. The ONNX graph itself is not run (parity vs onnxruntime unpinned)."""
    from ..formats.onnx import initializers
    tensors, _ = initializers(path)
    want = {k: tuple(v.shape) for k, v in synthetic_state_dict().items()}
    out = {}
    for k, shape in want.items():
        cands = [(q, a) for q, a in tensors.items() if q.endswith(k) and tuple(a.shape) == shape]
        if not cands:
            continue
        cands.sort(key=lambda qa: ("8k" in qa[0], len(qa[0])))  # 16 kHz branch first
        out[k] = torch.from_numpy(np.asarray(cands[0][1], np.float32).copy())
    missing = [k for k in want if k not in out and k != "stft.forward_basis_buffer"]
    if missing:
        raise ValueError(f"{path}: silero-vad weights not found in the ONNX initializers: {missing[:4]}... "
                         f"({len(tensors)} tensors present, e.g. {list(tensors)[:4]})")
    if "stft.forward_basis_buffer" not in out:
        out["stft.forward_basis_buffer"] = dft_basis()
    return out


def load_state_dict(path: str) -> dict:
    if path.startswith("synthetic:"):
        return synthetic_state_dict()
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path)
    elif path.endswith(".onnx"):
        return onnx_state_dict(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd:
            sd = sd["state_dict"]
    out = {}
    for k, v in sd.items():
        for pre in ("_model.", "model."):
            if k.startswith(pre):
                k = k[len(pre):]
        out[k] = v.float()
    if "stft.forward_basis_buffer" not in out:
        out["stft.forward_basis_buffer"] = dft_basis()
    return out


class SileroVAD:
    def __init__(self, sd: dict, device="cpu"):
        self.device = torch.device(device)
        d = {k: v.to(self.device).contiguous() for k, v in sd.items()}
        basis = d["stft.forward_basis_buffer"]
        self.basis_t = basis[:, 0, :].t().contiguous()  # [256, 258]
        self.enc = [(d[f"encoder.{i}.reparam_conv.weight"], d[f"encoder.{i}.reparam_conv.bias"], s)
                    for i, (_, _, s) in enumerate(ENC)]
        self.w_ih = d["decoder.rnn.weight_ih"]
        self.w_hh = d["decoder.rnn.weight_hh"].contiguous()
        self.b_gates = d["decoder.rnn.bias_ih"] + d["decoder.rnn.bias_hh"]
        self.head_w = d["decoder.decoder.2.weight"].reshape(-1).contiguous()
        self.head_b = float(d["decoder.decoder.2.bias"].reshape(-1)[0])

    @classmethod
    def load(cls, path: str, device="cpu") -> "SileroVAD":
        return cls(load_state_dict(path), device)

    # ---------------------------------------------------------------------------- model
    def _windows(self, audio: torch.Tensor) -> torch.Tensor:
        """[T, CONTEXT + WINDOW]: window t with the last CONTEXT samples of window t-1 in front
        (zeros before the first), as the Go detector feeds the ONNX graph. Like Detect, a trailing
        partial window is dropped (`for i := 0; i < len(pcm)-windowSize; i += windowSize`)."""
        T = max(0, (audio.numel() - 1) // WINDOW)
        if T == 0:
            return audio.new_zeros(0, CONTEXT + WINDOW)
        x = torch.cat([audio.new_zeros(CONTEXT), audio[: T * WINDOW]])
        return x.unfold(0, CONTEXT + WINDOW, WINDOW)

    def encode(self, win: torch.Tensor) -> torch.Tensor:
        """[T, 576] windows -> [T, 128] encoder features."""
        x = F.pad(win[:, None, :], (0, CONTEXT), mode="reflect")[:, 0]  # [T, 640]
        frames = x.unfold(1, N_FFT, HOP)  # [T, 4, 256]
        spec = frames.reshape(-1, N_FFT) @ self.basis_t  # [T*4, 258]
        half = N_FFT // 2 + 1
        mag = torch.sqrt(spec[:, :half] ** 2 + spec[:, half:] ** 2)
        h = mag.reshape(win.shape[0], -1, half).transpose(1, 2)  # [T, 129, 4]
        for w, b, s in self.enc:
            h = F.relu(F.conv1d(h, w, b, stride=s, padding=1))
        return h[:, :, 0]

    def probs(self, audio) -> torch.Tensor:
        """Speech probability per 512-sample window, [T] fp32 (on the model device)."""
        a = torch.as_tensor(np.asarray(audio, dtype=np.float32)).to(self.device)
        win = self._windows(a)
        T = win.shape[0]
        if T == 0:
            return torch.zeros(0, device=self.device)
        gx = torch.addmm(self.b_gates, self.encode(win), self.w_ih.t())  # [T, 512]
        if self.device.type == "cuda":
            from .. import _native as N
            h = torch.zeros(1, HIDDEN, device=self.device)
            c = torch.zeros(1, HIDDEN, device=self.device)
            out = torch.empty(1, T, device=self.device)
            N.kcall("mxk_lstm_scan", gx.data_ptr(), self.w_hh.data_ptr(), h.data_ptr(), c.data_ptr(),
                    self.head_w.data_ptr(), self.head_b, out.data_ptr(), 1, T, HIDDEN, N.stream_ptr())
            return out[0]
        return lstm_scan_ref(gx, self.w_hh, self.head_w, self.head_b)

    def detect(self, audio, p: VADParams | None = None) -> list[tuple[float, float]]:
        p = p or VADParams()
        return segments(self.probs(audio).cpu().numpy(), p)


def lstm_scan_ref(gx: torch.Tensor, w_hh: torch.Tensor, head_w, head_b: float) -> torch.Tensor:
    """fp32 reference of the fused scan (PyTorch LSTMCell gate order i, f, g, o)."""
    H = w_hh.shape[1]
    h = gx.new_zeros(H)
    c = gx.new_zeros(H)
    out = gx.new_empty(gx.shape[0])
    for t in range(gx.shape[0]):
        g = gx[t] + w_hh @ h
        i, f, gg, o = g[:H].sigmoid(), g[H:2 * H].sigmoid(), g[2 * H:3 * H].tanh(), g[3 * H:].sigmoid()
        c = f * c + i * gg
        h = o * c.tanh()
        out[t] = torch.sigmoid(F.relu(h) @ head_w + head_b)
    return out


def segments(probs: np.ndarray, p: VADParams) -> list[tuple[float, float]]:
    """speech.Detector.Detect's hysteresis (silero-vad-go): start when p >= threshold, end after
    p < threshold - 0.15 has held for min_silence; times in seconds. A segment still open at the end
    of the clip keeps end = 0, as the Go detector leaves it."""
    min_sil = p.min_silence_ms * SR // 1000
    pad = p.speech_pad_ms * SR // 1000
    segs: list[list[float]] = []
    triggered = False
    temp_end = 0
    cur = 0
    for prob in probs:
        cur += WINDOW
        if prob >= p.threshold and temp_end:
            temp_end = 0
        if prob >= p.threshold and not triggered:
            triggered = True
            segs.append([max(0.0, (cur - WINDOW - pad) / SR), 0.0])
        if prob < p.threshold - 0.15 and triggered:
            if not temp_end:
                temp_end = cur
            if cur - temp_end < min_sil:
                continue
            segs[-1][1] = (temp_end + pad) / SR
            temp_end = 0
            triggered = False
    return [(a, b) for a, b in segs]


def env_params() -> VADParams:
    return VADParams(threshold=float(os.environ.get("MX_VAD_THRESHOLD", "0.5")))
