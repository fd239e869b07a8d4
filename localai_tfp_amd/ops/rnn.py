"""Recurrent layers on the repo's kernels (csrc/kernels/audio.hip).

``lstm_bidir`` runs a bidirectional single-layer LSTM (PyTorch gate order and parameter names): the input
projections of both directions are one batched GEMM over all time steps, the recurrence is the cooperative
``lstm_bidir_coop`` kernel (hidden state spread over H/16 workgroups per direction, one grid barrier per
step) — no MIOpen RNN call. CPU tensors run torch.nn.LSTM, which is the oracle of the GPU tests.
Reference parity: the StyleTTS 2 / Kokoro text encoder and prosody predictor LSTMs
(backend/python/kokoro/models.py, bidirectional nn.LSTM, batch 1).
"""
from __future__ import annotations

import logging

import torch

from .. import _native as N

log = logging.getLogger("localai_tfp_amd.ops")


def _ref(x, p: dict, name: str):
    w = p[name + ".weight_ih_l0"]
    m = torch.nn.LSTM(w.shape[1], w.shape[0] // 4, 1, batch_first=True, bidirectional=True).to(x.device, x.dtype)
    with torch.no_grad():
        for n, prm in m.named_parameters():
            prm.copy_(p[f"{name}.{n}"])
    return m(x[None])[0][0]


def lstm_bidir(x: torch.Tensor, p: dict, name: str, cache: dict | None = None) -> torch.Tensor:
    """x [T, C] fp32 -> [T, 2H] (forward states | backward states); p holds the nn.LSTM parameters under
    `name` (weight_ih_l0, weight_hh_l0, bias_ih_l0, bias_hh_l0 and the _reverse set)."""
    H = p[name + ".weight_hh_l0"].shape[1]
    if not x.is_cuda or H not in (128, 256):
        return _ref(x, p, name)
    key = (name, x.device)
    c = cache.get(key) if cache is not None else None
    if c is None:
        wih = torch.stack([p[name + ".weight_ih_l0"], p[name + ".weight_ih_l0_reverse"]]).float()  # [2, 4H, C]
        b = torch.stack([p[name + ".bias_ih_l0"] + p[name + ".bias_hh_l0"],
                         p[name + ".bias_ih_l0_reverse"] + p[name + ".bias_hh_l0_reverse"]]).float()  # [2, 4H]
        whh = torch.stack([p[name + ".weight_hh_l0"], p[name + ".weight_hh_l0_reverse"]]).float().contiguous()
        c = (wih, b, whh)
        if cache is not None:
            cache[key] = c
    wih, b, whh = c
    T = x.shape[0]
    gx = torch.baddbmm(b[:, None, :], x.float()[None].expand(2, -1, -1), wih.transpose(1, 2)).contiguous()  # [2, T, 4H]
    hbuf = torch.zeros(2, 2, H, dtype=torch.float32, device=x.device)
    cnt = torch.zeros(3, dtype=torch.int32, device=x.device)  # two direction counters + the error flag
    out = torch.empty(T, 2 * H, dtype=torch.float32, device=x.device)
    N.kcall("mxk_lstm_bidir", gx.data_ptr(), whh.data_ptr(), hbuf.data_ptr(), out.data_ptr(), cnt.data_ptr(),
            cnt[2:].data_ptr(), T, H, N.stream_ptr())
    if int(cnt[2].item()):
        # a bounded grid-barrier spin timed out (a workgroup never arrived): the states are stale, so the
        # result is not used — recompute on the reference LSTM and say so
        log.warning("lstm_bidir %s: cooperative kernel barrier timed out (T=%d, H=%d); reference LSTM used", name, T, H)
        return _ref(x, p, name)
    return out


class LSTMStack:
    """Unidirectional multi-layer LSTM (torch.nn.LSTM parameter names / gate order, batch 1 per launch) on the
    cooperative scan kernel (mxk_lstm_coop, ND = 1): per layer one GEMM for the input gates of all time steps,
    then the recurrence. H in {128, 256, 512, 1024}; other sizes and CPU tensors run torch.nn.LSTM (the test oracle).
    Reference parity: EnCodec's decoder SLSTM (backend/python/bark, transformers MusicGen audio decoder)."""

    def __init__(self, lstm: torch.nn.LSTM):
        self.ref = lstm
        self.H, self.L = lstm.hidden_size, lstm.num_layers
        p = dict(lstm.named_parameters())
        self.layers = []
        for i in range(self.L):
            wih = p[f"weight_ih_l{i}"].detach().float().contiguous()
            whh = p[f"weight_hh_l{i}"].detach().float().contiguous()
            b = (p[f"bias_ih_l{i}"] + p[f"bias_hh_l{i}"]).detach().float().contiguous()
            self.layers.append((wih, whh, b))

    def native_ok(self, x: torch.Tensor) -> bool:
        return x.is_cuda and self.H in (128, 256, 512, 1024) and not self.ref.bidirectional and self.ref.batch_first is False

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """x [T, B, C] fp32 -> [T, B, H] (the last layer's hidden states)."""
        if not self.native_ok(x):
            return self.ref(x)[0]
        T, B, _ = x.shape
        H = self.H
        outs = []
        for bi in range(B):
            y = x[:, bi].contiguous()
            for wih, whh, b in self.layers:
                gx = torch.addmm(b, y, wih.t()).contiguous()  # [T, 4H]
                hbuf = torch.zeros(2, H, dtype=torch.float32, device=x.device)
                cnt = torch.zeros(2, dtype=torch.int32, device=x.device)  # direction counter + the error flag
                out = torch.empty(T, H, dtype=torch.float32, device=x.device)
                N.kcall("mxk_lstm_coop", gx.data_ptr(), whh.data_ptr(), hbuf.data_ptr(), out.data_ptr(), cnt.data_ptr(),
                        cnt[1:].data_ptr(), T, H, 1, N.stream_ptr())
                if int(cnt[1].item()):
                    log.warning("LSTMStack: cooperative kernel barrier timed out (T=%d, H=%d); reference LSTM used", T, H)
                    return self.ref(x)[0]
                y = out
            outs.append(y)
        return torch.stack(outs, 1)
