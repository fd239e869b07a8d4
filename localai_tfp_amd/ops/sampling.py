"""Batched token sampling (GPU: csrc/kernels/sampling.hip; CPU: PyTorch reference).

Sampling parameters follow llama.cpp's chain as driven by the reference worker
(grpc-server.cpp:690-964 `launch_slot_with_data`: temperature, top_k, top_p, min_p, typical_p,
repeat/presence/frequency penalties over the last `repeat_last_n` tokens, logit_bias, mirostat,
seed). Penalties and logit bias are passed sparsely per row as unique (token, count, bias).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from .. import _native as N

SAMPLE_DTYPE = np.dtype([
    ("temperature", np.float32), ("top_k", np.int32), ("top_p", np.float32), ("min_p", np.float32),
    ("typical_p", np.float32), ("mirostat_tau", np.float32), ("repeat_penalty", np.float32),
    ("presence_penalty", np.float32), ("frequency_penalty", np.float32), ("pen_offset", np.int32),
    ("pen_count", np.int32), ("pend", np.int32), ("seed", np.uint64)], align=True)


@dataclass
class SamplingParams:
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.95
    min_p: float = 0.05
    typical_p: float = 1.0
    repeat_penalty: float = 1.0
    repeat_last_n: int = 64
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    mirostat: int = 0
    mirostat_tau: float = 5.0
    mirostat_eta: float = 0.1
    seed: int = -1
    logit_bias: dict = field(default_factory=dict)
    ignore_eos: bool = False
    n_probs: int = 0

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0 or self.top_k == 1


def _check_size():
    sz = N.kernels().mxk_sample_params_size()
    if sz != SAMPLE_DTYPE.itemsize:
        raise N.NativeError(f"SampleParams ABI mismatch: C {sz} B vs numpy {SAMPLE_DTYPE.itemsize} B")


class SamplerBatch:
    """Host-side packing of per-row parameters + sparse penalty lists into device buffers."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._checked = False

    @staticmethod
    def _record(p: SamplingParams):
        """The request-constant part of a row (cached on the params object: a request's sampling settings do
        not change while it runs) and its base seed."""
        c = p.__dict__.get("_mx_rec")
        if c is None:
            r = np.zeros(1, SAMPLE_DTYPE)
            r["pend"] = -1
            r["temperature"] = 0.0 if p.greedy else p.temperature
            r["top_k"], r["top_p"], r["min_p"], r["typical_p"] = p.top_k, p.top_p, p.min_p, p.typical_p
            r["repeat_penalty"] = p.repeat_penalty
            r["presence_penalty"], r["frequency_penalty"] = p.presence_penalty, p.frequency_penalty
            seed = p.seed if p.seed is not None and p.seed >= 0 else 0x5DEECE66D
            simple = not (p.mirostat == 2 or p.repeat_penalty != 1.0 or p.presence_penalty or p.frequency_penalty
                          or p.logit_bias)
            # the record as bytes: the batch array is one b"".join (np.concatenate of 128 one-row structured
            # arrays took ~3 ms of host time per step)
            c = p.__dict__["_mx_rec"] = (r.tobytes(), int(seed) & 0xFFFFFFFFFFFFFFFF, simple)
        return c

    def pack(self, params: list[SamplingParams], histories: list[list[int]], steps: list[int],
             mirostat_mu: list[float] | None = None, pend: list[int] | None = None):
        """Vectorised over rows: cached per-request records, seeds advanced per step in numpy; only rows with
        penalties / logit bias / mirostat are visited in Python. pend[i] >= 0: row i's previous token is still
        in flight (overlap pipeline) at that index of the device token tensor passed to sample(); its history
        lacks that token, so the penalty window takes one token fewer here and the kernel counts the
        pending one."""
        B = len(params)
        recs = [self._record(p) for p in params]
        arr = np.frombuffer(bytearray(b"".join([r[0] for r in recs])), SAMPLE_DTYPE) if B else np.zeros(0, SAMPLE_DTYPE)
        base = np.fromiter((r[1] for r in recs), np.uint64, B)
        st = np.asarray(steps, np.uint64)
        with np.errstate(over="ignore"):
            arr["seed"] = base * np.uint64(1000003) + st
        toks, cnts, bias = [], [], []
        for i in (i for i, r in enumerate(recs) if not r[2]):
            p = params[i]
            arr[i]["mirostat_tau"] = (mirostat_mu[i] if mirostat_mu else 2 * p.mirostat_tau) if p.mirostat == 2 else 0.0
            d: dict[int, list] = {}
            pi = pend[i] if pend is not None else -1
            arr[i]["pend"] = pi
            if p.repeat_penalty != 1.0 or p.presence_penalty or p.frequency_penalty:
                n = p.repeat_last_n - (1 if pi >= 0 else 0)
                hist = histories[i][-n:] if n > 0 else ([] if p.repeat_last_n > 0 else histories[i])
                for t in hist:
                    e = d.setdefault(int(t), [0, 0.0])
                    e[0] += 1
            for t, b in (p.logit_bias or {}).items():
                e = d.setdefault(int(t), [0, 0.0])
                e[1] += float(b)
            arr[i]["pen_offset"] = len(toks)
            arr[i]["pen_count"] = len(d)
            for t, (c, b) in d.items():
                toks.append(t)
                cnts.append(c)
                bias.append(b)
        return arr, np.asarray(toks or [0], np.int32), np.asarray(cnts or [0], np.int32), np.asarray(bias or [0.0], np.float32)

    def _stage(self, dev, parts: list[np.ndarray]) -> list[torch.Tensor]:
        """Byte arrays -> device views (16-B aligned) through ONE copy from a pinned ring whose slots
        are reused only after the copy that read them ran (utils/pinned.py): a pageable H2D copy
        would make the host wait for the stream, stalling the next step's launch."""
        from ..utils.pinned import PinnedRing
        offs, n = [], 0
        for a in parts:
            offs.append(n)
            n += -(-a.size // 16) * 16
        ring = getattr(self, "_pin", None)
        if ring is None:
            ring = self._pin = PinnedRing(4, max(n, 1 << 20), dev)
        img = np.zeros(n, np.uint8)
        for o, a in zip(offs, parts):
            img[o:o + a.size] = a
        d = ring.stage(img)
        return [d[o:o + a.size] for o, a in zip(offs, parts)]

    def sample(self, logits: torch.Tensor, params: list[SamplingParams], histories: list[list[int]],
               steps: list[int], allow_mask: torch.Tensor | None = None, mirostat_mu=None,
               pend_tok: torch.Tensor | None = None, pend: list[int] | None = None):
        """logits fp32 [B, V] (modified in place) -> (tokens int32 [B], logprobs fp32 [B]) on device.
        pend_tok / pend: the previous step's token tensor (still in flight) and, per row, the index of that
        row's pending token in it or -1 (penalties in the overlap pipeline, see pack)."""
        B, V = logits.shape
        if pend is not None and (pend_tok is None or all(i < 0 for i in pend)):
            pend = None
        if not logits.is_cuda:
            if pend is not None:  # CPU tensors are already computed: append the pending token to the history
                pt = pend_tok.tolist()
                histories = [h + [int(pt[i])] if i >= 0 else h for h, i in zip(histories, pend)]
            return sample_ref(logits, params, histories, steps, allow_mask)
        if not self._checked:
            _check_size()
            self._checked = True
        if all(p.greedy and not p.logit_bias and p.repeat_penalty == 1.0 and not p.presence_penalty
               and not p.frequency_penalty for p in params) and allow_mask is None:
            tok = torch.empty(B, dtype=torch.int32, device=logits.device)
            N.kcall("mxk_argmax", logits.data_ptr(), logits.stride(0), B, V, tok.data_ptr(), N.stream_ptr())
            return tok, None
        arr, toks, cnts, bias = self.pack(params, histories, steps, mirostat_mu, pend)
        dev = logits.device
        ptok = None
        if pend is not None:
            ptok = pend_tok if (pend_tok.dtype == torch.int32 and pend_tok.is_contiguous()) else \
                pend_tok.to(torch.int32).contiguous()
        pbuf, t_t, c_t, b_t = self._stage(dev, [arr.view(np.uint8), toks.view(np.uint8), cnts.view(np.uint8),
                                                bias.view(np.uint8)])
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lp = torch.empty(B, dtype=torch.float32, device=dev)
        S = self._split_slices(params, B, V)
        if S:
            # small batch, top-k on: the vocabulary split over B x S workgroups instead of one CU per row
            cv, ci, cn, sz = self._split_scratch(dev, B, S)
            has_pen = bool(arr["pen_count"].any()) or bool((arr["pend"] >= 0).any())
            N.kcall("mxk_sample_topk_split", logits.data_ptr(), logits.stride(0), B, V, pbuf.data_ptr(),
                    int(has_pen), t_t.data_ptr(), c_t.data_ptr(), b_t.data_ptr(),
                    N.ptr(allow_mask), allow_mask.stride(0) if allow_mask is not None else 0, S, cv.data_ptr(),
                    ci.data_ptr(), cn.data_ptr(), sz.data_ptr(), tok.data_ptr(), lp.data_ptr(), N.ptr(ptok),
                    N.stream_ptr())
            return tok, lp
        N.kcall("mxk_sample", logits.data_ptr(), logits.stride(0), B, V, pbuf.data_ptr(), t_t.data_ptr(),
                c_t.data_ptr(), b_t.data_ptr(), N.ptr(allow_mask), allow_mask.stride(0) if allow_mask is not None else 0,
                tok.data_ptr(), lp.data_ptr(), N.ptr(ptok), N.stream_ptr())
        return tok, lp

    # the split top-k sampler (B x S register-resident slices + a per-row merge) serves every batch size whose
    # rows all have top-k on (the reference default, top_k 40) or are greedy; MX_SPLIT_SAMPLER_MAX_B caps it
    SPLIT_MAX_B = int(__import__("os").environ.get("MX_SPLIT_SAMPLER_MAX_B", str(1 << 20)))
    TOPK_CAP = 64
    SLICE = 8192   # vocabulary entries per slice (sampling.hip tk_nv() x 256, read from the library on first use)
    CAPS = 128     # candidates per slice (TK_CAPS)

    def _split_slices(self, params, B: int, V: int = 128256) -> int:
        """Slices per row for the split top-k sampler, or 0 where it does not apply (top-k off or above the
        cap, typical-p / mirostat rows, a vocabulary beyond 64 slices)."""
        if B > self.SPLIT_MAX_B:
            return 0
        if not getattr(self, "_slice_checked", False) and N.have_kernels():
            got = N.kernels().mxk_sample_topk_slice()  # MX_TK_NV selects 4096- or 8192-entry slices
            if got not in (4096, 8192):
                raise N.NativeError(f"split sampler: unexpected slice size {got} from the library")
            self.SLICE = got
            caps = N.kernels().mxk_sample_topk_caps()  # scratch below is sized from it: must match TK_CAPS
            if caps != self.CAPS:
                raise N.NativeError(f"split sampler: library TK_CAPS {caps} != host scratch capacity {self.CAPS}")
            self._slice_checked = True
        S = -(-V // self.SLICE)
        if S > 64:
            return 0
        for p in params:
            if p.greedy:
                continue
            if not (0 < p.top_k <= self.TOPK_CAP) or (0 < p.typical_p < 1) or p.mirostat == 2:
                return 0
        return S

    def _split_scratch(self, dev, B: int, S: int):
        key = (str(dev), B, S)
        c = getattr(self, "_scratch", None)
        if c is None or c[0] != key:
            cv = torch.empty(B * S * self.CAPS, dtype=torch.float32, device=dev)
            ci = torch.empty(B * S * self.CAPS, dtype=torch.int32, device=dev)
            cn = torch.empty(B * S, dtype=torch.int32, device=dev)
            sz = torch.empty(B * S * 2, dtype=torch.float32, device=dev)  # per-slice (max, sum exp)
            c = self._scratch = (key, cv, ci, cn, sz)
        return c[1], c[2], c[3], c[4]


def sample_ref(logits: torch.Tensor, params, histories, steps, allow_mask=None):
    """PyTorch reference of the same chain (CPU engine path)."""
    B, V = logits.shape
    toks = torch.empty(B, dtype=torch.int32)
    lps = torch.empty(B, dtype=torch.float32)
    for i, p in enumerate(params):
        x = logits[i].float().clone()
        counts: dict[int, int] = {}
        if p.repeat_penalty != 1.0 or p.presence_penalty or p.frequency_penalty:
            hist = histories[i][-p.repeat_last_n:] if p.repeat_last_n > 0 else histories[i]
            for t in hist:
                counts[int(t)] = counts.get(int(t), 0) + 1
        for t, c in counts.items():
            if 0 <= t < V:
                v = x[t]
                if p.repeat_penalty != 1.0:
                    v = v / p.repeat_penalty if v > 0 else v * p.repeat_penalty
                x[t] = v - p.frequency_penalty * c - p.presence_penalty
        for t, b in (p.logit_bias or {}).items():
            if 0 <= int(t) < V:
                x[int(t)] += float(b)
        if allow_mask is not None:
            m = allow_mask[i]
            bits = ((m[:, None] >> torch.arange(32, dtype=torch.int32)) & 1).reshape(-1)[:V].bool()
            x = torch.where(bits, x, torch.full_like(x, float("-inf")))
        if p.greedy:
            t = int(torch.argmax(x))
            toks[i] = t
            lps[i] = 0.0
            continue
        x = x / p.temperature
        keep = torch.isfinite(x)
        if p.top_k > 0 and p.top_k < V:
            kth = torch.topk(x, p.top_k).values[-1]
            keep &= x >= kth
        mx = x.max()
        if p.min_p > 0:
            keep &= x >= mx + np.log(p.min_p)
        if 0 < p.top_p < 1:
            xs = torch.where(keep, x, torch.full_like(x, float("-inf")))
            pr = torch.softmax(xs, -1)
            sp, si = torch.sort(pr, descending=True)
            cum = torch.cumsum(sp, 0)
            n_keep = int((cum < p.top_p).sum()) + 1
            k2 = torch.zeros_like(keep)
            k2[si[:n_keep]] = True
            keep &= k2
        if p.mirostat == 2:
            xs = torch.where(keep, x, torch.full_like(x, float("-inf")))
            lp = torch.log_softmax(xs, -1) / np.log(2)
            keep &= (-lp <= 2 * p.mirostat_tau) | (x == mx)
        xs = torch.where(keep, x, torch.full_like(x, float("-inf")))
        pr = torch.softmax(xs, -1)
        g = torch.Generator().manual_seed(((p.seed if p.seed >= 0 else 0x5DEECE66D) * 1000003 + steps[i]) & 0x7FFFFFFF)
        t = int(torch.multinomial(pr, 1, generator=g))
        toks[i] = t
        lps[i] = float(torch.log(pr[t].clamp_min(1e-30)))
    return toks, lps
