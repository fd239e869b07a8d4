"""Whisper speech recognition (encoder-decoder transformer) — the reference's whisper.cpp backend
(backend/go/transcribe/whisper/whisper.go:28-105; SURVEY §2 N8, BASELINE config #4) and the
faster-whisper backend (backend/python/faster-whisper/backend.py:26-62).

MI355X design:
* log-mel front end as two fp32 GEMMs on the matrix cores: framed audio x (Hann-windowed DFT basis)
  -> power spectrum -> x mel filterbank; no FFT library, one pass over the padded signal.
* conv1d stem as H = 1 convolutions on the implicit-GEMM MFMA kernel (ops/conv.py, bias + GELU fused).
* transformer blocks: hipBLASLt GEMMs with the residual add fused as beta = 1 into an fp32
  residual stream; LayerNorm from norm.hip; attention on the fused MFMA flash kernel
  (attention_dense.hip) — bidirectional in the encoder, cross-attention to the audio states and
  causal self-attention reading a fixed-capacity KV cache in place in the decoder.
* the per-token decoder step (B sequences, fixed capacity) is captured once into a hipGraph and
  replayed; only the token/position tensors change between replays.
* decoding follows whisper's published algorithm: SOT sequence, language detection, timestamp
  rules, greedy/temperature fallback (compression ratio / avg log-prob), beam search, segments
  from timestamp pairs with seek by the last timestamp.

Weights: whisper.cpp ggml files (formats/ggml_whisper.py), Hugging Face safetensors, or
random-init (`synthetic:whisper-*`).
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, replace

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import core as K
from ..ops import conv as CV
from ..ops.dense import Dense, model_dtype, to_dev

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160
CHUNK = 30
N_SAMPLES = CHUNK * SAMPLE_RATE
N_FRAMES = N_SAMPLES // HOP  # 3000
TS_STEP = 0.02               # seconds per timestamp token (2 mel frames)


@dataclass
class WhisperConfig:
    n_vocab: int = 51865
    n_audio_ctx: int = 1500
    n_audio_state: int = 512
    n_audio_head: int = 8
    n_audio_layer: int = 6
    n_text_ctx: int = 448
    n_text_state: int = 512
    n_text_head: int = 8
    n_text_layer: int = 6
    n_mels: int = 80
    name: str = "whisper-base"


WHISPER_TINY = WhisperConfig(n_audio_state=384, n_audio_head=6, n_audio_layer=4, n_text_state=384, n_text_head=6,
                             n_text_layer=4, name="whisper-tiny")
WHISPER_BASE = WhisperConfig()
WHISPER_SMALL = WhisperConfig(n_audio_state=768, n_audio_head=12, n_audio_layer=12, n_text_state=768,
                              n_text_head=12, n_text_layer=12, name="whisper-small")
WHISPER_MEDIUM = WhisperConfig(n_audio_state=1024, n_audio_head=16, n_audio_layer=24, n_text_state=1024,
                               n_text_head=16, n_text_layer=24, name="whisper-medium")
WHISPER_LARGE_V3 = WhisperConfig(n_vocab=51866, n_audio_state=1280, n_audio_head=20, n_audio_layer=32,
                                 n_text_state=1280, n_text_head=20, n_text_layer=32, n_mels=128,
                                 name="whisper-large-v3")
WHISPER_TEST = WhisperConfig(n_audio_state=64, n_audio_head=2, n_audio_layer=2, n_text_state=64, n_text_head=2,
                             n_text_layer=2, name="whisper-test")
PRESETS = {c.name: c for c in (WHISPER_TINY, WHISPER_BASE, WHISPER_SMALL, WHISPER_MEDIUM, WHISPER_LARGE_V3,
                               WHISPER_TEST)}


# ------------------------------------------------------------------------------------------------
# front end

def mel_filterbank(sr: int = SAMPLE_RATE, n_fft: int = N_FFT, n_mels: int = 80) -> np.ndarray:
    """Slaney-scale, area-normalised triangular filters [n_mels, n_fft//2 + 1] (the filterbank
    Whisper checkpoints were trained with; ggml files carry their own copy)."""
    f_sp, min_log_hz, min_log_mel, logstep = 200.0 / 3, 1000.0, 15.0, math.log(6.4) / 27.0

    def hz_to_mel(f):
        f = np.asarray(f, np.float64)
        m = f / f_sp
        return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, m)

    def mel_to_hz(m):
        m = np.asarray(m, np.float64)
        return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)

    fft_f = np.linspace(0, sr / 2, n_fft // 2 + 1)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(sr / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_f[None, :]
    w = np.zeros((n_mels, len(fft_f)))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


class LogMel:
    """Whisper log-mel spectrogram as GEMMs: frames [T, 400] @ [400, 2*201] (windowed cos | -sin)
    -> |X|^2 -> @ filters^T -> log10, clamp to (max - 8), (x + 4) / 4."""

    def __init__(self, filters: np.ndarray, device):
        self.device = torch.device(device)
        n = np.arange(N_FFT)
        win = 0.5 - 0.5 * np.cos(2 * np.pi * n / N_FFT)  # periodic Hann
        k = np.arange(N_FFT // 2 + 1)
        ang = 2 * np.pi * np.outer(n, k) / N_FFT
        basis = np.concatenate([win[:, None] * np.cos(ang), -win[:, None] * np.sin(ang)], 1)
        self.basis = torch.from_numpy(basis.astype(np.float32)).to(self.device)
        self.filt_t = torch.from_numpy(np.ascontiguousarray(filters.T, np.float32)).to(self.device)
        self.nf = N_FFT // 2 + 1

    def __call__(self, audio: torch.Tensor) -> torch.Tensor:
        """audio fp32 [N] (already padded by N_SAMPLES zeros) -> [n_mels, N // HOP]."""
        x = F.pad(audio.view(1, 1, -1), (N_FFT // 2, N_FFT // 2), mode="reflect").view(-1)
        frames = x.unfold(0, N_FFT, HOP)[:-1]  # torch.stft(center=True) frames minus the last
        spec = frames @ self.basis
        power = spec[:, :self.nf].square() + spec[:, self.nf:].square()
        mel = power @ self.filt_t
        log = mel.clamp_min(1e-10).log10()
        log = torch.maximum(log, log.max() - 8.0)
        return ((log + 4.0) / 4.0).t().contiguous()


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2))
    t = np.arange(length)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], 1).astype(np.float32)


# ------------------------------------------------------------------------------------------------
# weights

def hf_to_openai_name(n: str) -> str | None:
    """Hugging Face `WhisperForConditionalGeneration` names -> OpenAI / whisper.cpp names."""
    if n.startswith("model."):
        n = n[6:]
    if n in ("proj_out.weight",):
        return None
    rep = [("encoder.layers.", "encoder.blocks."), ("decoder.layers.", "decoder.blocks."),
           ("self_attn_layer_norm", "attn_ln"), ("encoder_attn_layer_norm", "cross_attn_ln"),
           ("final_layer_norm", "mlp_ln"), ("self_attn.", "attn."), ("encoder_attn.", "cross_attn."),
           ("q_proj", "query"), ("k_proj", "key"), ("v_proj", "value"), ("out_proj", "out"),
           ("fc1", "mlp.0"), ("fc2", "mlp.2"), ("encoder.embed_positions.weight", "encoder.positional_embedding"),
           ("decoder.embed_positions.weight", "decoder.positional_embedding"),
           ("decoder.embed_tokens", "decoder.token_embedding"), ("encoder.layer_norm", "encoder.ln_post"),
           ("decoder.layer_norm", "decoder.ln")]
    for a, b in rep:
        n = n.replace(a, b)
    return n


def synthetic_whisper(cfg: WhisperConfig, seed: int = 0):
    """Random-init tensors with OpenAI names (for tests / benchmarks; no checkpoint download)."""
    rng = np.random.default_rng(seed)
    da, dt = cfg.n_audio_state, cfg.n_text_state
    shapes = {"encoder.conv1.weight": (da, cfg.n_mels, 3), "encoder.conv1.bias": (da,),
              "encoder.conv2.weight": (da, da, 3), "encoder.conv2.bias": (da,),
              "encoder.ln_post.weight": (da,), "encoder.ln_post.bias": (da,),
              "decoder.token_embedding.weight": (cfg.n_vocab, dt), "decoder.positional_embedding": (cfg.n_text_ctx, dt),
              "decoder.ln.weight": (dt,), "decoder.ln.bias": (dt,)}

    def block(p, d, cross):
        for a in ("attn",) + (("cross_attn",) if cross else ()):
            for x in ("query", "key", "value", "out"):
                shapes[f"{p}{a}.{x}.weight"] = (d, d)
                if x != "key":
                    shapes[f"{p}{a}.{x}.bias"] = (d,)
            shapes[f"{p}{a}_ln.weight"] = (d,)
            shapes[f"{p}{a}_ln.bias"] = (d,)
        shapes.update({f"{p}mlp.0.weight": (4 * d, d), f"{p}mlp.0.bias": (4 * d,), f"{p}mlp.2.weight": (d, 4 * d),
                       f"{p}mlp.2.bias": (d,), f"{p}mlp_ln.weight": (d,), f"{p}mlp_ln.bias": (d,)})
    for i in range(cfg.n_audio_layer):
        block(f"encoder.blocks.{i}.", da, False)
    for i in range(cfg.n_text_layer):
        block(f"decoder.blocks.{i}.", dt, True)
    out = {"encoder.positional_embedding": sinusoids(cfg.n_audio_ctx, da)}
    for n, s in shapes.items():
        if n.endswith("ln.weight") or n.endswith("ln_post.weight"):
            out[n] = np.ones(s, np.float32)
        elif n.endswith(".bias"):
            out[n] = np.zeros(s, np.float32)
        else:
            fan_in = s[1] * (s[2] if len(s) > 2 else 1) if len(s) > 1 else 1
            std = 0.02 if "embedding" in n else 1.0 / math.sqrt(fan_in)
            out[n] = (rng.standard_normal(s) * std).astype(np.float32)
    return out


# ------------------------------------------------------------------------------------------------
# model

class _Block:
    def __init__(self, get, p: str, dev, dt, cross: bool):
        def ln(n):
            return (to_dev(get(f"{p}{n}.weight"), dev, torch.float32), to_dev(get(f"{p}{n}.bias"), dev, torch.float32))

        def qkv(a):
            w = [get(f"{p}{a}.{x}.weight") for x in ("query", "key", "value")]
            d = w[0].shape[0]
            kb = get(f"{p}{a}.key.bias")
            b = [get(f"{p}{a}.query.bias"), kb if kb is not None else np.zeros(d, np.float32), get(f"{p}{a}.value.bias")]
            return w, b
        w, b = qkv("attn")
        self.attn_ln = ln("attn_ln")
        self.qkv = Dense(np.concatenate(w, 0), np.concatenate(b, 0), dev, dt)
        self.out = Dense(get(f"{p}attn.out.weight"), get(f"{p}attn.out.bias"), dev, dt)
        if cross:
            w, b = qkv("cross_attn")
            self.cross_ln = ln("cross_attn_ln")
            self.cq = Dense(w[0], b[0], dev, dt)
            self.ckv = Dense(np.concatenate(w[1:], 0), np.concatenate(b[1:], 0), dev, dt)
            self.cout = Dense(get(f"{p}cross_attn.out.weight"), get(f"{p}cross_attn.out.bias"), dev, dt)
        self.mlp_ln = ln("mlp_ln")
        self.fc1 = Dense(get(f"{p}mlp.0.weight"), get(f"{p}mlp.0.bias"), dev, dt)
        self.fc2 = Dense(get(f"{p}mlp.2.weight"), get(f"{p}mlp.2.bias"), dev, dt)


class WhisperModel:
    def __init__(self, cfg: WhisperConfig, get, device="cpu", mel_filters: np.ndarray | None = None):
        """get(name) -> float32 numpy array (OpenAI tensor names) or None."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dt = model_dtype(device)
        dev = self.device
        self.mel = LogMel(mel_filters if mel_filters is not None else mel_filterbank(n_mels=cfg.n_mels), dev)
        # conv1d stem as H = 1 2-D convs on the implicit-GEMM MFMA kernel (ops/conv.py, GELU fused):
        # weights [out, in, 3] -> [out, in, 1, 3], packed once
        self.stem = []
        for n in ("conv1", "conv2"):
            w = to_dev(get(f"encoder.{n}.weight"), dev, torch.float32)[:, :, None, :]
            b = to_dev(get(f"encoder.{n}.bias"), dev, torch.float32)
            self.stem.append((w.to(dt), b, CV.pack_weight(w, dt) if dev.type == "cuda" else None))
        pe = get("encoder.positional_embedding")
        self.enc_pos = to_dev(pe if pe is not None else sinusoids(cfg.n_audio_ctx, cfg.n_audio_state), dev,
                              torch.float32)
        self.enc = [_Block(get, f"encoder.blocks.{i}.", dev, dt, False) for i in range(cfg.n_audio_layer)]
        self.ln_post = (to_dev(get("encoder.ln_post.weight"), dev, torch.float32),
                        to_dev(get("encoder.ln_post.bias"), dev, torch.float32))
        self.tok_emb = to_dev(get("decoder.token_embedding.weight"), dev, dt)
        self.dec_pos = to_dev(get("decoder.positional_embedding"), dev, torch.float32)
        self.dec = [_Block(get, f"decoder.blocks.{i}.", dev, dt, True) for i in range(cfg.n_text_layer)]
        self.ln_dec = (to_dev(get("decoder.ln.weight"), dev, torch.float32),
                       to_dev(get("decoder.ln.bias"), dev, torch.float32))
        self.eps = 1e-5
        self._graphs: dict[int, tuple] = {}

    # -------------------------------------------------------------- helpers
    def _ln(self, x, wb):
        out = torch.empty(x.shape, dtype=self.dtype, device=x.device)
        K.layernorm(x, wb[0], wb[1], self.eps, out)
        return out

    def log_mel(self, audio: np.ndarray) -> torch.Tensor:
        """float32 PCM (16 kHz) -> [n_mels, len//HOP + N_FRAMES] (audio padded with 30 s of zeros)."""
        a = torch.from_numpy(np.concatenate([np.asarray(audio, np.float32), np.zeros(N_SAMPLES, np.float32)]))
        return self.mel(a.to(self.device))

    # -------------------------------------------------------------- encoder
    @torch.no_grad()
    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        """mel [B, n_mels, 3000] fp32 -> audio states [B * n_audio_ctx, d] (model dtype)."""
        cfg = self.cfg
        B, C, T = mel.shape
        d = cfg.n_audio_state
        # [B, T, C] rows viewed as NCHW-shaped channels_last [B, C, 1, T]
        x = mel.transpose(1, 2).to(self.dtype).contiguous()[:, None].permute(0, 3, 1, 2)
        (w1, b1, p1), (w2, b2, p2) = self.stem
        y = CV.conv2d(x, weight=w1, bias=b1, stride=1, pad=(0, 1, 0, 1), act="gelu", packed=p1)
        y = CV.conv2d(y, weight=w2, bias=b2, stride=2, pad=(0, 1, 0, 1), act="gelu", packed=p2)
        T2 = y.shape[-1]
        h = y.permute(0, 2, 3, 1).reshape(B, T2, d).float()
        h = (h + self.enc_pos[:T2]).reshape(B * T2, d).contiguous()
        H = cfg.n_audio_head
        hd = d // H
        attn = torch.empty(B * T2, d, dtype=self.dtype, device=self.device)
        for blk in self.enc:
            qkv = blk.qkv(self._ln(h, blk.attn_ln))
            K.attn_dense(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], attn, B, T2, T2, H, H, hd, 1.0 / math.sqrt(hd))
            blk.out.acc(attn, h)
            blk.fc2.acc(blk.fc1(self._ln(h, blk.mlp_ln), act="gelu"), h)
        return self._ln(h, self.ln_post)

    # -------------------------------------------------------------- decoder
    def new_state(self, B: int) -> "DecoderState":
        return DecoderState(self, B)

    def _dec_layers(self, st: "DecoderState", x: torch.Tensor, rows: torch.Tensor, T: int, Sk: int,
                    klen: torch.Tensor | None, causal: bool):
        cfg = self.cfg
        d = cfg.n_text_state
        H = cfg.n_text_head
        hd = d // H
        B = st.B
        sc = 1.0 / math.sqrt(hd)
        attn = torch.empty(B * T, d, dtype=self.dtype, device=self.device)
        for i, blk in enumerate(self.dec):
            qkv = blk.qkv(self._ln(x, blk.attn_ln))
            st.k[i].index_copy_(0, rows, qkv[:, d:2 * d])
            st.v[i].index_copy_(0, rows, qkv[:, 2 * d:])
            K.attn_dense(qkv[:, :d], st.k[i], st.v[i], attn, B, T, Sk, H, H, hd, sc, causal, klen=klen,
                         kv_rows=st.cap)
            blk.out.acc(attn, x)
            q = blk.cq(self._ln(x, blk.cross_ln))
            K.attn_dense(q, st.ck[i], st.cv[i], attn, B, T, cfg.n_audio_ctx, H, H, hd, sc)
            blk.cout.acc(attn, x)
            blk.fc2.acc(blk.fc1(self._ln(x, blk.mlp_ln), act="gelu"), x)
        h = self._ln(x, self.ln_dec)
        if h.dtype == torch.float32:
            return h @ self.tok_emb.t()
        logits = torch.empty(h.shape[0], cfg.n_vocab, dtype=torch.float32, device=self.device)
        from ..ops.linear import _fp32_out_ok
        if _fp32_out_ok(h.dtype):
            torch.mm(h, self.tok_emb.t(), out_dtype=torch.float32, out=logits)
        else:
            logits.copy_(h @ self.tok_emb.t())
        return logits

    @torch.no_grad()
    def decode_prefix(self, st: "DecoderState", tokens: list[list[int]]) -> torch.Tensor:
        """Run B equal-length token prefixes from position st.pos; -> logits of the last position [B, V]."""
        B, T = len(tokens), len(tokens[0])
        assert B == st.B and st.pos + T <= st.cap
        pos0 = st.pos
        tok = torch.tensor(tokens, dtype=torch.long, device=self.device).view(-1)
        pos = torch.arange(pos0, pos0 + T, device=self.device).repeat(B)
        rows = (torch.arange(B, device=self.device).repeat_interleave(T) * st.cap + pos).contiguous()
        x = (self.tok_emb[tok].float() + self.dec_pos[pos]).contiguous()
        logits = self._dec_layers(st, x, rows, T, pos0 + T, None, True)
        st.pos += T
        return logits.view(B, T, -1)[:, -1]

    @torch.no_grad()
    def decode_step(self, st: "DecoderState", tokens: torch.Tensor) -> torch.Tensor:
        """One token per sequence at position st.pos (tokens: long [B] on device) -> logits [B, V].
        On GPU the step is captured into a hipGraph per (state) and replayed."""
        assert st.pos < st.cap
        if self.device.type != "cuda" or not st.use_graph:
            st.tok.copy_(tokens)
            st.set_pos(st.pos)
            out = self._step_eager(st)
            st.pos += 1
            return out
        st.tok.copy_(tokens)
        st.set_pos(st.pos)
        if st.graph is None:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._step_eager(st)  # warm up (allocator, hipBLASLt heuristics)
            torch.cuda.current_stream(self.device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st.logits = self._step_eager(st)
            st.graph = g
        st.graph.replay()
        st.pos += 1
        return st.logits

    def _step_eager(self, st: "DecoderState"):
        x = (self.tok_emb[st.tok].float() + self.dec_pos[st.posv]).contiguous()
        return self._dec_layers(st, x, st.rows, 1, st.cap, st.klen, False)


class DecoderState:
    """Per-batch decoder buffers: self-attention KV cache [B, n_text_ctx, d] per layer (fixed capacity,
    read in place by attention_dense.hip), cross-attention K/V [B, n_audio_ctx, d], static step inputs
    for hipGraph replay."""

    def __init__(self, m: WhisperModel, B: int):
        cfg = m.cfg
        d = cfg.n_text_state
        dev = m.device
        self.m = m
        self.B = B
        self.cap = cfg.n_text_ctx
        self.k = [torch.zeros(B * self.cap, d, dtype=m.dtype, device=dev) for _ in m.dec]
        self.v = [torch.zeros(B * self.cap, d, dtype=m.dtype, device=dev) for _ in m.dec]
        self.ck: list[torch.Tensor] = []
        self.cv: list[torch.Tensor] = []
        self.pos = 0
        self.tok = torch.zeros(B, dtype=torch.long, device=dev)
        self.posv = torch.zeros(B, dtype=torch.long, device=dev)
        self.rows = torch.zeros(B, dtype=torch.long, device=dev)
        self.klen = torch.zeros(B, dtype=torch.int32, device=dev)
        self._base = torch.arange(B, device=dev) * self.cap
        self.graph = None
        self.logits = None
        self.use_graph = True

    def set_pos(self, p: int):
        self.posv.fill_(p)
        torch.add(self._base, p, out=self.rows)
        self.klen.fill_(p + 1)

    @torch.no_grad()
    def set_audio(self, xa: torch.Tensor):
        """xa [B * n_audio_ctx, d] -> cross K/V for every decoder layer (computed once per window)."""
        d = self.m.cfg.n_text_state
        if not self.ck:
            self.ck = [torch.empty(xa.shape[0], d, dtype=self.m.dtype, device=xa.device) for _ in self.m.dec]
            self.cv = [torch.empty(xa.shape[0], d, dtype=self.m.dtype, device=xa.device) for _ in self.m.dec]
        for i, blk in enumerate(self.m.dec):
            kv = blk.ckv(xa)
            self.ck[i].copy_(kv[:, :d])
            self.cv[i].copy_(kv[:, d:])
        self.pos = 0

    def reorder(self, idx: torch.Tensor):
        """Beam search: gather sequences' self-attention caches by parent index."""
        for t in self.k + self.v:
            t.copy_(t.view(self.B, self.cap, -1)[idx].view(self.B * self.cap, -1))


# ------------------------------------------------------------------------------------------------
# transcription

@dataclass
class DecodeOptions:
    language: str | None = None  # None / "" / "auto" -> detect
    task: str = "transcribe"
    temperatures: tuple = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0)
    beam_size: int = 0           # 0 -> greedy
    sample_len: int = 224
    compression_ratio_threshold: float = 2.4
    logprob_threshold: float = -1.0
    no_speech_threshold: float = 0.6
    timestamps: bool = True
    max_initial_timestamp: float = 1.0
    condition_on_previous_text: bool = False
    initial_prompt: str = ""
    seed: int = 0


@dataclass
class Segment:
    id: int
    start: float
    end: float
    text: str
    tokens: list


def compression_ratio(text: str) -> float:
    b = text.encode("utf-8")
    return len(b) / max(1, len(zlib.compress(b)))


class Transcriber:
    def __init__(self, model: WhisperModel, tok):
        self.m = model
        self.tok = tok
        self._states: dict[int, DecoderState] = {}
        t = tok
        self.suppress = [t.sot, t.translate, t.transcribe, t.solm, t.prev, t.nosp] + \
            list(range(t.lang0, t.lang0 + t.n_lang))
        self.suppress = [s for s in self.suppress if s < model.cfg.n_vocab]
        self.blank = [t.eot] + [i for i in (t.rank.get(b" "),) if i is not None]

    def _state(self, B: int) -> DecoderState:
        if B not in self._states:
            self._states[B] = self.m.new_state(B)
        return self._states[B]

    @torch.no_grad()
    def detect_language(self, xa: torch.Tensor) -> str:
        t = self.tok
        if not t.multilingual:
            return "en"
        st = self._state(1)
        st.set_audio(xa)
        logits = self.m.decode_prefix(st, [[t.sot]])[0].float().cpu().numpy()
        lang = logits[t.lang0: t.lang0 + t.n_lang]
        return t.language_of(t.lang0 + int(np.argmax(lang)))

    def _apply_rules(self, logits: np.ndarray, sampled: list[int], opt: DecodeOptions, first: bool):
        t = self.tok
        tb = t.timestamp_begin
        logits[self.suppress] = -np.inf
        if first:
            logits[self.blank] = -np.inf
        if not opt.timestamps:
            logits[tb:] = -np.inf
            return logits
        logits[t.no_timestamps] = -np.inf
        last_ts = len(sampled) >= 1 and sampled[-1] >= tb
        pen_ts = len(sampled) < 2 or sampled[-2] >= tb
        if last_ts:
            if pen_ts:
                logits[tb:] = -np.inf
            else:
                logits[:t.eot] = -np.inf
        ts = [s for s in sampled if s >= tb]
        if ts:
            last = ts[-1] if (last_ts and not pen_ts) else ts[-1] + 1
            logits[tb:last] = -np.inf
        if not sampled:
            logits[:tb] = -np.inf
            logits[tb + int(round(opt.max_initial_timestamp / TS_STEP)) + 1:] = -np.inf
        lp = logits - _logsumexp(logits)
        if _logsumexp(lp[tb:]) > lp[:tb].max():
            logits[:tb] = -np.inf
        return logits

    def _decode_window(self, xa, prompt: list[int], opt: DecodeOptions, temperature: float, rng):
        """-> (tokens, avg_logprob, no_speech_prob)"""
        t = self.tok
        st = self._state(1)
        st.set_audio(xa)
        prefix = ([t.prev] + prompt[-(self.m.cfg.n_text_ctx // 2 - 1):] if prompt else []) + \
            t.sot_sequence(opt.language, opt.task) + ([] if opt.timestamps else [t.no_timestamps])
        logits_t = self.m.decode_prefix(st, [prefix])
        no_speech = 0.0
        sampled: list[int] = []
        sum_lp = 0.0
        limit = min(opt.sample_len, st.cap - len(prefix))
        tokv = torch.zeros(1, dtype=torch.long, device=self.m.device)
        for i in range(limit):
            logits = logits_t[0].float().cpu().numpy().astype(np.float64)
            if i == 0 and t.nosp < len(logits):
                p = np.exp(logits - _logsumexp(logits))
                no_speech = float(p[t.nosp])
            logits = self._apply_rules(logits, sampled, opt, i == 0)
            lp = logits - _logsumexp(logits)
            if temperature > 0:
                p = np.exp((logits - logits.max()) / temperature)
                p /= p.sum()
                nxt = int(rng.choice(len(p), p=p))
            else:
                nxt = int(np.argmax(logits))
            sum_lp += float(lp[nxt])
            if nxt == t.eot:
                break
            sampled.append(nxt)
            if st.pos >= st.cap:
                break
            tokv.fill_(nxt)
            logits_t = self.m.decode_step(st, tokv)
        return sampled, sum_lp / max(1, len(sampled) + 1), no_speech

    def _beam_window(self, xa, prompt: list[int], opt: DecodeOptions):
        """Beam search (faster-whisper default beam 5) with length-normalised scores."""
        t = self.tok
        W = opt.beam_size
        st = self._state(W)
        st.set_audio(xa.repeat(W, 1))
        prefix = ([t.prev] + prompt[-(self.m.cfg.n_text_ctx // 2 - 1):] if prompt else []) + \
            t.sot_sequence(opt.language, opt.task) + ([] if opt.timestamps else [t.no_timestamps])
        logits_t = self.m.decode_prefix(st, [prefix] * W)
        beams = [([], 0.0)]  # (tokens, sum logprob); start with a single live beam
        finished = []
        limit = min(opt.sample_len, st.cap - len(prefix))
        no_speech = 0.0
        for i in range(limit):
            L = logits_t.float().cpu().numpy().astype(np.float64)
            if i == 0 and t.nosp < L.shape[1]:
                p = np.exp(L[0] - _logsumexp(L[0]))
                no_speech = float(p[t.nosp])
            cands = []
            for bi, (toks, score) in enumerate(beams):
                lg = self._apply_rules(L[bi].copy(), toks, opt, i == 0)
                lp = lg - _logsumexp(lg)
                top = np.argpartition(-lp, W)[:W + 1]
                for tk in top:
                    if np.isfinite(lp[tk]):
                        cands.append((score + lp[tk], bi, int(tk)))
            cands.sort(key=lambda c: -c[0])
            new, parents = [], []
            for score, bi, tk in cands:
                toks = beams[bi][0] + [tk]
                if tk == t.eot:
                    if len(finished) < W:
                        finished.append((beams[bi][0], score))
                    continue
                new.append((toks, score))
                parents.append(bi)
                if len(new) == W:
                    break
            if len(finished) >= W or not new or st.pos >= st.cap:
                break
            while len(new) < W:  # keep the batch full (duplicates are harmless)
                new.append(new[-1])
                parents.append(parents[-1])
            st.reorder(torch.tensor(parents, device=self.m.device))
            beams = new
            logits_t = self.m.decode_step(st, torch.tensor([b[0][-1] for b in beams], device=self.m.device))
        pool = finished or beams
        best = max(pool, key=lambda b: b[1] / max(1, len(b[0]) + 1))
        return best[0], best[1] / max(1, len(best[0]) + 1), no_speech

    @torch.no_grad()
    def transcribe(self, audio: np.ndarray, opt: DecodeOptions | None = None) -> tuple[str, list[Segment], str]:
        """-> (text, segments, language)"""
        opt = opt or DecodeOptions()
        t = self.tok
        mel = self.m.log_mel(audio)
        content = max(0, len(audio) // HOP)
        seek = 0
        segments: list[Segment] = []
        all_tokens: list[int] = t.encode(" " + opt.initial_prompt.strip()) if opt.initial_prompt else []
        rng = np.random.default_rng(opt.seed)
        lang = opt.language if opt.language not in (None, "", "auto") else None
        while seek < content:
            win = min(N_FRAMES, content - seek)
            seg_mel = mel[:, seek:seek + N_FRAMES]
            if seg_mel.shape[1] < N_FRAMES:
                seg_mel = F.pad(seg_mel, (0, N_FRAMES - seg_mel.shape[1]))
            xa = self.m.encode(seg_mel[None])
            if lang is None:
                lang = self.detect_language(xa) if t.multilingual else "en"
            o = replace(opt, language=lang)
            prompt = all_tokens if (opt.condition_on_previous_text or (opt.initial_prompt and not segments)) else []
            toks, avg_lp, no_speech = [], -np.inf, 0.0
            for temp in opt.temperatures:
                if o.beam_size > 1 and temp == 0:
                    toks, avg_lp, no_speech = self._beam_window(xa, prompt, o)
                else:
                    toks, avg_lp, no_speech = self._decode_window(xa, prompt, o, temp, rng)
                text = t.decode([x for x in toks if x < t.eot])
                if compression_ratio(text) > opt.compression_ratio_threshold or avg_lp < opt.logprob_threshold:
                    if no_speech > opt.no_speech_threshold:
                        break
                    continue
                break
            t_off = seek * HOP / SAMPLE_RATE
            if no_speech > opt.no_speech_threshold and avg_lp < opt.logprob_threshold:
                seek += win
                continue
            seek += self._segments(toks, t_off, win, segments)
            all_tokens.extend(x for x in toks if x < t.eot)
        text = "".join(s.text for s in segments)
        return text, segments, lang or "en"

    def _segments(self, toks: list[int], t_off: float, win: int, segments: list[Segment]) -> int:
        """Split sampled tokens at timestamp pairs; -> mel frames to advance."""
        t = self.tok
        tb = t.timestamp_begin
        is_ts = [x >= tb for x in toks]
        single_end = len(toks) >= 2 and not is_ts[-2] and is_ts[-1]
        cuts = [i for i in range(1, len(toks)) if is_ts[i] and is_ts[i - 1]]

        def add(a, b, body):
            text_toks = [x for x in body if x < t.eot]
            txt = t.decode(text_toks)
            if txt.strip():
                segments.append(Segment(len(segments), round(a, 3), round(b, 3), txt, text_toks))
        if cuts:
            if single_end:
                cuts.append(len(toks))
            last = 0
            for c in cuts:
                sl = toks[last:c]
                add(t_off + (sl[0] - tb) * TS_STEP, t_off + (sl[-1] - tb) * TS_STEP, sl)
                last = c
            if single_end:
                return win
            return (toks[last - 1] - tb) * 2 if last > 0 else win
        dur = win * HOP / SAMPLE_RATE
        ts = [x for x in toks if x >= tb]
        if ts and ts[-1] != tb:
            dur = (ts[-1] - tb) * TS_STEP
        add(t_off, t_off + dur, toks)
        return win


def _logsumexp(x: np.ndarray) -> float:
    m = np.max(x)
    if not np.isfinite(m):
        return m
    return float(m + np.log(np.sum(np.exp(x - m))))


# ------------------------------------------------------------------------------------------------
# loading

def load_whisper(path: str, device="cpu"):
    """-> (WhisperModel, WhisperTokenizer). `path`: ggml .bin, HF directory / .safetensors, a CTranslate2
    (faster-whisper) directory with model.bin, or `synthetic:<preset>`."""
    import os
    from ..tokenizer.whisper import WhisperTokenizer
    if path.startswith("synthetic:"):
        name = path.split(":", 1)[1]
        cfg = PRESETS.get(name) or PRESETS.get("whisper-" + name)
        if cfg is None:
            raise ValueError(f"unknown synthetic whisper preset {name!r}")
        w = synthetic_whisper(cfg, 0)
        return WhisperModel(cfg, w.get, device), WhisperTokenizer.synthetic(cfg.n_vocab)
    ct2 = os.path.join(path, "model.bin") if os.path.isdir(path) else path if path.endswith("model.bin") else ""
    if ct2 and os.path.isfile(ct2):
        # CTranslate2 (faster-whisper) directory: model.bin + config.json + tokenizer / vocabulary files
        from ..formats.ctranslate2 import read_model_bin, whisper_to_openai
        d = os.path.dirname(ct2)
        v, meta = read_model_bin(ct2)
        if not meta["spec"].startswith("Whisper"):
            raise ValueError(f"{ct2}: CTranslate2 spec {meta['spec']!r} is not a Whisper model")
        w, heads = whisper_to_openai(v)

        def nl(side):
            return 1 + max(int(k.split(".")[2]) for k in w if k.startswith(f"{side}.blocks."))
        cfg = WhisperConfig(n_vocab=w["decoder.token_embedding.weight"].shape[0],
                            n_audio_ctx=w["encoder.positional_embedding"].shape[0],
                            n_audio_state=w["encoder.conv1.weight"].shape[0], n_audio_head=heads["enc_heads"],
                            n_audio_layer=nl("encoder"), n_text_ctx=w["decoder.positional_embedding"].shape[0],
                            n_text_state=w["decoder.token_embedding.weight"].shape[1], n_text_head=heads["dec_heads"],
                            n_text_layer=nl("decoder"), n_mels=w["encoder.conv1.weight"].shape[1],
                            name=os.path.basename(os.path.abspath(d)))
        return WhisperModel(cfg, w.get, device), WhisperTokenizer.from_hf_dir(d, cfg.n_vocab)
    if os.path.isdir(path) or path.endswith(".safetensors"):
        import json
        from safetensors.numpy import load_file
        d = path if os.path.isdir(path) else os.path.dirname(path)
        st = os.path.join(d, "model.safetensors") if os.path.isdir(path) else path
        with open(os.path.join(d, "config.json")) as f:
            hc = json.load(f)
        cfg = WhisperConfig(n_vocab=hc["vocab_size"], n_audio_ctx=hc["max_source_positions"],
                            n_audio_state=hc["d_model"], n_audio_head=hc["encoder_attention_heads"],
                            n_audio_layer=hc["encoder_layers"], n_text_ctx=hc["max_target_positions"],
                            n_text_state=hc["d_model"], n_text_head=hc["decoder_attention_heads"],
                            n_text_layer=hc["decoder_layers"], n_mels=hc.get("num_mel_bins", 80),
                            name=hc.get("_name_or_path", "whisper"))
        raw = load_file(st)
        w = {}
        for k, v in raw.items():
            n = hf_to_openai_name(k)
            if n is not None:
                w[n] = v.astype(np.float32)
        return WhisperModel(cfg, w.get, device), WhisperTokenizer.from_hf_dir(d, cfg.n_vocab)
    from ..formats.ggml_whisper import GGMLWhisperFile
    f = GGMLWhisperFile(path)
    hp = f.hparams
    cfg = WhisperConfig(**{k: hp[k] for k in hp if k != "ftype"}, name=os.path.basename(path))
    model = WhisperModel(cfg, f.tensor, device, mel_filters=f.mel_filters)
    return model, WhisperTokenizer.from_ggml_vocab(f.vocab, cfg.n_vocab)
