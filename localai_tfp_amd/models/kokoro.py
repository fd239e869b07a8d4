"""Kokoro-82M (StyleTTS 2 with an iSTFTNet decoder): the reference's `kokoro` backend.

Reference: backend/python/kokoro/backend.py:47-99 (LoadModel: `ModelFile` = the .pth checkpoint, option
`voice:<name>` or `voice:<a>+<b>` (averaged) loading `<ModelPath>/<voice>.pt` voice packs; TTS writes the
waveform to `dst`), with the model code in kokoro/models.py, istftnet.py, kokoro.py, plbert.py. Checkpoint
layout: {"net": {"bert", "bert_encoder", "predictor", "decoder", "text_encoder"}} state dicts (an optional
"module." prefix), weight-normalised convolutions as weight_g / weight_v (folded at load). Loaded with
torch.load(weights_only=True).

Pipeline for one utterance (phoneme ids t, voice pack row ref = pack[len(t)] split into a 128-d decoder
style and a 128-d prosody style):
  PL-BERT (ALBERT, 12 shared layers) -> linear -> duration encoder (3 x [BiLSTM, AdaLayerNorm], style
  concatenated) -> BiLSTM -> per-token durations (sigmoid bins summed, / speed, rounded) -> hard alignment;
  shared BiLSTM on the aligned features -> F0 and energy curves (AdaIN residual blocks, 2x upsampled);
  text encoder (embedding, 3 x [conv5, LayerNorm, LeakyReLU], BiLSTM) aligned -> decoder: AdaIN residual
  blocks -> iSTFTNet generator (harmonic-plus-noise source from F0 through a 9-harmonic sine bank and an
  STFT, 2 transposed-conv upsamplers with Snake AdaIN resblocks, conv_post -> magnitude / phase -> iSTFT).
Text normalisation and phonemisation: espeak-ng is not available here; the English rule phonemiser of the
piper voices (models/piper.py) produces the IPA string, mapped onto Kokoro's symbol table. Audio is 24 kHz
(the generator's harmonic source runs at 24 kHz; the reference's backend writes it with a 22050 Hz header).
The ALBERT encoder runs on the repo's GEMM + flash attention kernels; LSTMs, 1D convolutions and the
iSTFT run on PyTorch ops. Parity: the ALBERT tower is checked against transformers' AlbertModel; the rest
against a re-statement in the tests (no Kokoro weights here: audio parity unpinned).
"""
from __future__ import annotations

import math
import os
import re
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

SAMPLE_RATE = 24000

_PAD = "$"
_PUNCT = ';:,.!?¡¿—…"«»“” '
_LETTERS = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
_IPA = ("ɑɐɒæɓʙβɔɕçɗɖðʤəɘɚɛɜɝɞɟʄɡɠɢʛɦɧħɥʜɨɪʝɭɬɫɮʟɱɯɰŋɳɲɴøɵɸθœɶʘɹɺɾɻʀʁɽʂʃʈʧʉʊʋⱱʌɣɤʍχʎʏʑʐʒʔʡʕʢǀǁǂǃˈˌːˑʼʴʰʱʲʷˠˤ˞↓↑→↗↘'̩'ᵻ")
VOCAB = {}
for _i, _s in enumerate([_PAD] + list(_PUNCT) + list(_LETTERS) + list(_IPA)):
    VOCAB[_s] = _i  # later duplicates (the apostrophe) keep the last index, as a dict comprehension would


@dataclass
class KokoroConfig:
    hidden: int = 512
    style: int = 128
    n_token: int = 178
    n_layer: int = 3
    max_dur: int = 50
    upsample_rates: tuple = (10, 6)
    upsample_initial: int = 512
    resblock_kernels: tuple = (3, 7, 11)
    resblock_dilations: tuple = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    upsample_kernels: tuple = (20, 12)
    n_fft: int = 20
    hop: int = 5
    bert_hidden: int = 768
    bert_heads: int = 12
    bert_inter: int = 2048
    bert_layers: int = 12
    bert_emb: int = 128
    bert_max_pos: int = 512
    decoder_dims: tuple = (1024, 64)  # AdaIN block width, asr residual width


KOKORO_V019 = KokoroConfig()
KOKORO_TEST = KokoroConfig(hidden=64, style=16, n_layer=2, max_dur=8, upsample_rates=(4, 2), upsample_initial=32,
                           upsample_kernels=(8, 4), n_fft=8, hop=2, bert_hidden=128, bert_heads=2, bert_inter=64,
                           bert_layers=2, bert_emb=16, bert_max_pos=128, decoder_dims=(48, 8))


# ------------------------------------------------------------------------------------------ text
def _split_num(m):
    num = m.group()
    if "." in num:
        return num
    if ":" in num:
        h, mi = (int(x) for x in num.split(":"))
        return f"{h} o'clock" if mi == 0 else (f"{h} oh {mi}" if mi < 10 else f"{h} {mi}")
    year = int(num[:4])
    if year < 1100 or year % 1000 < 10:
        return num
    left, right = num[:2], int(num[2:4])
    s = "s" if num.endswith("s") else ""
    if 100 <= year % 1000 <= 999:
        if right == 0:
            return f"{left} hundred{s}"
        if right < 10:
            return f"{left} oh {right}{s}"
    return f"{left} {right}{s}"


def normalize_text(text: str) -> str:
    """Kokoro's English text normalisation (quotes, titles, times / years, decimal points, ranges)."""
    t = text.replace("‘", "'").replace("’", "'").replace("“", '"').replace("”", '"')
    t = re.sub(r"[^\S \n]", " ", t)
    t = re.sub(r"  +", " ", t)
    t = re.sub(r"\bD[Rr]\.(?= [A-Z])", "Doctor", t)
    t = re.sub(r"\b(?:Mr\.|MR\.(?= [A-Z]))", "Mister", t)
    t = re.sub(r"\b(?:Ms\.|MS\.(?= [A-Z]))", "Miss", t)
    t = re.sub(r"\b(?:Mrs\.|MRS\.(?= [A-Z]))", "Mrs", t)
    t = re.sub(r"\d*\.\d+|\b\d{4}s?\b|(?<!:)\b(?:[1-9]|1[0-2]):[0-5]\d\b(?!:)", _split_num, t)
    t = re.sub(r"(?<=\d),(?=\d)", "", t)
    t = re.sub(r"\d*\.\d+", lambda m: " point ".join([m.group().split(".")[0], " ".join(m.group().split(".")[1])]), t)
    t = re.sub(r"(?<=\d)-(?=\d)", " to ", t)
    return t.strip()


def phonemize(text: str, lang: str = "a", espeak=None) -> str:
    """IPA string in Kokoro's symbol set: espeak-ng when a backend callable is given, else the built-in
    English rules (models/piper.py)."""
    t = normalize_text(text)
    if espeak is not None:
        ps = espeak(t)
    else:
        from .piper import english_to_ipa
        ps = english_to_ipa(t)
    ps = ps.replace("ʲ", "j").replace("r", "ɹ").replace("x", "k").replace("ɬ", "l")
    return "".join(c for c in ps if c in VOCAB).strip()


def tokenize(ps: str) -> list[int]:
    return [VOCAB[c] for c in ps if c in VOCAB]


# ------------------------------------------------------------------------------------------ weights
def _fold_weight_norm(sd: dict) -> dict:
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_v"):
            base = k[:-2]
            g = sd[base + "_g"].float()
            vv = v.float()
            n = vv.norm(dim=tuple(range(1, vv.ndim)), keepdim=True)
            out[base] = g * vv / n
        elif k.endswith(".weight_g"):
            continue
        else:
            out[k] = v
    return out


def load_checkpoint(path: str) -> dict:
    """-> {"bert.*", "bert_encoder.*", "predictor.*", "decoder.*", "text_encoder.*"} fp32 tensors."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    net = ck.get("net", ck)
    out = {}
    for part, sd in net.items():
        sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
        for k, v in _fold_weight_norm(sd).items():
            if torch.is_tensor(v):
                out[f"{part}.{k}"] = v.float()
    return out


# ------------------------------------------------------------------------------------------ model
class Kokoro:
    def __init__(self, cfg: KokoroConfig, params: dict, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.p = {k: v.to(self.device) for k, v in params.items()}
        self._lstms = {}
        self._cw = {}  # GPU: packed conv.hip weights per conv name

    # ---- building blocks
    def _lin(self, x, name, bias=True):
        return F.linear(x, self.p[name + ".weight"], self.p.get(name + ".bias") if bias else None)

    def _conv(self, x, name, stride=1, padding=0, dilation=1):
        """Conv1d [B, C, T] -> [B, Cout, T']: on the GPU the implicit-GEMM conv kernel (conv.hip, f16 operands,
        fp32 accumulation; ops/conv.py conv1d), elsewhere F.conv1d."""
        if x.is_cuda:
            from ..ops import conv as CV
            cw = self._cw.get(name)
            if cw is None:
                cw = self._cw[name] = CV.conv1d_weights(self.p[name + ".weight"], self.p.get(name + ".bias"))
            return CV.conv1d(x, cw, stride=stride, padding=padding, dilation=dilation)
        return F.conv1d(x, self.p[name + ".weight"], self.p.get(name + ".bias"), stride=stride, padding=padding,
                        dilation=dilation)

    def _up_transpose(self, x, name, u, k):
        """The generator's ConvTranspose1d(k, stride u, padding (k - u) / 2): on the GPU, for the HiFi-GAN geometry
        k = 2u, as the k = 2 conv producing the u output phases per frame (ops/conv.py conv_transpose1d)."""
        w, b = self.p[name + ".weight"], self.p.get(name + ".bias")
        if x.is_cuda and k == 2 * u:
            from ..ops import conv as CV
            cwt = self._cw.get(name)
            if cwt is None:
                cwt = self._cw[name] = CV.conv_transpose1d_weights(w, b, u)
            return CV.conv_transpose1d(x, cwt, (k - u) // 2)
        return F.conv_transpose1d(x, w, b, stride=u, padding=(k - u) // 2)

    @staticmethod
    def _pool_up2(x, w, b):
        """Depthwise ConvTranspose1d(k 3, stride 2, padding 1, output_padding 1) [B, C, T] -> [B, C, 2T] as two
        elementwise phases: y[2i] = w1 x[i], y[2i+1] = w2 x[i] + w0 x[i+1] (no library conv)."""
        w = w[:, 0]  # [C, 3]
        nxt = F.pad(x[:, :, 1:], (0, 1))
        ev = w[:, 1, None] * x
        od = w[:, 2, None] * x + w[:, 0, None] * nxt
        y = torch.stack([ev, od], -1).reshape(x.shape[0], x.shape[1], 2 * x.shape[2])
        return y + b[:, None] if b is not None else y

    def _lstm(self, x, name):
        """Bidirectional single-layer LSTM over [1, T, C] -> [1, T, 2H]: on the GPU the cooperative scan kernel
        (ops/rnn.py, audio.hip lstm_bidir_coop), elsewhere torch.nn.LSTM."""
        if x.is_cuda and self.p[name + ".weight_hh_l0"].shape[1] in (128, 256):
            from ..ops.rnn import lstm_bidir
            return lstm_bidir(x[0], self.p, name, self._lstms)[None]
        m = self._lstms.get(name)
        if m is None:
            w = self.p[name + ".weight_ih_l0"]
            m = torch.nn.LSTM(w.shape[1], w.shape[0] // 4, 1, batch_first=True, bidirectional=True).to(self.device)
            with torch.no_grad():
                for n, prm in m.named_parameters():
                    prm.copy_(self.p[f"{name}.{n}"])
            m.eval()
            self._lstms[name] = m
        return m(x)[0]

    def _adain(self, x, s, name):
        """AdaIN1d: (1 + gamma) * InstanceNorm(x) + beta, (gamma, beta) = fc(s)."""
        h = self._lin(s, name + ".fc")
        g, b = h.chunk(2, dim=-1)
        if x.is_cuda:  # InstanceNorm1d as reductions (no library norm kernel)
            var, mean = torch.var_mean(x, dim=-1, keepdim=True, unbiased=False)
            xn = (x - mean) * torch.rsqrt(var + 1e-5)
        else:
            xn = F.instance_norm(x, eps=1e-5)
        return (1 + g[..., None]) * xn + b[..., None]

    def _adain_res_blk(self, x, s, name, upsample: bool):
        """StyleTTS 2 AdainResBlk1d: (residual + shortcut) / sqrt(2), optional 2x upsampling."""
        h = F.leaky_relu(self._adain(x, s, name + ".norm1"), 0.2)
        if upsample:
            w = self.p[name + ".pool.weight"]
            if h.is_cuda and w.shape[1:] == (1, 3):
                h = self._pool_up2(h, w, self.p.get(name + ".pool.bias"))
            else:
                h = F.conv_transpose1d(h, w, self.p.get(name + ".pool.bias"), stride=2, padding=1, output_padding=1,
                                       groups=w.shape[0])
        h = self._conv(h, name + ".conv1", padding=1)
        h = F.leaky_relu(self._adain(h, s, name + ".norm2"), 0.2)
        h = self._conv(h, name + ".conv2", padding=1)
        sc = F.interpolate(x, scale_factor=2, mode="nearest") if upsample else x
        if name + ".conv1x1.weight" in self.p:
            sc = self._conv(sc, name + ".conv1x1")
        return (h + sc) / math.sqrt(2)

    def _snake_res(self, x, s, name, k, dil):
        """iSTFTNet AdaINResBlock1 with Snake activations x + sin^2(a x) / a."""
        for j, d in enumerate(dil):
            a1, a2 = self.p[f"{name}.alpha1.{j}"], self.p[f"{name}.alpha2.{j}"]
            t = self._adain(x, s, f"{name}.adain1.{j}")
            t = t + (1 / a1) * torch.sin(a1 * t) ** 2
            t = self._conv(t, f"{name}.convs1.{j}", dilation=d, padding=(k * d - d) // 2)
            t = self._adain(t, s, f"{name}.adain2.{j}")
            t = t + (1 / a2) * torch.sin(a2 * t) ** 2
            x = x + self._conv(t, f"{name}.convs2.{j}", padding=(k - 1) // 2)
        return x

    # ---- ALBERT (PL-BERT) on the repo kernels
    def bert(self, ids: torch.Tensor) -> torch.Tensor:
        from ..ops import core as K
        c, P = self.cfg, self.p
        L = ids.shape[0]
        pre = "bert.embeddings."
        e = P[pre + "word_embeddings.weight"][ids] + P[pre + "position_embeddings.weight"][:L] + \
            P[pre + "token_type_embeddings.weight"][0]
        e = F.layer_norm(e, (c.bert_emb,), P[pre + "LayerNorm.weight"], P[pre + "LayerNorm.bias"], 1e-12)
        h = self._lin(e, "bert.encoder.embedding_hidden_mapping_in")
        lp = "bert.encoder.albert_layer_groups.0.albert_layers.0."
        D, H = c.bert_hidden, c.bert_heads
        hd = D // H
        for _ in range(c.bert_layers):  # ALBERT: one layer's weights, applied bert_layers times
            q = self._lin(h, lp + "attention.query")
            k = self._lin(h, lp + "attention.key")
            v = self._lin(h, lp + "attention.value")
            if h.is_cuda:
                dt = torch.bfloat16
                o = torch.empty(L, D, dtype=dt, device=h.device)
                K.attn_dense(q.to(dt), k.to(dt), v.to(dt), o, 1, L, L, H, H, hd, hd ** -0.5)
                o = o.float()
            else:
                o = F.scaled_dot_product_attention(q.view(L, H, hd).transpose(0, 1), k.view(L, H, hd).transpose(0, 1),
                                                   v.view(L, H, hd).transpose(0, 1)).transpose(0, 1).reshape(L, D)
            a = F.layer_norm(h + self._lin(o, lp + "attention.dense"), (D,), P[lp + "attention.LayerNorm.weight"],
                             P[lp + "attention.LayerNorm.bias"], 1e-12)
            f = self._lin(F.gelu(self._lin(a, lp + "ffn"), approximate="tanh"), lp + "ffn_output")
            h = F.layer_norm(f + a, (D,), P[lp + "full_layer_layer_norm.weight"], P[lp + "full_layer_layer_norm.bias"],
                             1e-12)
        return h

    # ---- the utterance
    @torch.no_grad()
    def synthesize(self, tokens: list[int], ref_s: torch.Tensor, speed: float = 1.0, seed: int = 0) -> np.ndarray:
        c = self.cfg
        dev = self.device
        gen = torch.Generator(device="cpu").manual_seed(seed)
        ids = torch.tensor([0, *tokens[:510], 0], device=dev)
        L = ids.shape[0]
        ref_s = ref_s.reshape(1, -1).float().to(dev)
        s_dec, s = ref_s[:, :c.style], ref_s[:, c.style:]
        d_en = self._lin(self.bert(ids), "bert_encoder")  # [L, hidden]
        # duration encoder: [BiLSTM, AdaLayerNorm] x n_layer with the style concatenated
        x = torch.cat([d_en, s.expand(L, -1)], -1)[None]
        for i in range(c.n_layer):
            x = self._lstm(x, f"predictor.text_encoder.lstms.{2 * i}")[0]
            h = self._lin(s, f"predictor.text_encoder.lstms.{2 * i + 1}.fc")
            g, b = h.chunk(2, dim=-1)
            x = (1 + g) * F.layer_norm(x, (c.hidden,), eps=1e-5) + b
            x = torch.cat([x, s.expand(L, -1)], -1)[None]
        d = x[0]  # [L, hidden + style]
        dur = torch.sigmoid(self._lin(self._lstm(d[None], "predictor.lstm")[0], "predictor.duration_proj.linear_layer"))
        pred = torch.round(dur.sum(-1) / speed).clamp(min=1).long()  # [L]
        Fr = int(pred.sum())
        aln = torch.zeros(L, Fr, device=dev)
        aln[torch.repeat_interleave(torch.arange(L, device=dev), pred), torch.arange(Fr, device=dev)] = 1.0
        en = d.T @ aln  # [hidden + style, F]
        sh = self._lstm(en.T[None], "predictor.shared")[0].T[None]  # [1, hidden, F]
        curves = []
        for head in ("F0", "N"):
            y = sh
            for j, up in enumerate((False, True, False)):
                y = self._adain_res_blk(y, s, f"predictor.{head}.{j}", up)
            curves.append(self._conv(y, f"predictor.{head}_proj")[:, 0])  # [1, 2F]
        f0, nn_ = curves
        # text encoder
        t = self.p["text_encoder.embedding.weight"][ids].T[None]  # [1, hidden, L]
        for i in range(c.n_layer):
            t = self._conv(t, f"text_encoder.cnn.{i}.0", padding=2)
            t = F.layer_norm(t.transpose(1, 2), (c.hidden,), self.p[f"text_encoder.cnn.{i}.1.gamma"],
                             self.p[f"text_encoder.cnn.{i}.1.beta"], 1e-5).transpose(1, 2)
            t = F.leaky_relu(t, 0.2)
        t = self._lstm(t.transpose(1, 2), "text_encoder.lstm").transpose(1, 2)  # [1, hidden, L]
        asr = t @ aln[None]
        return self.decode(asr, f0, nn_, s_dec, gen).cpu().numpy()

    def decode(self, asr, f0_curve, n_curve, s, gen) -> torch.Tensor:
        c = self.cfg
        f0 = self._conv(f0_curve[:, None], "decoder.F0_conv", stride=2, padding=1)
        nn_ = self._conv(n_curve[:, None], "decoder.N_conv", stride=2, padding=1)
        x = self._adain_res_blk(torch.cat([asr, f0, nn_], 1), s, "decoder.encode", False)
        ar = self._conv(asr, "decoder.asr_res.0")
        for i in range(4):
            x = self._adain_res_blk(torch.cat([x, ar, f0, nn_], 1), s, f"decoder.decode.{i}", i == 3)
        return self.generator(x, s, f0_curve, gen)

    def _harmonic_source(self, f0_curve, gen):
        """9-harmonic sine bank at 24 kHz from the frame-rate F0 (phase integrated at frame rate, then
        linearly upsampled), unvoiced below 10 Hz, merged by a linear + tanh."""
        c = self.cfg
        up = int(np.prod(c.upsample_rates) * c.hop)
        f0 = f0_curve[:, None].repeat_interleave(up, dim=2).transpose(1, 2)  # [1, T, 1] nearest upsampling
        fn = f0 * torch.arange(1, 10, device=f0.device, dtype=f0.dtype)
        rad = (fn / SAMPLE_RATE) % 1
        ini = torch.rand(1, 9, generator=gen).to(f0.device)
        ini[:, 0] = 0
        rad[:, 0, :] = rad[:, 0, :] + ini
        r = F.interpolate(rad.transpose(1, 2), scale_factor=1 / up, mode="linear").transpose(1, 2)
        phase = torch.cumsum(r, dim=1) * 2 * np.pi
        phase = F.interpolate(phase.transpose(1, 2) * up, scale_factor=up, mode="linear").transpose(1, 2)
        sines = torch.sin(phase) * 0.1
        uv = (f0 > 10).float()
        noise = (uv * 0.003 + (1 - uv) * 0.1 / 3) * torch.randn(sines.shape, generator=gen).to(f0.device)
        sw = sines * uv + noise
        return torch.tanh(self._lin(sw, "decoder.generator.m_source.l_linear"))[..., 0]  # [1, T]

    def generator(self, x, s, f0_curve, gen):
        c = self.cfg
        win = torch.hann_window(c.n_fft, device=x.device)
        har = self._harmonic_source(f0_curve, gen)
        st = torch.stft(har, c.n_fft, c.hop, c.n_fft, window=win, return_complex=True)
        har = torch.cat([st.abs(), st.angle()], 1)  # [1, n_fft + 2, frames]
        nu = len(c.upsample_rates)
        nk = len(c.resblock_kernels)
        for i in range(nu):
            x = F.leaky_relu(x, 0.1)
            if i + 1 < nu:
                sf = int(np.prod(c.upsample_rates[i + 1:]))
                xs = self._conv(har, f"decoder.generator.noise_convs.{i}", stride=sf, padding=(sf + 1) // 2)
                xs = self._snake_res(xs, s, f"decoder.generator.noise_res.{i}", 7, (1, 3, 5))
            else:
                xs = self._conv(har, f"decoder.generator.noise_convs.{i}")
                xs = self._snake_res(xs, s, f"decoder.generator.noise_res.{i}", 11, (1, 3, 5))
            u, k = c.upsample_rates[i], c.upsample_kernels[i]
            x = self._up_transpose(x, f"decoder.generator.ups.{i}", u, k)
            if i == nu - 1:
                x = F.pad(x, (1, 0), mode="reflect")
            x = x + xs
            acc = None
            for j in range(nk):
                y = self._snake_res(x, s, f"decoder.generator.resblocks.{i * nk + j}", c.resblock_kernels[j],
                                    c.resblock_dilations[j])
                acc = y if acc is None else acc + y
            x = acc / nk
        x = self._conv(F.leaky_relu(x), "decoder.generator.conv_post", padding=3)
        nb = c.n_fft // 2 + 1
        spec = torch.exp(x[:, :nb]) * torch.exp(1j * torch.sin(x[:, nb:]))
        return torch.istft(spec, c.n_fft, c.hop, c.n_fft, window=win)[0]


def load_voice(model_path: str, voice: str, device) -> torch.Tensor:
    """`<name>.pt` voice pack [511, 1, 2*style]; `a+b` averages two packs (backend.py:72-79)."""
    names = voice.split("+")
    packs = [torch.load(os.path.join(model_path, f"{n}.pt"), map_location="cpu", weights_only=True).float() for n in names]
    return torch.stack(packs).mean(0).to(device) if len(packs) > 1 else packs[0].to(device)


def config_for(params: dict) -> KokoroConfig:
    """Dimensions from the checkpoint (v0.19 defaults for the iSTFT / upsampling hyper-parameters)."""
    p = params
    hidden = p["text_encoder.embedding.weight"].shape[1]
    style = p["decoder.encode.norm1.fc.weight"].shape[1]
    n_layer = sum(1 for k in p if re.fullmatch(r"text_encoder\.cnn\.\d+\.0\.weight", k))
    bh = p["bert.encoder.embedding_hidden_mapping_in.weight"].shape[0]
    kw = dict(hidden=hidden, style=style, n_token=p["text_encoder.embedding.weight"].shape[0], n_layer=n_layer,
              max_dur=p["predictor.duration_proj.linear_layer.weight"].shape[0], bert_hidden=bh,
              bert_emb=p["bert.embeddings.word_embeddings.weight"].shape[1],
              bert_inter=p["bert.encoder.albert_layer_groups.0.albert_layers.0.ffn.weight"].shape[0],
              bert_max_pos=p["bert.embeddings.position_embeddings.weight"].shape[0],
              upsample_initial=p["decoder.generator.ups.0.weight"].shape[0],
              n_fft=p["decoder.generator.conv_post.weight"].shape[0] - 2,
              decoder_dims=(p["decoder.encode.conv1.weight"].shape[0], p["decoder.asr_res.0.weight"].shape[0]))
    nu = sum(1 for k in p if re.fullmatch(r"decoder\.generator\.ups\.\d+\.weight", k))
    kernels = tuple(p[f"decoder.generator.ups.{i}.weight"].shape[-1] for i in range(nu))
    nk = sum(1 for k in p if re.fullmatch(r"decoder\.generator\.resblocks\.\d+\.convs1\.0\.weight", k)) // nu
    kw.update(upsample_kernels=kernels, upsample_rates=tuple(k // 2 for k in kernels),  # v0.19: k = 2 x rate
              resblock_kernels=tuple(p[f"decoder.generator.resblocks.{j}.convs1.0.weight"].shape[-1] for j in range(nk)),
              resblock_dilations=((1, 3, 5),) * nk, hop=kw["n_fft"] // 4)
    return KokoroConfig(**kw, bert_heads=max(1, bh // 64))


def synthetic_params(c: KokoroConfig, seed: int = 0) -> dict:
    """Random tensors under the checkpoint's (weight-norm folded) names and shapes (tests / benchmarks)."""
    g = torch.Generator().manual_seed(seed)
    P = {}

    def t(name, *shape, std=None, one=False):
        if one:
            P[name] = 1 + 0.1 * torch.randn(*shape, generator=g)
        else:
            fan = int(np.prod(shape[1:])) if len(shape) > 1 else shape[0]
            P[name] = torch.randn(*shape, generator=g) * (std if std is not None else 1.0 / math.sqrt(max(fan, 1)))

    def lin(name, o, i, bias=True):
        t(name + ".weight", o, i)
        if bias:
            t(name + ".bias", o, std=0.02)

    def conv(name, o, i, k, bias=True):
        t(name + ".weight", o, i, k)
        if bias:
            t(name + ".bias", o, std=0.02)

    def lstm(name, i, h):
        for sfx in ("", "_reverse"):
            t(f"{name}.weight_ih_l0{sfx}", 4 * h, i)
            t(f"{name}.weight_hh_l0{sfx}", 4 * h, h)
            t(f"{name}.bias_ih_l0{sfx}", 4 * h, std=0.05)
            t(f"{name}.bias_hh_l0{sfx}", 4 * h, std=0.05)

    def adain_blk(name, di, do, up):
        conv(name + ".conv1", do, di, 3)
        conv(name + ".conv2", do, do, 3)
        lin(name + ".norm1.fc", 2 * di, c.style)
        lin(name + ".norm2.fc", 2 * do, c.style)
        if di != do:
            conv(name + ".conv1x1", do, di, 1, bias=False)
        if up:
            conv(name + ".pool", di, 1, 3)

    def snake(name, ch, k):
        for j in range(3):
            conv(f"{name}.convs1.{j}", ch, ch, k)
            conv(f"{name}.convs2.{j}", ch, ch, k)
            lin(f"{name}.adain1.{j}.fc", 2 * ch, c.style)
            lin(f"{name}.adain2.{j}.fc", 2 * ch, c.style)
            t(f"{name}.alpha1.{j}", 1, ch, 1, one=True)
            t(f"{name}.alpha2.{j}", 1, ch, 1, one=True)
    bh, e = c.bert_hidden, c.bert_emb
    t("bert.embeddings.word_embeddings.weight", c.n_token, e, std=0.5)
    t("bert.embeddings.position_embeddings.weight", c.bert_max_pos, e, std=0.1)
    t("bert.embeddings.token_type_embeddings.weight", 2, e, std=0.1)
    t("bert.embeddings.LayerNorm.weight", e, one=True)
    t("bert.embeddings.LayerNorm.bias", e, std=0.02)
    lin("bert.encoder.embedding_hidden_mapping_in", bh, e)
    lp = "bert.encoder.albert_layer_groups.0.albert_layers.0."
    for n in ("query", "key", "value", "dense"):
        lin(lp + "attention." + n, bh, bh)
    t(lp + "attention.LayerNorm.weight", bh, one=True)
    t(lp + "attention.LayerNorm.bias", bh, std=0.02)
    lin(lp + "ffn", c.bert_inter, bh)
    lin(lp + "ffn_output", bh, c.bert_inter)
    t(lp + "full_layer_layer_norm.weight", bh, one=True)
    t(lp + "full_layer_layer_norm.bias", bh, std=0.02)
    lin("bert_encoder", c.hidden, bh)
    hs, h2 = c.hidden + c.style, c.hidden // 2
    for i in range(c.n_layer):
        lstm(f"predictor.text_encoder.lstms.{2 * i}", hs, h2)
        lin(f"predictor.text_encoder.lstms.{2 * i + 1}.fc", 2 * c.hidden, c.style)
    lstm("predictor.lstm", hs, h2)
    lin("predictor.duration_proj.linear_layer", c.max_dur, c.hidden)
    lstm("predictor.shared", hs, h2)
    for head in ("F0", "N"):
        adain_blk(f"predictor.{head}.0", c.hidden, c.hidden, False)
        adain_blk(f"predictor.{head}.1", c.hidden, h2, True)
        adain_blk(f"predictor.{head}.2", h2, h2, False)
        conv(f"predictor.{head}_proj", 1, h2, 1)
    t("text_encoder.embedding.weight", c.n_token, c.hidden, std=0.3)
    for i in range(c.n_layer):
        conv(f"text_encoder.cnn.{i}.0", c.hidden, c.hidden, 5)
        t(f"text_encoder.cnn.{i}.1.gamma", c.hidden, one=True)
        t(f"text_encoder.cnn.{i}.1.beta", c.hidden, std=0.02)
    lstm("text_encoder.lstm", c.hidden, h2)
    D1, D2 = c.decoder_dims
    adain_blk("decoder.encode", c.hidden + 2, D1, False)
    for i in range(3):
        adain_blk(f"decoder.decode.{i}", D1 + 2 + D2, D1, False)
    adain_blk("decoder.decode.3", D1 + 2 + D2, c.upsample_initial, True)
    conv("decoder.F0_conv", 1, 1, 3)
    conv("decoder.N_conv", 1, 1, 3)
    conv("decoder.asr_res.0", D2, c.hidden, 1)
    lin("decoder.generator.m_source.l_linear", 1, 9)
    nu = len(c.upsample_rates)
    for i in range(nu):
        cur = c.upsample_initial // 2 ** (i + 1)
        if i + 1 < nu:
            sf = int(np.prod(c.upsample_rates[i + 1:]))
            conv(f"decoder.generator.noise_convs.{i}", cur, c.n_fft + 2, 2 * sf)
            snake(f"decoder.generator.noise_res.{i}", cur, 7)
        else:
            conv(f"decoder.generator.noise_convs.{i}", cur, c.n_fft + 2, 1)
            snake(f"decoder.generator.noise_res.{i}", cur, 11)
        t(f"decoder.generator.ups.{i}.weight", c.upsample_initial // 2 ** i, cur, c.upsample_kernels[i])
        t(f"decoder.generator.ups.{i}.bias", cur, std=0.02)
        for j, k in enumerate(c.resblock_kernels):
            snake(f"decoder.generator.resblocks.{i * len(c.resblock_kernels) + j}", cur, k)
    conv("decoder.generator.conv_post", c.n_fft + 2, c.upsample_initial // 2 ** nu, 7)
    return P
