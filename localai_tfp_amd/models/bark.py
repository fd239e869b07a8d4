"""Bark text-to-speech (the reference's ``bark`` / ``bark-cpp`` backends: backend/python/bark/backend.py:32-56,
backend/go/bark/gobark.cpp:22-80), on Hugging Face ``BarkModel`` checkpoint names and generation semantics.

Three GPT-2-style transformers and a codec:

1. semantic ("text") model, causal: BERT-tokenised text (+10 048 offset, padded to 256 with the text pad
   token) summed with the speaker's semantic history, an infer token, then greedy / sampled semantic tokens
   (vocab 10 000, EOS 10 000; ids 10 001..10 047 suppressed; optional min-EOS-probability early stop);
2. coarse acoustics model, causal: semantic tokens -> the first two EnCodec codebooks, interleaved
   (codebook 0 at even steps, 1 at odd steps, each restricted to its 1024-id band above 10 000), generated
   in sliding windows of 60 tokens over a 256-token semantic window + 630 tokens of coarse history;
3. fine acoustics model, NON-causal: fills codebooks 2..7 one at a time over 1024-frame windows (one
   embedding table per codebook, summed over the codebooks known so far; one LM head per predicted codebook);
4. EnCodec 24 kHz decoder (models/encodec.py, ``codec_model.*``) -> waveform.

MI355X mapping: every GPT block runs fused-QKV / MLP GEMMs on hipBLASLt and attention through PyTorch
SDPA over a preallocated per-model KV cache (prefill once per window, then one-token decode steps); the
codec runs on the implicit-GEMM MFMA conv kernel. CPU tensors run the same code in fp32 — the oracle for
the transformers-parity tests (greedy).
Speaker presets (``history_prompt``): suno/HF ``.npz`` voice files with ``semantic_prompt``,
``coarse_prompt`` and ``fine_prompt`` arrays (loaded with allow_pickle=False).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..ops.core import attn_dense
from .encodec import EncodecConfig, EncodecDecoder


@dataclass
class BarkGen:
    """Generation constants (transformers BarkSemantic/Coarse/FineGenerationConfig defaults)."""
    text_encoding_offset: int = 10_048
    text_pad_token: int = 129_595
    semantic_infer_token: int = 129_599
    semantic_vocab_size: int = 10_000
    eos: int = 10_000
    max_input_semantic_length: int = 256
    semantic_rate_hz: float = 49.9
    max_semantic_new: int = 768
    coarse_semantic_pad_token: int = 12_048
    coarse_rate_hz: float = 75
    n_coarse: int = 2
    coarse_infer_token: int = 12_050
    max_coarse_input_length: int = 256
    max_coarse_history: int = 630
    sliding_window_len: int = 60
    max_fine_history_length: int = 512
    max_fine_input_length: int = 1024
    n_fine: int = 8
    codebook_size: int = 1024
    sample_rate: int = 24_000


class _GPT:
    """Bark GPT core (pre-LN blocks, fused att_proj, GELU MLP); causal or not; one or many embeddings/heads."""

    def __init__(self, sd: dict, prefix: str, cfg: dict, device, dtype, causal: bool):
        self.causal = causal
        self.gelu_approx = cfg.get("gelu_approx", "none")  # "tanh": GPT-2's gelu_new (XTTS, models/xtts.py)
        self.H = cfg["num_heads"]
        self.D = cfg["hidden_size"]
        self.device, self.dtype = torch.device(device), dtype
        dev, dt = self.device, dtype

        def t(name, d=dt):
            v = sd.get(prefix + name)
            return None if v is None else v.to(dev, d).contiguous()

        if causal:
            self.emb = [t("input_embeds_layer.weight")]
            self.heads = [t("lm_head.weight")]
        else:
            n = cfg.get("n_codes_total", 8)
            self.emb = [t(f"input_embeds_layers.{i}.weight") for i in range(n)]
            self.heads = [t(f"lm_heads.{i}.weight") for i in range(n - cfg.get("n_codes_given", 1))]
        self.pos = t("position_embeds_layer.weight", torch.float32)
        self.layers = []
        for i in range(cfg["num_layers"]):
            L = f"layers.{i}."
            self.layers.append(dict(
                ln1=(t(L + "layernorm_1.weight", torch.float32), t(L + "layernorm_1.bias", torch.float32)),
                ln2=(t(L + "layernorm_2.weight", torch.float32), t(L + "layernorm_2.bias", torch.float32)),
                qkv=t(L + "attn.att_proj.weight"), qkv_b=t(L + "attn.att_proj.bias"),
                o=t(L + "attn.out_proj.weight"), o_b=t(L + "attn.out_proj.bias"),
                fc1=t(L + "mlp.in_proj.weight"), fc1_b=t(L + "mlp.in_proj.bias"),
                fc2=t(L + "mlp.out_proj.weight"), fc2_b=t(L + "mlp.out_proj.bias")))
        self.ln_f = (t("layernorm_final.weight", torch.float32), t("layernorm_final.bias", torch.float32))

    def _ln(self, x, wb):
        return F.layer_norm(x, (self.D,), wb[0], wb[1], 1e-5).to(self.dtype)

    def new_cache(self, B: int, T: int):
        """Token-major K / V rows [B, T, D] per layer (the layout attn_dense reads, capacity T)."""
        return [[torch.empty(B, T, self.D, device=self.device, dtype=self.dtype),
                 torch.empty(B, T, self.D, device=self.device, dtype=self.dtype)] for _ in self.layers]

    def forward(self, x: torch.Tensor, pos0: int = 0, cache=None, head: int = 0) -> torch.Tensor:
        """x: input embeddings [B, S, D] fp32 (positions pos0..pos0+S) -> logits [B, S, V] fp32.
        Attention runs on the MFMA flash kernel (ops.core.attn_dense): causal masks are bottom-right aligned,
        so a cached chunk at pos0 attends keys 0..pos0+S-1 exactly as the reference's chunk mask."""
        x = x + self.pos[pos0:pos0 + x.shape[1]][None]
        return F.linear(self.trunk(x, pos0, cache), self.heads[head]).float()

    def trunk(self, x: torch.Tensor, pos0: int = 0, cache=None) -> torch.Tensor:
        """The transformer blocks + final LayerNorm over input embeddings x [B, S, D] fp32 (positions already
        added) -> [B, S, D] 16-bit."""
        B, S, _ = x.shape
        D, hd = self.D, self.D // self.H
        for li, L in enumerate(self.layers):
            h = self._ln(x, L["ln1"])
            qkv = F.linear(h, L["qkv"], L["qkv_b"]).view(B * S, 3 * D)
            q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
            Sk, rows = S, 0
            if cache is not None:
                kc, vc = cache[li]
                kc[:, pos0:pos0 + S] = k.view(B, S, D)
                vc[:, pos0:pos0 + S] = v.view(B, S, D)
                k, v = kc.view(-1, D), vc.view(-1, D)
                Sk, rows = pos0 + S, kc.shape[1]
            a = torch.empty(B * S, D, dtype=qkv.dtype, device=qkv.device)
            attn_dense(q, k, v, a, B, S, Sk, self.H, self.H, hd, hd ** -0.5, causal=self.causal, kv_rows=rows)
            x = x + F.linear(a.view(B, S, D), L["o"], L["o_b"]).float()
            h = self._ln(x, L["ln2"])
            x = x + F.linear(F.gelu(F.linear(h, L["fc1"], L["fc1_b"]), approximate=self.gelu_approx), L["fc2"],
                             L["fc2_b"]).float()
        return self._ln(x, self.ln_f)

    def decode_step(self, tok: torch.Tensor, pos: torch.Tensor, cache, head: int = 0) -> torch.Tensor:
        """One token (int64 [1], device) at device position pos (int64 [1]) against the cache -> logits [1, V]
        fp32. Shape-static (no host values), so the decode loop replays it as one HIP graph."""
        x = (self.emb[0].index_select(0, tok).float() + self.pos.index_select(0, pos))[None]  # [1, 1, D]
        return F.linear(self.decode_trunk(x, pos, cache), self.heads[head]).float()[:, -1]

    def decode_trunk(self, x: torch.Tensor, pos: torch.Tensor, cache) -> torch.Tensor:
        """The blocks for one token embedding x [1, 1, D] fp32 at device position pos -> [1, 1, D] 16-bit."""
        D, hd = self.D, self.D // self.H
        T = cache[0][0].shape[1]
        klen = pos.to(torch.int32) + 1
        a = torch.empty(1, D, dtype=self.dtype, device=self.device)
        for li, L in enumerate(self.layers):
            h = self._ln(x, L["ln1"])
            qkv = F.linear(h, L["qkv"], L["qkv_b"]).view(1, 3 * D)
            kc, vc = cache[li]
            kc.index_copy_(1, pos, qkv[:, None, D:2 * D])
            vc.index_copy_(1, pos, qkv[:, None, 2 * D:])
            attn_dense(qkv, kc.view(-1, D), vc.view(-1, D), a, 1, 1, T, self.H, self.H, hd, hd ** -0.5, klen=klen,
                       kv_rows=T)
            x = x + F.linear(a.view(1, 1, D), L["o"], L["o_b"]).float()
            h = self._ln(x, L["ln2"])
            x = x + F.linear(F.gelu(F.linear(h, L["fc1"], L["fc1_b"]), approximate=self.gelu_approx), L["fc2"],
                             L["fc2_b"]).float()
        return self._ln(x, self.ln_f)

    def embed(self, ids: torch.Tensor, table: int = 0) -> torch.Tensor:
        return self.emb[table][ids.to(self.device).long()].float()


def _pick(logits: torch.Tensor, temp: float | None, gen) -> torch.Tensor:
    if not temp:
        return logits.argmax(-1)
    p = torch.softmax(logits / temp, -1)
    return torch.multinomial(p, 1, generator=gen).squeeze(-1)


class Bark:
    def __init__(self, cfg: dict, sd: dict, device="cpu", dtype=None):
        self.device = torch.device(device)
        self.dtype = dtype or (torch.float16 if self.device.type == "cuda" else torch.float32)
        self.cfg = cfg
        self.g = BarkGen(codebook_size=int(cfg.get("codebook_size", 1024)),
                         sample_rate=int(cfg.get("sample_rate", 24_000)))
        self.semantic = _GPT(sd, "semantic.", cfg["semantic_config"], self.device, self.dtype, True)
        self.coarse = _GPT(sd, "coarse_acoustics.", cfg["coarse_acoustics_config"], self.device, self.dtype, True)
        self.fine = _GPT(sd, "fine_acoustics.", cfg["fine_acoustics_config"], self.device, self.dtype, False)
        self.codec = EncodecDecoder(EncodecConfig.from_dict(cfg["codec_config"]), sd, self.device,
                                    prefix="codec_model.")
        self.tokenizer = None

    # ------------------------------------------------------------------ stage 1: semantic
    def _ar(self, gpt: _GPT, prefix_emb: torch.Tensor, max_new: int, process, temp, gen, stop=None):
        """Autoregressive loop: prefill prefix_emb [1, S, D], then one token per step -> list of ids."""
        S = prefix_emb.shape[1]
        cache = gpt.new_cache(1, S + max_new)
        logits = gpt.forward(prefix_emb, 0, cache)[:, -1]
        if gpt.device.type == "cuda" and max_new > 1:
            return self._ar_graph(gpt, cache, logits, S, max_new, process, temp, gen, stop)
        out = []
        for i in range(max_new):
            nxt = int(_pick(process(logits, len(out)), temp, gen))
            out.append(nxt)
            if stop is not None and nxt == stop:
                break
            if i + 1 == max_new:
                break
            logits = gpt.forward(gpt.embed(torch.tensor([[nxt]])), S + i, cache)[:, -1]
        return out

    def _ar_graph(self, gpt: _GPT, cache, logits, S: int, max_new: int, process, temp, gen, stop, check: int = 32):
        """The decode loop on the GPU without a host round trip per token: each step's transformer is one HIP
        graph replay (decode_step captured once per loop), sampling stays on the device and feeds the next
        step's input buffer; the stop token is looked for every `check` tokens (steps run past it are
        discarded — the same tokens as the eager loop, which stops at the first stop token)."""
        dev = gpt.device
        tok = torch.zeros(1, dtype=torch.long, device=dev)
        pos = torch.full((1,), S, dtype=torch.long, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            gpt.decode_step(tok, pos, cache)  # warm-up outside capture (writes slot S, rewritten by step 0)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out = gpt.decode_step(tok, pos, cache)
        toks = torch.empty(max_new, dtype=torch.long, device=dev)
        n = max_new
        for i in range(max_new):
            nxt = _pick(process(logits, i), temp, gen).view(-1)
            toks[i:i + 1].copy_(nxt)
            if stop is not None and (i % check == check - 1 or i + 1 == max_new):
                hit = (toks[i + 1 - (i % check + 1):i + 1] == stop).nonzero()
                if hit.numel():
                    n = i + 1 - (i % check + 1) + int(hit[0, 0]) + 1
                    break
            if i + 1 == max_new:
                break
            tok.copy_(nxt)
            pos.fill_(S + i)
            graph.replay()
            logits = g_out
        return toks[:n].tolist()

    @torch.no_grad()
    def semantic_tokens(self, text_ids: list[int], history=None, temp=None, gen=None, min_eos_p=None,
                        max_new: int | None = None) -> list[int]:
        g = self.g
        L = g.max_input_semantic_length
        ids = [t + g.text_encoding_offset for t in text_ids[:L]]
        ids = ids + [g.text_pad_token] * (L - len(ids))
        if history is not None:
            hist = [int(v) for v in np.asarray(history["semantic_prompt"])[-L:]]
            hist = hist + [g.eos] * (L - len(hist))
        else:
            hist = [g.eos] * L
        gp = self.semantic
        x = gp.embed(torch.tensor([ids])) + gp.embed(torch.tensor([hist]))
        x = torch.cat([x, gp.embed(torch.tensor([[g.semantic_infer_token]]))], 1)
        V = gp.heads[0].shape[0]
        supp = torch.zeros(V, dtype=torch.bool, device=self.device)
        supp[g.semantic_vocab_size + 1:] = True  # 10 001 .. vocab-1 (10 000 = EOS stays)

        def process(logits, _n):
            lg = logits.masked_fill(supp, float("-inf"))
            if min_eos_p:  # device-side: no host sync per token
                p = torch.softmax(lg, -1)
                only = torch.full_like(lg, float("-inf"))
                only[:, g.eos] = lg[:, g.eos]
                lg = torch.where(p[:, g.eos:g.eos + 1] > min_eos_p, only, lg)
            return lg

        out = self._ar(gp, x, max_new or g.max_semantic_new, process, temp, gen, stop=g.eos)
        return [t for t in out if t != g.eos]

    # ------------------------------------------------------------------ stage 2: coarse
    @torch.no_grad()
    def coarse_tokens(self, semantic: list[int], history=None, temp=None, gen=None) -> np.ndarray:
        """-> [n_coarse, frames] codebook ids (0..codebook_size-1)."""
        g = self.g
        ratio = g.coarse_rate_hz / g.semantic_rate_hz * g.n_coarse
        max_sem_hist = int(np.floor(g.max_coarse_history / ratio))
        n_out = int(round(np.floor(len(semantic) * ratio / g.n_coarse) * g.n_coarse))
        if history is not None:
            sh = [int(v) for v in np.asarray(history["semantic_prompt"])]
            ch = np.asarray(history["coarse_prompt"]).astype(np.int64).copy()
            for n in range(1, ch.shape[0]):
                ch[n] += g.codebook_size * n
            ch = (ch.T.reshape(-1) + g.semantic_vocab_size).tolist()
            n_sem = min(max_sem_hist, len(sh) - len(sh) % 2, int(np.floor(len(ch) / ratio)))
            n_co = int(round(n_sem * ratio))
            sh, ch = sh[len(sh) - n_sem:] if n_sem else [], ch[len(ch) - n_co:] if n_co else []
            ch = ch[:-2]
        else:
            sh, ch = [], []
        base = len(sh)
        sem = sh + semantic
        x_coarse = list(ch)
        len_hist = len(x_coarse)
        total = 0
        gp = self.coarse
        V = gp.heads[0].shape[0]
        band0 = torch.full((V,), float("-inf"), device=self.device)
        band0[g.semantic_vocab_size:g.semantic_vocab_size + g.codebook_size] = 0
        band1 = torch.full((V,), float("-inf"), device=self.device)
        band1[g.semantic_vocab_size + g.codebook_size:] = 0
        for _ in range(int(np.ceil(n_out / g.sliding_window_len))):
            sidx = base + int(round(total / ratio))
            win = sem[max(0, sidx - max_sem_hist):][:g.max_coarse_input_length]
            win = win + [g.coarse_semantic_pad_token] * (g.max_coarse_input_length - len(win))
            inp = win + [g.coarse_infer_token] + x_coarse[-g.max_coarse_history:] if x_coarse else \
                win + [g.coarse_infer_token]
            n_new = min(g.sliding_window_len, n_out - total)
            start = len(inp)

            def process(logits, n, _start=start):
                return logits + (band0 if n % 2 == 0 else band1)  # even -> codebook 0, odd -> 1

            x_coarse += self._ar(gp, gp.embed(torch.tensor([inp])), n_new, process, temp, gen)
            total = len(x_coarse) - len_hist
        out = np.array(x_coarse[len_hist:], dtype=np.int64).reshape(-1, g.n_coarse).T
        return np.remainder(out - g.semantic_vocab_size, g.codebook_size)

    # ------------------------------------------------------------------ stage 3: fine
    @torch.no_grad()
    def fine_tokens(self, coarse: np.ndarray, history=None, temp=None, gen=None) -> np.ndarray:
        """[n_coarse, T] -> [n_fine, T]."""
        g = self.g
        T = coarse.shape[1]
        fine = np.full((T, g.n_fine), g.codebook_size, dtype=np.int64)
        fine[:, :g.n_coarse] = coarse.T
        n_hist = 0
        if history is not None:
            fh = np.asarray(history["fine_prompt"]).T.astype(np.int64)[-g.max_fine_history_length:]
            fine = np.concatenate([fh, fine], 0)
            n_hist = fh.shape[0]
        n_rem = 0
        if fine.shape[0] < g.max_fine_input_length:
            n_rem = g.max_fine_input_length - fine.shape[0]
            fine = np.concatenate([fine, np.full((n_rem, g.n_fine), g.codebook_size, np.int64)], 0)
        n_loops = max(0, int(np.ceil((T - (g.max_fine_input_length - n_hist)) / g.max_fine_history_length))) + 1
        gp = self.fine
        W = g.max_fine_input_length
        for n_outer in range(n_loops):
            s0 = min(n_outer * g.max_fine_history_length, fine.shape[0] - W)
            f0 = min(n_hist + n_outer * g.max_fine_history_length, fine.shape[0] - g.max_fine_history_length)
            rel = f0 - s0
            buf = torch.from_numpy(fine[s0:s0 + W].copy()).to(self.device)
            for ci in range(g.n_coarse, g.n_fine):
                x = sum(gp.embed(buf[None, :, j], j) for j in range(ci + 1))
                logits = gp.forward(x, 0, None, head=ci - 1)[0, :, :g.codebook_size]
                if temp is None or temp == 1.0:
                    pred = logits[rel:].argmax(-1)
                else:
                    p = torch.softmax(logits / temp, -1)[rel:W]
                    pred = torch.multinomial(p, 1, generator=gen).squeeze(-1)
                buf[rel:, ci] = pred
            fine[f0:f0 + (W - rel), g.n_coarse:] = buf[rel:, g.n_coarse:].cpu().numpy()
        fine = fine.T[:, n_hist:]
        if n_rem:
            fine = fine[:, :-n_rem]
        return fine

    # ------------------------------------------------------------------ full pipeline
    @torch.no_grad()
    def generate(self, text_ids: list[int], history=None, text_temp: float | None = 0.7,
                 waveform_temp: float | None = 0.7, seed: int | None = None, min_eos_p: float | None = None,
                 max_semantic: int | None = None) -> np.ndarray:
        """text token ids -> float32 mono waveform at 24 kHz (suno bark defaults: temperature 0.7)."""
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(seed) if seed is not None else int.from_bytes(os.urandom(4), "little"))
        sem = self.semantic_tokens(text_ids, history, text_temp, gen, min_eos_p, max_semantic)
        if not sem:
            raise ValueError("Bark produced no semantic tokens")
        co = self.coarse_tokens(sem, history, waveform_temp, gen)
        fi = self.fine_tokens(co, history, 1.0 if waveform_temp is None else waveform_temp, gen)
        audio = self.codec.decode(torch.from_numpy(fi)[None].to(self.device))
        return audio[0, 0].float().cpu().numpy()

    def tokenize(self, text: str) -> list[int]:
        if self.tokenizer is None:
            raise RuntimeError("no tokenizer (tokenizer.json / vocab.txt) next to the Bark checkpoint")
        return self.tokenizer(text)


def load_voice(path: str) -> dict:
    """suno / HF Bark speaker preset (.npz: semantic_prompt, coarse_prompt, fine_prompt)."""
    with np.load(path, allow_pickle=False) as z:
        return {k: np.asarray(z[k]) for k in ("semantic_prompt", "coarse_prompt", "fine_prompt")}


def _load_tokenizer(d: str):
    p = os.path.join(d, "tokenizer.json")
    if os.path.isfile(p):
        from tokenizers import Tokenizer
        tk = Tokenizer.from_file(p)
        return lambda s: tk.encode(s, add_special_tokens=False).ids
    p = os.path.join(d, "vocab.txt")
    if os.path.isfile(p):
        from tokenizers import Tokenizer, models, normalizers, pre_tokenizers
        vocab = {w.rstrip("\n"): i for i, w in enumerate(open(p, encoding="utf-8"))}
        tk = Tokenizer(models.WordPiece(vocab, unk_token="[UNK]"))
        tk.normalizer = normalizers.BertNormalizer(lowercase=False)
        tk.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
        return lambda s: tk.encode(s).ids
    return None


def load_bark(path: str, device="cpu", dtype=None) -> Bark:
    """A Hugging Face Bark directory (config.json + *.safetensors [+ tokenizer files, speaker_embeddings/])."""
    from safetensors.torch import load_file
    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    if cfg.get("model_type") not in ("bark", None):
        raise ValueError(f"{path}: model_type {cfg.get('model_type')!r} is not bark")
    sd = {}
    for fn in sorted(os.listdir(path)):
        if fn.endswith(".safetensors"):
            sd.update(load_file(os.path.join(path, fn)))
    if not sd:
        raise FileNotFoundError(f"{path}: no .safetensors weights")
    m = Bark(cfg, sd, device, dtype)
    m.tokenizer = _load_tokenizer(path)
    m.path = path
    return m


# ------------------------------------------------------------------------------------------------ synthetic
def synthetic_bark(name: str = "bark-test", device="cpu", seed: int = 0) -> Bark:
    """Random-init Bark of the suno/bark-small (``bark-small``) or a tiny (``bark-test``) architecture."""
    from .musicgen import synthetic_encodec
    if name == "bark-small":
        gpt = dict(num_layers=12, num_heads=12, hidden_size=768)
    elif name == "bark-test":
        gpt = dict(num_layers=2, num_heads=2, hidden_size=32)
    else:
        raise ValueError(f"unknown synthetic Bark {name!r} (have bark-small, bark-test)")
    sem = dict(gpt, block_size=1024, input_vocab_size=129_600, output_vocab_size=10_048, bias=False)
    coa = dict(gpt, block_size=1024, input_vocab_size=12_096, output_vocab_size=12_096, bias=False)
    fin = dict(gpt, block_size=1024, input_vocab_size=1056, output_vocab_size=1056, bias=True, n_codes_total=8,
               n_codes_given=1)
    codec = dict(audio_channels=1, num_filters=32 if name == "bark-small" else 8, upsampling_ratios=[8, 5, 4, 2],
                 hidden_size=128 if name == "bark-small" else 32, codebook_size=1024, num_lstm_layers=2,
                 use_causal_conv=True, pad_mode="reflect", use_conv_shortcut=True, sampling_rate=24000,
                 norm_type="weight_norm")
    cfg = dict(semantic_config=sem, coarse_acoustics_config=coa, fine_acoustics_config=fin, codec_config=codec,
               codebook_size=1024, sample_rate=24000)
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for prefix, c, causal in (("semantic.", sem, True), ("coarse_acoustics.", coa, True),
                              ("fine_acoustics.", fin, False)):
        D = c["hidden_size"]

        def rnd(*shape):
            return torch.randn(*shape, generator=g) / math.sqrt(shape[-1])

        if causal:
            sd[prefix + "input_embeds_layer.weight"] = torch.randn(c["input_vocab_size"], D, generator=g) * 0.5
            sd[prefix + "lm_head.weight"] = rnd(c["output_vocab_size"], D)
        else:
            for i in range(c["n_codes_total"]):
                sd[prefix + f"input_embeds_layers.{i}.weight"] = torch.randn(c["input_vocab_size"], D, generator=g) * .5
            for i in range(c["n_codes_total"] - c["n_codes_given"]):
                sd[prefix + f"lm_heads.{i}.weight"] = rnd(c["output_vocab_size"], D)
        sd[prefix + "position_embeds_layer.weight"] = torch.randn(c["block_size"], D, generator=g) * 0.1
        for i in range(c["num_layers"]):
            L = f"{prefix}layers.{i}."
            for n in ("layernorm_1", "layernorm_2"):
                sd[L + n + ".weight"] = torch.ones(D)
                sd[L + n + ".bias"] = torch.zeros(D)
            sd[L + "attn.att_proj.weight"] = rnd(3 * D, D)
            sd[L + "attn.out_proj.weight"] = rnd(D, D)
            sd[L + "mlp.in_proj.weight"] = rnd(4 * D, D)
            sd[L + "mlp.out_proj.weight"] = rnd(D, 4 * D)
        sd[prefix + "layernorm_final.weight"] = torch.ones(D)
        sd[prefix + "layernorm_final.bias"] = torch.zeros(D)
    sd.update(synthetic_encodec(EncodecConfig.from_dict(codec), 8, g, prefix="codec_model."))
    m = Bark(cfg, sd, device)
    m.tokenizer = lambda s: [100 + (b % 5000) for b in s.encode("utf-8")]
    return m
