"""MusicGen text-to-music (the reference's ``transformers-musicgen`` backend: ``SoundGeneration``,
backend/python/transformers/backend.py:452-507, ElevenLabs-style /v1/sound-generation).

Pipeline (Hugging Face ``MusicgenForConditionalGeneration`` checkpoint names and semantics):

1. T5 text encoder (models/diffusion/text_encoders.py ``T5Encoder``, ``text_encoder.*``) -> hidden states,
   ``enc_to_dec_proj`` when the widths differ. Classifier-free guidance appends a null row (zeros).
2. Decoder: K parallel codebooks; input embedding = sum of K codebook embeddings + sinusoidal positions;
   pre-LN blocks (causal self-attention, cross-attention to the text, GELU MLP), final LayerNorm, K LM heads.
   Codebook k is delayed by k steps (the "delay pattern"): at step t codebook k predicts frame t - k, so
   the first/last k positions of codebook k hold the pad token.
3. Sampling per codebook: CFG logits = uncond + g * (cond - uncond), top-k / temperature (or greedy).
4. EnCodec decoder (models/encodec.py, ``audio_encoder.*``) -> waveform at the codec's sample rate.

MI355X mapping: decode is launch-bound (one token per codebook per step at batch 2), so the whole decoder
step — embedding sum, every layer (self-attention over a preallocated KV cache written at a device-side
position index, cross-attention over K/V projected once per request), heads, CFG combine — is captured
once into a HIP graph and replayed per step; attention masks are built from the device position so the
graph is shape-static. The CPU path runs the same code in fp32 eagerly (the transformers oracle tests
compare against it).
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
from .diffusion.text_encoders import T5Config, T5Encoder
from .encodec import EncodecDecoder, EncodecConfig


@dataclass
class DecoderConfig:
    vocab: int = 2048
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    ffn: int = 4096
    codebooks: int = 4
    max_pos: int = 2048
    act: str = "gelu"
    pad_id: int = 2048
    bos_id: int = 2048
    audio_channels: int = 1

    @classmethod
    def from_hf(cls, d: dict) -> "DecoderConfig":
        if d.get("audio_channels", 1) != 1:
            raise NotImplementedError("stereo MusicGen checkpoints (audio_channels = 2)")
        pad = d.get("pad_token_id", 2048)
        return cls(vocab=d.get("vocab_size", 2048), hidden=d["hidden_size"], layers=d["num_hidden_layers"],
                   heads=d["num_attention_heads"], ffn=d["ffn_dim"], codebooks=d["num_codebooks"],
                   max_pos=d.get("max_position_embeddings", 2048), act=d.get("activation_function", "gelu"),
                   pad_id=pad, bos_id=d.get("bos_token_id", pad) if d.get("bos_token_id") is not None else pad)


def sinusoidal(n: int, dim: int) -> torch.Tensor:
    half = dim // 2
    e = math.log(10000) / (half - 1)
    f = torch.exp(torch.arange(half, dtype=torch.float32) * -e)
    a = torch.arange(n, dtype=torch.float32)[:, None] * f[None, :]
    emb = torch.cat([torch.cos(a), torch.sin(a)], 1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros(n, 1)], 1)
    return emb


def _act(x, name):
    if name == "gelu":
        return F.gelu(x)
    if name in ("gelu_new", "gelu_pytorch_tanh"):
        return F.gelu(x, approximate="tanh")
    if name == "relu":
        return F.relu(x)
    if name == "silu":
        return F.silu(x)
    raise NotImplementedError(f"activation {name!r}")


class MusicgenDecoder:
    def __init__(self, c: DecoderConfig, sd: dict, device, dtype, prefix: str = "decoder."):
        self.c = c
        dev, dt = torch.device(device), dtype
        self.device, self.dtype = dev, dt
        P = prefix + "model.decoder."

        def t(name, d=dt):
            return sd[name].to(dev, d).contiguous()

        self.emb = [t(f"{P}embed_tokens.{k}.weight") for k in range(c.codebooks)]
        self.pos = sinusoidal(c.max_pos, c.hidden).to(dev, torch.float32)
        self.layers = []
        for i in range(c.layers):
            L = f"{P}layers.{i}."
            self.layers.append({
                "ln1": (t(L + "self_attn_layer_norm.weight", torch.float32), t(L + "self_attn_layer_norm.bias", torch.float32)),
                "qkv": torch.cat([t(L + f"self_attn.{n}_proj.weight") for n in "qkv"], 0),
                "o": t(L + "self_attn.out_proj.weight"),
                "ln2": (t(L + "encoder_attn_layer_norm.weight", torch.float32), t(L + "encoder_attn_layer_norm.bias", torch.float32)),
                "xq": t(L + "encoder_attn.q_proj.weight"),
                "xkv": torch.cat([t(L + f"encoder_attn.{n}_proj.weight") for n in "kv"], 0),
                "xo": t(L + "encoder_attn.out_proj.weight"),
                "ln3": (t(L + "final_layer_norm.weight", torch.float32), t(L + "final_layer_norm.bias", torch.float32)),
                "fc1": t(L + "fc1.weight"), "fc2": t(L + "fc2.weight"),
            })
        self.ln_f = (t(P + "layer_norm.weight", torch.float32), t(P + "layer_norm.bias", torch.float32))
        self.heads = torch.stack([t(f"{prefix}lm_heads.{k}.weight") for k in range(c.codebooks)], 0)  # [K, V, D]

    def _ln(self, x, wb):
        return F.layer_norm(x.float(), (x.shape[-1],), wb[0], wb[1], 1e-5).to(self.dtype)

    def cross_kv(self, enc: torch.Tensor):
        """enc [B, S, D] (decoder width) -> per layer (k, v) token-major rows [B*S, D]."""
        B, S, D = enc.shape
        out = []
        e = enc.to(self.dtype)
        for L in self.layers:
            kv = F.linear(e, L["xkv"]).view(B * S, 2 * D)
            out.append((kv[:, :D].contiguous(), kv[:, D:].contiguous()))
        return out

    def new_cache(self, B: int, T: int):
        """Token-major self-attention K / V rows [B, T, D] per layer (attn_dense layout, capacity T)."""
        D = self.c.hidden
        return [(torch.zeros(B, T, D, device=self.device, dtype=self.dtype),
                 torch.zeros(B, T, D, device=self.device, dtype=self.dtype)) for _ in self.layers]

    def step(self, ids: torch.Tensor, pos: torch.Tensor, cache, xkv, xlen) -> torch.Tensor:
        """One decode step. ids [B, K] int64, pos [1] int64 (device); cache from new_cache; xkv from
        cross_kv; xlen int32 [B]: valid encoder keys per row (device) -> logits [B, K, V] fp32. Both attentions
        run on the flash kernel (ops.core.attn_dense) with device-side key lengths, so the step stays
        shape-static for the HIP graph."""
        c = self.c
        B = ids.shape[0]
        D, hd = c.hidden, c.hidden // c.heads
        x = self.pos.index_select(0, pos).expand(B, -1).clone()
        for k in range(c.codebooks):
            x = x + self.emb[k].index_select(0, ids[:, k]).float()
        T = cache[0][0].shape[1]
        S = xkv[0][0].shape[0] // B
        klen = (pos.to(torch.int32) + 1).expand(B).contiguous()  # keys written so far
        a = torch.empty(B, D, dtype=self.dtype, device=x.device)
        for L, (kc, vc), (xk, xv) in zip(self.layers, cache, xkv):
            h = self._ln(x, L["ln1"])
            qkv = F.linear(h, L["qkv"])  # [B, 3D]
            kc.index_copy_(1, pos, qkv[:, None, D:2 * D])
            vc.index_copy_(1, pos, qkv[:, None, 2 * D:])
            attn_dense(qkv, kc.view(-1, D), vc.view(-1, D), a, B, 1, T, c.heads, c.heads, hd, hd ** -0.5,
                         klen=klen, kv_rows=T)
            x = x + F.linear(a, L["o"]).float()
            h = self._ln(x, L["ln2"])
            q = F.linear(h, L["xq"])
            attn_dense(q, xk, xv, a, B, 1, S, c.heads, c.heads, hd, hd ** -0.5, klen=xlen)
            x = x + F.linear(a, L["xo"]).float()
            h = self._ln(x, L["ln3"])
            x = x + F.linear(_act(F.linear(h, L["fc1"]), c.act), L["fc2"]).float()
        h = self._ln(x, self.ln_f)
        return torch.einsum("bd,kvd->bkv", h, self.heads).float()


def delay_pattern(c: DecoderConfig, max_len: int) -> torch.Tensor:
    """[K, max_len] int64: -1 where codebook k may be predicted, pad elsewhere (BOS triangle + EOS triangle);
    column 0 is the BOS/pad column (HF build_delay_pattern_mask with a 1-token prompt)."""
    K = c.codebooks
    pat = torch.full((K, max_len), -1, dtype=torch.long)
    if max_len < 2 * K - 1:
        return pat
    upper = torch.triu(torch.ones(K, max_len, dtype=torch.bool), diagonal=max_len - K + 1)
    lower = torch.tril(torch.ones(K, max_len, dtype=torch.bool))
    pat[upper | lower] = c.pad_id
    return pat


class MusicGen:
    def __init__(self, cfg: dict, sd: dict, device="cpu", dtype=None):
        self.device = torch.device(device)
        self.dtype = dtype or (torch.float16 if self.device.type == "cuda" else torch.float32)
        self.cfg = cfg
        self.t5cfg = T5Config.from_hf(cfg["text_encoder"])
        t5 = T5Encoder(self.t5cfg)
        t5sd = {k[len("text_encoder."):]: v for k, v in sd.items()
                if k.startswith("text_encoder.") and not k.startswith("text_encoder.encoder.embed_tokens")}
        t5.load_state_dict(t5sd, strict=True)
        from .diffusion.nn import cast_module
        # original T5 overflows in f16 (FFN activations): the encoder runs bf16 on the GPU
        self.t5 = cast_module(t5.eval(), self.device,
                              torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.dc = DecoderConfig.from_hf(cfg["decoder"])
        self.proj = None
        if "enc_to_dec_proj.weight" in sd:
            self.proj = (sd["enc_to_dec_proj.weight"].float().to(self.device),
                         sd["enc_to_dec_proj.bias"].float().to(self.device))
        self.decoder = MusicgenDecoder(self.dc, sd, self.device, self.dtype)
        self.codec = EncodecDecoder(EncodecConfig.from_dict(cfg["audio_encoder"]), sd, self.device,
                                    prefix="audio_encoder.")
        self.sample_rate = int(cfg["audio_encoder"].get("sampling_rate", 32000))
        self.tokenizer = None
        self._graph = None

    # ------------------------------------------------------------------ text
    @torch.no_grad()
    def encode_text(self, ids: torch.Tensor | None, mask: torch.Tensor | None, guidance: float):
        if ids is None:  # unconditional (HF get_unconditional_inputs): one zero state, fully masked
            h = torch.zeros(1, 1, self.t5cfg.d_model, device=self.device)
            m = torch.zeros(1, 1, device=self.device)
        else:
            h = self.t5(ids.to(self.device), mask.to(self.device) if mask is not None else None)  # [B, S, D]
            m = mask.to(self.device) if mask is not None else torch.ones(ids.shape, device=self.device)
        if guidance > 1:
            h = torch.cat([h, torch.zeros_like(h)], 0)
            m = torch.cat([m, torch.zeros_like(m)], 0)
        if self.proj is not None:
            h = F.linear(h, self.proj[0], self.proj[1])
        # valid (right-padded) encoder keys per row; a fully masked row (the CFG null row) attends uniformly to
        # all of its keys, as HF's finite-min additive mask makes it do
        n = m.sum(-1).to(torch.int32)
        xlen = torch.where(n > 0, n, torch.full_like(n, m.shape[-1])).contiguous()
        return h, xlen

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def generate_codes(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
                       max_new_tokens: int = 256, guidance_scale: float = 3.0, do_sample: bool = True,
                       top_k: int = 250, temperature: float = 1.0, seed: int | None = None,
                       use_graph: bool | None = None) -> torch.Tensor:
        """input_ids [B, S] T5 ids -> audio codes [B, K, frames] (pad tokens of the delay pattern removed)."""
        c = self.dc
        B = input_ids.shape[0] if input_ids is not None else 1
        K = c.codebooks
        if max_new_tokens < 2 * K:
            raise ValueError(f"max_new_tokens must be >= {2 * K} (delay pattern of {K} codebooks)")
        enc, xlen = self.encode_text(input_ids, attention_mask, guidance_scale)
        BB = enc.shape[0]
        max_len = max_new_tokens + 1
        pat = delay_pattern(c, max_len).to(self.device)
        ids = torch.full((B, K, max_len), -1, dtype=torch.long, device=self.device)
        ids[:, :, 0] = c.bos_id
        cache = self.decoder.new_cache(BB, max_len)
        xkv = self.decoder.cross_kv(enc)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(seed) if seed is not None else int.from_bytes(os.urandom(4), "little"))
        use_graph = (self.device.type == "cuda") if use_graph is None else use_graph
        step_in = torch.zeros(BB, K, dtype=torch.long, device=self.device)
        pos_t = torch.zeros(1, dtype=torch.long, device=self.device)

        def run_step():
            return self.decoder.step(step_in, pos_t, cache, xkv, xlen)

        graph, g_out = None, None
        for t in range(max_len - 1):
            cur = torch.where(pat[None, :, t] == -1, ids[:, :, t], pat[None, :, t])  # delay mask on the input
            step_in.copy_(cur.repeat(BB // B, 1))
            pos_t.fill_(t)
            if use_graph:
                if graph is None:
                    s = torch.cuda.Stream()
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        run_step()  # warm-up (allocations, library handles) outside capture
                    torch.cuda.current_stream().wait_stream(s)
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        g_out = run_step()
                graph.replay()
                logits = g_out
            else:
                logits = run_step()
            if guidance_scale > 1:
                cond, unc = logits[:B], logits[B:]
                logits = unc + (cond - unc) * guidance_scale
            logits = logits.reshape(B * K, -1)
            if do_sample:
                if temperature and temperature != 1.0:
                    logits = logits / temperature
                if top_k and top_k < logits.shape[-1]:
                    kth = torch.topk(logits, top_k, -1).values[:, -1:]
                    logits = logits.masked_fill(logits < kth, float("-inf"))
                probs = torch.softmax(logits, -1)
                nxt = torch.multinomial(probs, 1, generator=gen).view(B, K)
            else:
                nxt = logits.argmax(-1).view(B, K)
            ids[:, :, t + 1] = nxt
        out = torch.where(pat[None] == -1, ids, pat[None])
        # drop the delay-pattern pads: codebook k keeps frames k+1 .. max_len-K+k
        frames = max_len - K
        return torch.stack([out[:, k, k + 1:k + 1 + frames] for k in range(K)], 1)

    @torch.no_grad()
    def decode_audio(self, codes: torch.Tensor) -> torch.Tensor:
        return self.codec.decode(codes)

    def tokenize(self, text: str):
        if self.tokenizer is None:
            raise RuntimeError("no tokenizer (tokenizer.json / spiece.model) next to the MusicGen checkpoint")
        ids = self.tokenizer(text)
        return torch.tensor([ids], dtype=torch.long)

    def generate(self, text: str, duration_s: float | None = None, guidance_scale: float = 3.0,
                 do_sample: bool = True, seed: int | None = None) -> np.ndarray:
        """text -> mono float32 waveform (reference: 256 tokens default, 51.2 tokens per second)."""
        tokens = int(duration_s * 51.2) if duration_s else 256
        codes = self.generate_codes(self.tokenize(text), None, tokens, guidance_scale, do_sample, seed=seed)
        return self.decode_audio(codes)[0, 0].cpu().numpy()


def _load_tokenizer(d: str):
    p = os.path.join(d, "tokenizer.json")
    if os.path.isfile(p):
        from tokenizers import Tokenizer
        tk = Tokenizer.from_file(p)
        return lambda s: tk.encode(s).ids
    p = os.path.join(d, "spiece.model")
    if os.path.isfile(p):
        import sentencepiece as spm
        sp = spm.SentencePieceProcessor(model_file=p)
        return lambda s: sp.encode(s) + [1]  # T5 appends </s> (id 1)
    return None


def load_musicgen(path: str, device="cpu", dtype=None) -> MusicGen:
    """A Hugging Face MusicGen directory (config.json + *.safetensors [+ tokenizer.json / spiece.model])."""
    from safetensors.torch import load_file
    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    if cfg.get("model_type") not in ("musicgen", None):
        raise ValueError(f"{path}: model_type {cfg.get('model_type')!r} is not musicgen")
    sd = {}
    for fn in sorted(os.listdir(path)):
        if fn.endswith(".safetensors"):
            sd.update(load_file(os.path.join(path, fn)))
    if not sd:
        raise FileNotFoundError(f"{path}: no .safetensors weights")
    m = MusicGen(cfg, sd, device, dtype)
    m.tokenizer = _load_tokenizer(path)
    gc = os.path.join(path, "generation_config.json")
    m.generation = json.load(open(gc)) if os.path.isfile(gc) else {}
    return m


# ------------------------------------------------------------------------------------------------ synthetic
SYNTHETIC = {
    # facebook/musicgen-small architecture (t5-base text encoder, 32 kHz EnCodec, 4 codebooks)
    "musicgen-small": dict(
        text_encoder=dict(vocab_size=32128, d_model=768, d_kv=64, d_ff=3072, num_layers=12, num_heads=12,
                          feed_forward_proj="relu", relative_attention_num_buckets=32,
                          relative_attention_max_distance=128, layer_norm_epsilon=1e-6),
        audio_encoder=dict(audio_channels=1, num_filters=64, upsampling_ratios=[8, 5, 4, 4], hidden_size=128,
                           codebook_size=2048, kernel_size=7, last_kernel_size=7, residual_kernel_size=3,
                           dilation_growth_rate=2, num_residual_layers=1, num_lstm_layers=2, compress=2,
                           use_causal_conv=False, pad_mode="reflect", trim_right_ratio=1.0,
                           use_conv_shortcut=False, sampling_rate=32000, norm_type="weight_norm"),
        decoder=dict(vocab_size=2048, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                     ffn_dim=4096, num_codebooks=4, max_position_embeddings=2048, activation_function="gelu",
                     pad_token_id=2048, bos_token_id=2048)),
    "musicgen-test": dict(
        text_encoder=dict(vocab_size=256, d_model=64, d_kv=16, d_ff=128, num_layers=2, num_heads=4,
                          feed_forward_proj="relu"),
        audio_encoder=dict(audio_channels=1, num_filters=8, upsampling_ratios=[4, 2], hidden_size=32,
                           codebook_size=64, num_lstm_layers=2, use_causal_conv=False, pad_mode="reflect",
                           use_conv_shortcut=False, sampling_rate=4000, norm_type="weight_norm"),
        decoder=dict(vocab_size=64, hidden_size=128, num_hidden_layers=2, num_attention_heads=4, ffn_dim=256,
                     num_codebooks=4, max_position_embeddings=512, pad_token_id=64, bos_token_id=64)),
}


def synthetic_state_dict(cfg: dict, seed: int = 0) -> dict:
    """Random-init weights in Hugging Face names for a MusicGen config (no checkpoint download)."""
    g = torch.Generator().manual_seed(seed)

    def rnd(*shape, fan=None):
        fan = fan or shape[-1]
        return torch.randn(*shape, generator=g) / math.sqrt(fan)

    sd = {}
    t5 = T5Encoder(T5Config.from_hf(cfg["text_encoder"]))
    for k, v in t5.state_dict().items():
        sd["text_encoder." + k] = torch.ones_like(v) if k.endswith("layer_norm.weight") else rnd(*v.shape)
    d = DecoderConfig.from_hf(cfg["decoder"])
    P = "decoder.model.decoder."
    for k in range(d.codebooks):
        sd[f"{P}embed_tokens.{k}.weight"] = rnd(d.vocab + 1, d.hidden, fan=d.hidden) * 0.5
        sd[f"decoder.lm_heads.{k}.weight"] = rnd(d.vocab, d.hidden)
    for i in range(d.layers):
        L = f"{P}layers.{i}."
        for a in ("self_attn", "encoder_attn"):
            for n in ("q", "k", "v", "out"):
                sd[f"{L}{a}.{n}_proj.weight"] = rnd(d.hidden, d.hidden)
        for n in ("self_attn_layer_norm", "encoder_attn_layer_norm", "final_layer_norm"):
            sd[f"{L}{n}.weight"] = torch.ones(d.hidden)
            sd[f"{L}{n}.bias"] = torch.zeros(d.hidden)
        sd[L + "fc1.weight"] = rnd(d.ffn, d.hidden)
        sd[L + "fc2.weight"] = rnd(d.hidden, d.ffn)
    sd[P + "layer_norm.weight"] = torch.ones(d.hidden)
    sd[P + "layer_norm.bias"] = torch.zeros(d.hidden)
    te = cfg["text_encoder"]["d_model"]
    if te != d.hidden:
        sd["enc_to_dec_proj.weight"] = rnd(d.hidden, te)
        sd["enc_to_dec_proj.bias"] = torch.zeros(d.hidden)
    sd.update(synthetic_encodec(EncodecConfig.from_dict(cfg["audio_encoder"]), d.codebooks, g))
    return sd


def synthetic_encodec(c: EncodecConfig, n_q: int, g: torch.Generator, prefix: str = "audio_encoder.") -> dict:
    """Random EnCodec decoder + RVQ weights (plain conv weights, no weight-norm split)."""
    sd = {}

    def conv(name, co, ci, k, transpose=False):
        shape = (ci, co, k) if transpose else (co, ci, k)
        sd[name + ".conv.weight"] = torch.randn(*shape, generator=g) / math.sqrt(ci * k)
        sd[name + ".conv.bias"] = torch.zeros(co)

    for q in range(n_q):
        sd[f"{prefix}quantizer.layers.{q}.codebook.embed"] = torch.randn(c.codebook_size, c.hidden_size, generator=g)
    D = f"{prefix}decoder.layers."
    scaling = 2 ** len(c.upsampling_ratios)
    conv(f"{D}0", scaling * c.num_filters, c.hidden_size, c.kernel_size)
    dim = scaling * c.num_filters
    for l in range(c.num_lstm_layers):
        for n, shape in ((f"weight_ih_l{l}", (4 * dim, dim)), (f"weight_hh_l{l}", (4 * dim, dim)),
                         (f"bias_ih_l{l}", (4 * dim,)), (f"bias_hh_l{l}", (4 * dim,))):
            sd[f"{D}1.lstm.{n}"] = torch.randn(*shape, generator=g) / math.sqrt(dim)
    li = 2
    for ratio in c.upsampling_ratios:
        cur = scaling * c.num_filters
        conv(f"{D}{li + 1}", cur // 2, cur, 2 * ratio, transpose=True)
        li += 2
        for _ in range(c.num_residual_layers):
            hid = (cur // 2) // c.compress
            conv(f"{D}{li}.block.1", hid, cur // 2, c.residual_kernel_size)
            conv(f"{D}{li}.block.3", cur // 2, hid, 1)
            if c.use_conv_shortcut:
                conv(f"{D}{li}.shortcut", cur // 2, cur // 2, 1)
            li += 1
        scaling //= 2
    conv(f"{D}{li + 1}", c.audio_channels, c.num_filters, c.last_kernel_size)
    return sd


def synthetic_musicgen(name: str, device="cpu", seed: int = 0) -> MusicGen:
    if name not in SYNTHETIC:
        raise ValueError(f"unknown synthetic MusicGen {name!r} (have {sorted(SYNTHETIC)})")
    cfg = SYNTHETIC[name]
    m = MusicGen(cfg, synthetic_state_dict(cfg, seed), device)
    vocab = cfg["text_encoder"]["vocab_size"]
    m.tokenizer = lambda s: [2 + (b % (vocab - 2)) for b in s.encode("utf-8")] + [1]  # byte stand-in + </s>
    m.generation = {"top_k": 250}
    return m
