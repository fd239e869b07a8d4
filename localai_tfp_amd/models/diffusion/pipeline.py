"""Text-to-image / image-to-image pipeline for SD3-class models (MMDiT + CLIP-L + CLIP-G [+ T5-XXL]
+ 16-channel VAE). Reference behaviour: gosd.cpp gen_image (txt2img with cfg scale, steps, seed,
sampler/schedule options, PNG output; gosd.cpp:164-226) and the diffusers backend's SD3 pipeline
(negative prompt, img2img strength).

Classifier-free guidance runs the conditional and unconditional branches as one batch of 2 through
the transformer. Components load from a diffusers-layout directory (safetensors) or are
random-initialised directly on the GPU for `synthetic:` models.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from ...tokenizer.clip import CLIPTokenizer, T5Tokenizer
from . import samplers as S
from .mmdit import MMDIT_TEST, MMDITX_TEST, SD3_MEDIUM, SD35_LARGE, SD35_MEDIUM, MMDiT, MMDiTConfig
from .nn import cast_module, init_synthetic
from .text_encoders import CLIP_G, CLIP_L, T5_XXL, CLIPTextConfig, CLIPTextEncoder, T5Config, T5Encoder
from .vae import VAE_SD3, VAE_TEST, AutoencoderKL, VAEConfig


@dataclass
class SD3Preset:
    mmdit: MMDiTConfig
    clip_l: CLIPTextConfig
    clip_g: CLIPTextConfig
    t5: T5Config | None
    vae: VAEConfig
    t5_tokens: int = 256


_CLIP_T1 = CLIPTextConfig(vocab=600, hidden=32, layers=2, heads=2, ffn=64, proj=32)
_CLIP_T2 = CLIPTextConfig(vocab=600, hidden=32, layers=2, heads=2, ffn=64, act="gelu", proj=32)
_T5_T = T5Config(vocab=300, d_model=64, heads=2, d_kv=32, d_ff=128, layers=2)
# quantisation tests: every GEMM dimension a multiple of 256 so GGUF block weights stay quantised
_CLIP_Q1 = CLIPTextConfig(vocab=600, hidden=256, layers=2, heads=4, ffn=512, proj=256)
_CLIP_Q2 = CLIPTextConfig(vocab=600, hidden=256, layers=2, heads=4, ffn=512, act="gelu", proj=256)
_T5_Q = T5Config(vocab=300, d_model=512, heads=4, d_kv=64, d_ff=512, layers=2)
_MMDITX_Q = MMDiTConfig(layers=3, heads=4, joint_dim=512, caption_dim=256, pooled_dim=512, pos_max=32, sample_size=16,
                        qk_norm=True, dual_attention_layers=(0, 1))
PRESETS = {
    "sd3-medium": SD3Preset(SD3_MEDIUM, CLIP_L, CLIP_G, T5_XXL, VAE_SD3),
    "sd3-medium-no-t5": SD3Preset(SD3_MEDIUM, CLIP_L, CLIP_G, None, VAE_SD3),
    "sd3.5-medium": SD3Preset(SD35_MEDIUM, CLIP_L, CLIP_G, T5_XXL, VAE_SD3),
    "sd3.5-large": SD3Preset(SD35_LARGE, CLIP_L, CLIP_G, T5_XXL, VAE_SD3),
    "sd3-test": SD3Preset(MMDIT_TEST, _CLIP_T1, _CLIP_T2, _T5_T, VAE_TEST, t5_tokens=16),
    "sd3.5m-test": SD3Preset(MMDITX_TEST, _CLIP_T1, _CLIP_T2, _T5_T, VAE_TEST, t5_tokens=16),
    "sd3.5m-qtest": SD3Preset(_MMDITX_Q, _CLIP_Q1, _CLIP_Q2, _T5_Q, VAE_TEST, t5_tokens=16),
}


@dataclass
class GenParams:
    width: int = 512
    height: int = 512
    steps: int = 20
    cfg_scale: float = 7.0
    seed: int = 0
    sampler: str = "euler"
    schedule: str = "default"
    strength: float = 0.75
    negative: str = ""
    extra: dict = field(default_factory=dict)


class SD3Pipeline:
    def __init__(self, preset: SD3Preset, mmdit: MMDiT, clip_l: CLIPTextEncoder, clip_g: CLIPTextEncoder,
                 t5: T5Encoder | None, vae: AutoencoderKL, tok_l: CLIPTokenizer, tok_g: CLIPTokenizer,
                 tok_t5: T5Tokenizer | None, device, shift: float = 3.0):
        self.p = preset
        self.mmdit, self.clip_l, self.clip_g, self.t5, self.vae = mmdit, clip_l, clip_g, t5, vae
        self.tok_l, self.tok_g, self.tok_t5 = tok_l, tok_g, tok_t5
        self.device = torch.device(device)
        self.sched = S.FlowSchedule(shift)
        self.mmdit.prepare()

    # ------------------------------------------------------------------ construction
    @classmethod
    def synthetic(cls, name: str, device, dtype=None, seed: int = 0) -> "SD3Pipeline":
        pr = PRESETS[name]
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)

        def build(mod, s):
            with torch.device(dev):
                m = mod()
            init_synthetic(m, seed + s)
            return cast_module(m, dev, dtype).eval()
        mm = build(lambda: MMDiT(pr.mmdit), 1)
        cl = build(lambda: CLIPTextEncoder(pr.clip_l), 2)
        cg = build(lambda: CLIPTextEncoder(pr.clip_g), 3)
        t5 = build(lambda: T5Encoder(pr.t5), 4) if pr.t5 is not None else None
        vae = build(lambda: AutoencoderKL(pr.vae), 5)
        tl = CLIPTokenizer.synthetic(pr.clip_l.vocab)
        tg = CLIPTokenizer.synthetic(pr.clip_g.vocab)
        tt = T5Tokenizer(None, pr.t5.vocab, pr.t5_tokens) if pr.t5 is not None else None
        return cls(pr, mm, cl, cg, t5, vae, tl, tg, tt, dev)

    @classmethod
    def from_diffusers(cls, d: str, device, dtype=None, use_t5: bool = True) -> "SD3Pipeline":
        """Load a diffusers-layout SD3 directory (model_index.json + component folders)."""
        from safetensors.torch import load_file
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)

        def cfg_of(sub):
            with open(os.path.join(d, sub, "config.json")) as f:
                return json.load(f)

        def weights(sub):
            sd = {}
            for fn in sorted(os.listdir(os.path.join(d, sub))):
                if fn.endswith(".safetensors"):
                    sd.update(load_file(os.path.join(d, sub, fn)))
            return sd

        def load(m, sub):
            sd = weights(sub)
            missing, unexpected = m.load_state_dict(sd, strict=False)
            missing = [k for k in missing if not k.endswith("pos_embed.pos_embed")]
            if missing:
                raise ValueError(f"{sub}: missing weights {missing[:5]}")
            return cast_module(m, dev, dtype).eval()
        tc = cfg_of("transformer")
        mc = MMDiTConfig(patch=tc.get("patch_size", 2), in_channels=tc.get("in_channels", 16),
                         out_channels=tc.get("out_channels", 16), layers=tc["num_layers"],
                         head_dim=tc["attention_head_dim"], heads=tc["num_attention_heads"],
                         joint_dim=tc["joint_attention_dim"], caption_dim=tc["caption_projection_dim"],
                         pooled_dim=tc["pooled_projection_dim"], pos_max=tc.get("pos_embed_max_size", 192),
                         sample_size=tc.get("sample_size", 128), qk_norm=tc.get("qk_norm") is not None)
        mm = load(MMDiT(mc), "transformer")

        def clip(sub):
            c = cfg_of(sub)
            cc = CLIPTextConfig(vocab=c["vocab_size"], hidden=c["hidden_size"], layers=c["num_hidden_layers"],
                                heads=c["num_attention_heads"], ffn=c["intermediate_size"],
                                max_pos=c["max_position_embeddings"], act=c.get("hidden_act", "quick_gelu"),
                                proj=c.get("projection_dim", c["hidden_size"]), eps=c.get("layer_norm_eps", 1e-5))
            return load(CLIPTextEncoder(cc), sub)
        cl, cg = clip("text_encoder"), clip("text_encoder_2")
        t5 = tt = None
        if use_t5 and os.path.isdir(os.path.join(d, "text_encoder_3")):
            c = cfg_of("text_encoder_3")
            t5 = load(T5Encoder(T5Config(vocab=c["vocab_size"], d_model=c["d_model"], heads=c["num_heads"],
                                         d_kv=c["d_kv"], d_ff=c["d_ff"], layers=c["num_layers"],
                                         buckets=c.get("relative_attention_num_buckets", 32),
                                         max_distance=c.get("relative_attention_max_distance", 128))),
                      "text_encoder_3")
            tt = T5Tokenizer.from_file(os.path.join(d, "tokenizer_3", "spiece.model"))
        vc = cfg_of("vae")
        vae = load(AutoencoderKL(VAEConfig(latent=vc["latent_channels"], channels=tuple(vc["block_out_channels"]),
                                           layers=vc["layers_per_block"], groups=vc.get("norm_num_groups", 32),
                                           scaling=vc.get("scaling_factor", 1.5305),
                                           shift=vc.get("shift_factor") or 0.0,
                                           quant_conv=vc.get("use_quant_conv", False))), "vae")
        tl = CLIPTokenizer.from_dir(os.path.join(d, "tokenizer"))
        tg = CLIPTokenizer.from_dir(os.path.join(d, "tokenizer_2"), pad_token="!")
        sh = 3.0
        sp = os.path.join(d, "scheduler", "scheduler_config.json")
        if os.path.exists(sp):
            with open(sp) as f:
                sh = json.load(f).get("shift", 3.0)
        preset = SD3Preset(mc, cl.cfg, cg.cfg, t5.cfg if t5 is not None else None, vae.cfg)
        return cls(preset, mm, cl, cg, t5, vae, tl, tg, tt, dev, shift=sh)

    # ------------------------------------------------------------------ text conditioning
    @torch.no_grad()
    def encode_prompts(self, prompts: list[str], clip_skip: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
        dev = self.device
        skip = max(1, clip_skip or 1)
        il = torch.tensor([self.tok_l(p) for p in prompts], device=dev)
        ig = torch.tensor([self.tok_g(p) for p in prompts], device=dev)
        hl, pl = self.clip_l(il, self.tok_l.eos, skip)
        hg, pg = self.clip_g(ig, self.tok_g.eos, skip)
        jd = self.p.mmdit.joint_dim
        clip = torch.cat([hl, hg], -1)
        clip = F.pad(clip, (0, jd - clip.shape[-1]))
        if self.t5 is not None:
            it = torch.tensor([self.tok_t5(p) for p in prompts], device=dev)
            t5 = self.t5(it)
        else:
            t5 = torch.zeros(len(prompts), self.p.t5_tokens, jd, device=dev)
        return torch.cat([clip, t5], 1), torch.cat([pl, pg], -1)

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def generate(self, prompt: str, gp: GenParams, init_image: torch.Tensor | None = None) -> torch.Tensor:
        """-> image [3, H, W] in [0, 1] (fp32, CPU)."""
        dev = self.device
        W, H = (gp.width // 16) * 16, (gp.height // 16) * 16
        ctx, pooled = self.encode_prompts([prompt, gp.negative], gp.extra.get("clip_skip", 0))
        gen = torch.Generator(device=dev).manual_seed(int(gp.seed) & 0x7FFFFFFFFFFFFFFF)
        C = self.p.mmdit.in_channels
        shape = (1, C, H // 8, W // 8)
        sig = S.get_sigmas(self.sched, gp.steps, gp.schedule)
        noise = torch.randn(shape, generator=gen, device=dev, dtype=torch.float32)
        if init_image is not None:
            x0 = self.vae.encode(init_image.to(dev)[None] * 2 - 1)
            x0 = F.interpolate(x0, size=shape[2:], mode="bilinear") if x0.shape[2:] != shape[2:] else x0
            k = min(len(sig) - 2, int(round((1 - gp.strength) * (len(sig) - 1))))
            sig = sig[k:]
            x = (1 - sig[0]) * x0 + sig[0] * noise
        else:
            x = noise * sig[0]
        cfg = float(gp.cfg_scale)

        def denoise(xt: torch.Tensor, sigma: float) -> torch.Tensor:
            xin = torch.cat([xt, xt]) if cfg != 1.0 else xt
            t = torch.full((xin.shape[0],), sigma * 1000.0, device=dev)
            n = xin.shape[0]
            v = self.mmdit(xin, t, ctx[:n], pooled[:n])
            if cfg != 1.0:
                v = v[1:] + cfg * (v[:1] - v[1:])
            return xt - sigma * v
        x = S.sample(denoise, x, sig, gp.sampler, flow=True, generator=gen)
        img = self.vae.decode(x)[0]
        return ((img + 1) / 2).clamp(0, 1).cpu()


def save_png(img: torch.Tensor, path: str) -> str:
    from PIL import Image
    a = (img.permute(1, 2, 0).numpy() * 255.0 + 0.5).clip(0, 255).astype(np.uint8)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    Image.fromarray(a).save(path, format="PNG")
    return path


def load_image(path: str, width: int, height: int) -> torch.Tensor:
    from PIL import Image
    im = Image.open(path).convert("RGB").resize((width, height))
    return torch.from_numpy(np.asarray(im, np.float32) / 255.0).permute(2, 0, 1).contiguous()
