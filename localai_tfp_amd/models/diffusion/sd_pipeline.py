"""Text-to-image / image-to-image for UNet (epsilon-prediction) models: SD 1.x / 2.x (one CLIP
text encoder) and SDXL (CLIP-L + CLIP-G, pooled text embedding + size/crop time ids). Reference:
the diffusers backend's StableDiffusionPipeline / StableDiffusionXLPipeline
(backend/python/diffusers/backend.py:169-191) and sd.cpp's txt2img (gosd.cpp:164-226: cfg scale,
steps, seed, sampler / schedule, CLIP skip).

Depth-to-image (the reference's StableDiffusionDepth2ImgPipeline, backend.py:172-173): a UNet with one
input channel more than the VAE latent (SD 2 depth: 5) gets, next to the noisy latent, the source image's
depth map — a DPT depth estimator (transformers DPTForDepthEstimation, the pipeline's depth_estimator/)
run on the image resized to its feature-extractor size, resampled to the latent grid (bicubic) and
normalised to [-1, 1] per image; the latent itself starts from the noised source image (strength) as
in image-to-image.

Sampling uses the shared k-diffusion samplers over the discrete DDPM schedule (samplers.EpsSchedule):
x_in = x / sqrt(sigma^2 + 1), t = t(sigma), x0 = x - sigma * eps; classifier-free guidance runs the
positive and negative branches as one batch of 2 through the UNet, and the text context's
cross-attention K/V are computed once per generation (unet.py).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from ...tokenizer.clip import CLIPTokenizer
from . import samplers as S
from .nn import cast_module, init_synthetic
from .pipeline import GenParams
from .text_encoders import CLIP_G, CLIP_L, CLIPTextConfig, CLIPTextEncoder
from .unet import SD15_UNET, SDXL_UNET, UNET_TEST, UNET_XL_TEST, UNet2DConditionModel, UNetConfig, config_from_diffusers
from .vae import VAE_SD15, AutoencoderKL, VAEConfig


@dataclass
class UNetPreset:
    unet: UNetConfig
    clip_l: CLIPTextConfig
    clip_g: CLIPTextConfig | None  # SDXL second encoder
    vae: VAEConfig
    default_size: int = 512


_T_L = CLIPTextConfig(vocab=600, hidden=32, layers=2, heads=2, ffn=64, proj=32)
_T_G = CLIPTextConfig(vocab=600, hidden=16, layers=2, heads=2, ffn=32, act="gelu", proj=32)
_VAE4_TEST = VAEConfig(latent=4, channels=(32, 32, 64, 64), layers=1, groups=8, scaling=0.18215, shift=0.0,
                       quant_conv=True)
PRESETS = {
    "sd15": UNetPreset(SD15_UNET, CLIP_L, None, VAE_SD15, 512),
    "sdxl": UNetPreset(SDXL_UNET, CLIP_L, CLIP_G, VAEConfig(latent=4, scaling=0.13025, shift=0.0, quant_conv=True),
                       1024),
    "sd15-test": UNetPreset(UNET_TEST, _T_L, None, _VAE4_TEST, 64),
    "sd2-depth-test": UNetPreset(UNetConfig(**{**UNET_TEST.__dict__, "in_channels": 5}), _T_L, None, _VAE4_TEST, 64),
    "sdxl-test": UNetPreset(UNET_XL_TEST, _T_L, _T_G, _VAE4_TEST, 64),
}


class UNetPipeline:
    def __init__(self, preset: UNetPreset, unet: UNet2DConditionModel, te1: CLIPTextEncoder,
                 te2: CLIPTextEncoder | None, vae: AutoencoderKL, tok1: CLIPTokenizer, tok2: CLIPTokenizer | None,
                 device):
        self.p = preset
        self.unet, self.te1, self.te2, self.vae = unet, te1, te2, vae
        self.tok1, self.tok2 = tok1, tok2
        self.device = torch.device(device)
        self.sched = S.EpsSchedule()
        self.depth = None  # (DPT depth estimator, input size, mean, std) for depth-conditioned UNets

    @property
    def xl(self) -> bool:
        return self.te2 is not None

    @property
    def depth_cond(self) -> bool:
        """The UNet takes a depth channel next to the latent (SD 2 depth)."""
        return self.p.unet.in_channels == self.vae.cfg.latent + 1

    def set_depth_estimator(self, model, size: int = 384, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
        self.depth = (model.to(self.device).float().eval(), int(size), torch.tensor(mean).view(1, 3, 1, 1),
                      torch.tensor(std).view(1, 3, 1, 1))
        return self

    @torch.no_grad()
    def depth_map(self, image: torch.Tensor, h: int, w: int) -> torch.Tensor:
        """image [3, H, W] in [0, 1] -> depth [1, 1, h, w] in [-1, 1] (diffusers prepare_depth_map)."""
        if self.depth is None:
            raise ValueError("this depth-conditioned model has no depth estimator (depth_estimator/)")
        m, sz, mean, std = self.depth
        x = F.interpolate(image[None].float(), size=(sz, sz), mode="bicubic", align_corners=False)
        x = ((x - mean) / std).to(self.device)
        d = m(pixel_values=x).predicted_depth[:, None].float()
        d = F.interpolate(d, size=(h, w), mode="bicubic", align_corners=False)
        lo = d.amin(dim=(1, 2, 3), keepdim=True)
        hi = d.amax(dim=(1, 2, 3), keepdim=True)
        return 2.0 * (d - lo) / (hi - lo).clamp_min(1e-6) - 1.0

    # ------------------------------------------------------------------ construction
    @classmethod
    def synthetic(cls, name: str, device, dtype=None, seed: int = 0) -> "UNetPipeline":
        pr = PRESETS[name]
        dev = torch.device(device)
        dtype = dtype or (torch.float16 if dev.type == "cuda" else torch.float32)

        def build(mod, s):
            with torch.device(dev):
                m = mod()
            init_synthetic(m, seed + s)
            return cast_module(m, dev, dtype).eval()
        un = build(lambda: UNet2DConditionModel(pr.unet), 1)
        t1 = build(lambda: CLIPTextEncoder(pr.clip_l, with_projection=False), 2)
        t2 = build(lambda: CLIPTextEncoder(pr.clip_g), 3) if pr.clip_g is not None else None
        vae = build(lambda: AutoencoderKL(pr.vae), 4)
        tk1 = CLIPTokenizer.synthetic(pr.clip_l.vocab)
        tk2 = CLIPTokenizer.synthetic(pr.clip_g.vocab, pad_token="!") if pr.clip_g is not None else None
        pipe = cls(pr, un, t1, t2, vae, tk1, tk2, dev)
        if pipe.depth_cond:  # a tiny random DPT (ViT backbone + reassemble / fusion neck + depth head)
            from transformers import DPTConfig, DPTForDepthEstimation
            torch.manual_seed(seed + 5)
            dc = DPTConfig(hidden_size=32, num_hidden_layers=4, num_attention_heads=2, intermediate_size=64,
                           image_size=64, patch_size=16, backbone_out_indices=[0, 1, 2, 3],
                           neck_hidden_sizes=[8, 16, 32, 32], fusion_hidden_size=16, is_hybrid=False)
            pipe.set_depth_estimator(DPTForDepthEstimation(dc), size=64)
        return pipe

    @classmethod
    def from_diffusers(cls, d: str, device, dtype=None) -> "UNetPipeline":
        """diffusers-layout SD1.x / SD2.x / SDXL directory (unet/, vae/, text_encoder[_2]/, tokenizer[_2]/)."""
        from safetensors.torch import load_file
        dev = torch.device(device)
        dtype = dtype or (torch.float16 if dev.type == "cuda" else torch.float32)

        def cfg_of(sub):
            with open(os.path.join(d, sub, "config.json")) as f:
                return json.load(f)

        def load(m, sub):
            sd = {}
            for fn in sorted(os.listdir(os.path.join(d, sub))):
                if fn.endswith(".safetensors"):
                    sd.update(load_file(os.path.join(d, sub, fn)))
            missing, unexpected = m.load_state_dict(sd, strict=False)
            missing = [k for k in missing if "position_ids" not in k]
            if missing:
                raise ValueError(f"{sub}: missing weights {missing[:5]}")
            return cast_module(m, dev, dtype).eval()
        uc = config_from_diffusers(cfg_of("unet"))
        un = load(UNet2DConditionModel(uc), "unet")

        def clip(sub, proj):
            c = cfg_of(sub)
            cc = CLIPTextConfig(vocab=c["vocab_size"], hidden=c["hidden_size"], layers=c["num_hidden_layers"],
                                heads=c["num_attention_heads"], ffn=c["intermediate_size"],
                                max_pos=c["max_position_embeddings"], act=c.get("hidden_act", "quick_gelu"),
                                proj=c.get("projection_dim", c["hidden_size"]), eps=c.get("layer_norm_eps", 1e-5))
            return load(CLIPTextEncoder(cc, with_projection=proj), sub)
        xl = os.path.isdir(os.path.join(d, "text_encoder_2"))
        t1 = clip("text_encoder", False)
        t2 = clip("text_encoder_2", True) if xl else None
        vc = cfg_of("vae")
        vae = load(AutoencoderKL(VAEConfig(latent=vc["latent_channels"], channels=tuple(vc["block_out_channels"]),
                                           layers=vc["layers_per_block"], groups=vc.get("norm_num_groups", 32),
                                           scaling=vc.get("scaling_factor", 0.18215), shift=vc.get("shift_factor") or 0.0,
                                           quant_conv=vc.get("use_quant_conv", True))), "vae")
        tk1 = CLIPTokenizer.from_dir(os.path.join(d, "tokenizer"))
        tk2 = CLIPTokenizer.from_dir(os.path.join(d, "tokenizer_2"), pad_token="!") if xl else None
        pr = UNetPreset(uc, t1.cfg, t2.cfg if t2 is not None else None, vae.cfg, uc.sample_size * 8)
        pipe = cls(pr, un, t1, t2, vae, tk1, tk2, dev)
        de = os.path.join(d, "depth_estimator")
        if pipe.depth_cond and os.path.isdir(de):
            from transformers import DPTForDepthEstimation
            size, mean, std = 384, (0.5, 0.5, 0.5), (0.5, 0.5, 0.5)
            fe = os.path.join(d, "feature_extractor", "preprocessor_config.json")
            if os.path.isfile(fe):
                with open(fe) as f:
                    pc = json.load(f)
                sz = pc.get("size", 384)
                size = sz.get("height", 384) if isinstance(sz, dict) else int(sz)
                mean, std = pc.get("image_mean", mean), pc.get("image_std", std)
            pipe.set_depth_estimator(DPTForDepthEstimation.from_pretrained(de, local_files_only=True), size, mean, std)
        return pipe

    def set_controlnet(self, path: str, seed: int = 0):
        """diffusers ControlNetModel directory, or `synthetic` (random init with this UNet's config)."""
        from .controlnet import ControlNetModel, controlnet_from_diffusers
        dtype = self.unet.conv_in.weight.dtype
        if path.startswith("synthetic"):
            with torch.device(self.device):
                m = ControlNetModel(self.p.unet)
            init_synthetic(m, seed + 7)
            self.controlnet = cast_module(m, self.device, dtype).eval()
        else:
            self.controlnet = controlnet_from_diffusers(path, self.device, dtype)
        return self

    # ------------------------------------------------------------------ conditioning
    @torch.no_grad()
    def encode_prompts(self, prompts: list[str], clip_skip: int = 0):
        """-> (context [B, 77, D], pooled or None). With prompt weighting on (env COMPEL=1, as the reference's
        diffusers backend, or the pipeline's `compel` attribute) and weighted prompts, per-token weights scale
        each position's offset from the empty-prompt embedding (models/diffusion/prompt_weights.py)."""
        from . import prompt_weights as PW
        if (os.environ.get("COMPEL", "0") == "1" or getattr(self, "compel", False)) and \
                any(PW.has_syntax(p) for p in prompts):
            parts = [PW.weighted_ids(self.tok1, p) for p in prompts]
            h, pooled = self._encode_ids([x[0] for x in parts], [PW.parse(p) for p in prompts], clip_skip)
            he, _ = self._encode_ids([self.tok1("")] * len(prompts), None, clip_skip)
            h = torch.stack([PW.apply(h[b], he[b], parts[b][1]) for b in range(len(prompts))])
            return h, pooled
        return self._encode_ids([self.tok1(p) for p in prompts], None, clip_skip, prompts)

    def _encode_ids(self, ids1: list, chunks, clip_skip: int, prompts: list[str] | None = None):
        dev = self.device
        i1 = torch.tensor(ids1, device=dev)
        if not self.xl:
            # SD1.x/2.x: last hidden state through the final LayerNorm (clip_skip N: layer -(N+1), normed)
            h, _ = self.te1(i1, self.tok1.eos, max(0, clip_skip - 1) if clip_skip > 1 else 0)
            if clip_skip > 1:
                tm = self.te1.text_model
                h = F.layer_norm(h, (h.shape[-1],), tm.final_layer_norm.weight.float(),
                                 tm.final_layer_norm.bias.float(), self.te1.cfg.eps)
            return h, None
        # SDXL: penultimate hidden states of both encoders (no final LN), pooled from CLIP-G
        skip = 1 + max(0, clip_skip - 1)
        h1, _ = self.te1(i1, self.tok1.eos, skip)
        if chunks is not None:  # weighted prompts: CLIP-G sees the same syntax-free text
            from . import prompt_weights as PW
            i2 = torch.tensor([PW.weighted_ids(self.tok2, "".join(t for t, _ in c))[0] for c in chunks], device=dev)
        elif prompts is not None:
            i2 = torch.tensor([self.tok2(p) for p in prompts], device=dev)
        else:
            i2 = torch.tensor([self.tok2("")] * len(ids1), device=dev)
        h2, pooled = self.te2(i2, self.tok2.eos, skip)
        return torch.cat([h1, h2], -1), pooled

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def generate(self, prompt: str, gp: GenParams, init_image: torch.Tensor | None = None) -> torch.Tensor:
        """-> image [3, H, W] in [0, 1] (fp32, CPU)."""
        dev = self.device
        W, H = (gp.width // 8) * 8, (gp.height // 8) * 8
        ctx, pooled = self.encode_prompts([prompt, gp.negative], gp.extra.get("clip_skip", 0))
        gen = torch.Generator(device=dev).manual_seed(int(gp.seed) & 0x7FFFFFFFFFFFFFFF)
        dmap = None
        if self.depth_cond:
            if init_image is None:
                raise ValueError("depth-to-image needs a source image (src)")
            dmap = self.depth_map(init_image, H // 8, W // 8).to(dev).expand(2, -1, -1, -1)
        shape = (1, self.vae.cfg.latent, H // 8, W // 8)
        sig = S.get_sigmas(self.sched, gp.steps, gp.schedule)
        noise = torch.randn(shape, generator=gen, device=dev, dtype=torch.float32)
        if init_image is not None:
            x0 = self.vae.encode(init_image.to(dev)[None] * 2 - 1)
            x0 = F.interpolate(x0, size=shape[2:], mode="bilinear") if x0.shape[2:] != shape[2:] else x0
            k = min(len(sig) - 2, int(round((1 - gp.strength) * (len(sig) - 1))))
            sig = sig[k:]
            x = x0 + noise * sig[0]
        else:
            x = noise * sig[0]
        cfg = float(gp.cfg_scale)
        added = None
        if self.xl:
            tid = torch.tensor([[H, W, 0, 0, H, W]], dtype=torch.float32, device=dev)
            added = {"text_embeds": pooled, "time_ids": tid.expand(2, 6)}
        ctx_key = ctx
        cn = getattr(self, "controlnet", None)
        cimg = gp.extra.get("control_image")
        if cn is not None and cimg is not None:
            cimg = F.interpolate(cimg[None].float(), size=(H, W), mode="bilinear") if cimg.shape[1:] != (H, W) \
                else cimg[None].float()
            cimg = cimg.to(dev).expand(2, -1, -1, -1)
        cscale = float(gp.extra.get("control_scale", 1.0))

        def denoise(xt: torch.Tensor, sigma: float) -> torch.Tensor:
            xin = torch.cat([xt, xt]) / math.sqrt(sigma * sigma + 1.0)
            if dmap is not None:  # the depth channel rides unscaled next to the scaled latent
                xin = torch.cat([xin, dmap.to(xin.dtype)], 1)
            t = torch.full((2,), self.sched.t_of(sigma), device=dev)
            ctl = cn(xin, t, ctx, cimg, cscale, added, ctx_key) if cn is not None and cimg is not None else None
            eps = self.unet(xin, t, ctx, added, ctx_key, control=ctl)
            e = eps[1:] + cfg * (eps[:1] - eps[1:])
            return xt - sigma * e
        x = S.sample(denoise, x, sig, gp.sampler, flow=False, generator=gen)
        img = self.vae.decode(x)[0]
        return ((img + 1) / 2).clamp(0, 1).cpu()
