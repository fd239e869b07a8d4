"""stable-diffusion.cpp-style checkpoints: ONE file holding a model in its original training-code
names — .safetensors, .ckpt or a GGUF with quantised tensors — plus optional separate component files
given by the model options `clip_l_path`, `clip_g_path`, `t5xxl_path`, `vae_path`. Reference:
backend/go/image/stablediffusion-ggml/gosd.cpp:56-162 (new_sd_ctx with those paths); the gallery's
sd-ggml / flux-ggml configs (SD1.5 Q4_0 GGUF, Flux.1-dev Q2_K GGUF + ae / clip_l / t5xxl files).

Families are recognised by their tensor names and mapped onto this framework's (diffusers-layout)
modules:
* Flux.1 (Black Forest Labs names: img_in, double_blocks.*, single_blocks.*, final_layer): fused
  img/txt qkv and the single-block linear1 are split into q / k / v (/ mlp), the final adaLN's
  (shift, scale) halves swapped to diffusers' (scale, shift);
* SD1.x / SD2.x / SDXL (CompVis LDM / SGM UNet names under model.diffusion_model., via sgm_names);
  CLIP-L from cond_stage_model.transformer. / conditioner.embedders.0.transformer., OpenCLIP-G
  (conditioner.embedders.1.model.: fused in_proj split, c_fc / c_proj, transposed text_projection);
* SD3 / SD3.5-large (Stability MMDiT names: joint_blocks.i.{x,context}_block, fused qkv, pre-only
  last context block, ln_q / ln_k QK-norm) with text_encoders.{clip_l,clip_g,t5xxl}.transformer.*;
* LDM VAE (first_stage_model. or a bare ae.safetensors): down/up/mid blocks renamed, up blocks
  reversed, 1x1-conv attention weights flattened to linears.
GGUF block-quantised matrices (Q4_0 / Q5_0 / Q8_0 / Q4_K / Q6_K / Q2_K ... with K % 256 == 0) stay
quantised: they travel through the name mapping as `GGMLTensor`s (row slices and row concatenations act
on the ggml bytes) and every nn.Linear weight among them becomes a `nn.QParam` run by the quantised
GEMM; only non-linear tensors (embeddings, convolutions, norms) are dequantised at load.
Tokenizer files (CLIP vocab.json + merges.txt, T5 spiece.model) are searched next to the model and
component files; without them a byte-level stand-in is used and a warning logged.
"""
from __future__ import annotations

import logging
import os
import re

import numpy as np
import torch

log = logging.getLogger("localai_tfp_amd.diffusion")


# ---------------------------------------------------------------- reading
class GGMLTensor:
    """A GGUF block-quantised [N, K] matrix in its ggml row bytes. Supports what the name mappings do to
    weights — `.shape`, row slices, `torch.cat` along rows — without dequantising; anything else
    (a reshape, arithmetic) dequantises to fp32 first."""

    def __init__(self, raw: np.ndarray, qtype: int, n: int, k: int):
        self.raw, self.qtype, self.n, self.k = raw.reshape(n, -1), int(qtype), int(n), int(k)

    @property
    def shape(self):
        return torch.Size((self.n, self.k))

    ndim = 2

    def dim(self) -> int:
        return 2

    def contiguous(self):
        return self

    def dense(self) -> torch.Tensor:
        from ...ops.quant import dequantize
        return torch.from_numpy(np.ascontiguousarray(dequantize(self.raw, self.qtype, (self.k, self.n))).reshape(
            self.n, self.k).copy())

    def __getitem__(self, idx):
        if isinstance(idx, slice) and idx.step in (None, 1):
            r = self.raw[idx]
            return GGMLTensor(r, self.qtype, r.shape[0], self.k)
        return self.dense()[idx]

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is torch.cat and kwargs.get("dim", args[1] if len(args) > 1 else 0) == 0:
            parts = list(args[0])
            if all(isinstance(p, GGMLTensor) and p.qtype == parts[0].qtype and p.k == parts[0].k for p in parts):
                raw = np.concatenate([p.raw for p in parts], 0)
                return GGMLTensor(raw, parts[0].qtype, raw.shape[0], parts[0].k)

        def dq(a):
            if isinstance(a, GGMLTensor):
                return a.dense()
            if isinstance(a, (list, tuple)):
                return type(a)(dq(x) for x in a)
            return a
        return func(*dq(tuple(args)), **{k: dq(v) for k, v in kwargs.items()})

    def __getattr__(self, name):  # any other tensor method: on the dequantised matrix
        if name.startswith("__"):
            raise AttributeError(name)
        return getattr(self.dense(), name)


def _keep_quant(ti) -> bool:
    from ...formats.gguf import QType
    from ...ops import quant as Q
    q = QType(ti.qtype)
    return (len(ti.shape) == 2 and ti.shape[0] % 256 == 0 and
            q in (*Q.GPU_NATIVE, *Q.Q8_EXACT, *Q.Q8_REQUANT))


def read_tensors(path: str, keep_quant: bool = False) -> dict[str, torch.Tensor]:
    """All tensors of a .safetensors / .gguf / .ckpt|.pt file. GGUF block formats: fp32, or with
    keep_quant GGMLTensors for the matrices a quantised GEMM can run (see _keep_quant)."""
    if path.endswith(".safetensors"):
        from safetensors import safe_open
        out = {}
        with safe_open(path, framework="pt") as f:
            for k in f.keys():
                out[k] = f.get_tensor(k)
        return out
    if path.endswith(".gguf"):
        from ...formats.gguf import GGUFReader
        from ...ops.quant import dequantize
        r = GGUFReader(path)
        out = {}
        for name, ti in r.tensors.items():
            if keep_quant and _keep_quant(ti):
                out[name] = GGMLTensor(np.array(r.tensor_bytes(name)), ti.qtype, ti.shape[1], ti.shape[0])
                continue
            a = dequantize(r.tensor_bytes(name), ti.qtype, ti.shape)
            out[name] = torch.from_numpy(np.ascontiguousarray(a).reshape(tuple(reversed(ti.shape))).copy())
        return out
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd:
        sd = sd["state_dict"]
    return dict(sd)


def strip(sd: dict, prefix: str) -> dict:
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


def detect(sd: dict) -> str:
    keys = sd.keys()
    if any(k.startswith(("double_blocks.", "model.diffusion_model.double_blocks.")) for k in keys):
        return "flux"
    if any(".joint_blocks." in k or k.startswith("joint_blocks.") for k in keys):
        return "sd3"
    if any(k.startswith("model.diffusion_model.label_emb.") for k in keys):
        return "sdxl"
    if any(k.startswith("model.diffusion_model.input_blocks.") for k in keys):
        return "sd1"
    raise ValueError("unrecognised single-file diffusion checkpoint (no Flux / SD3 / SD UNet tensor names)")


# ---------------------------------------------------------------- LDM VAE
def ldm_vae_to_diffusers(sd: dict) -> dict:
    """first_stage_model.* (prefix already stripped) / ae.safetensors names -> AutoencoderKL names."""
    n_up = 1 + max((int(m.group(1)) for k in sd for m in [re.match(r"decoder\.up\.(\d+)\.", k)] if m), default=-1)
    out = {}
    res = {"nin_shortcut": "conv_shortcut"}
    attn = {"norm": "group_norm", "q": "to_q", "k": "to_k", "v": "to_v", "proj_out": "to_out.0"}
    for k, v in sd.items():
        nk = None
        m = re.match(r"(encoder|decoder)\.(.*)$", k)
        if m:
            side, rest = m.groups()
            mm = re.match(r"down\.(\d+)\.block\.(\d+)\.(\w+)\.(weight|bias)$", rest)
            mu = re.match(r"up\.(\d+)\.block\.(\d+)\.(\w+)\.(weight|bias)$", rest)
            if mm:
                nk = f"{side}.down_blocks.{mm[1]}.resnets.{mm[2]}.{res.get(mm[3], mm[3])}.{mm[4]}"
            elif mu:
                nk = f"{side}.up_blocks.{n_up - 1 - int(mu[1])}.resnets.{mu[2]}.{res.get(mu[3], mu[3])}.{mu[4]}"
            elif re.match(r"down\.(\d+)\.downsample\.conv\.", rest):
                i = rest.split(".")[1]
                nk = f"{side}.down_blocks.{i}.downsamplers.0.conv.{rest.split('.')[-1]}"
            elif re.match(r"up\.(\d+)\.upsample\.conv\.", rest):
                i = int(rest.split(".")[1])
                nk = f"{side}.up_blocks.{n_up - 1 - i}.upsamplers.0.conv.{rest.split('.')[-1]}"
            elif (mb := re.match(r"mid\.block_(\d)\.(\w+)\.(weight|bias)$", rest)):
                nk = f"{side}.mid_block.resnets.{int(mb[1]) - 1}.{res.get(mb[2], mb[2])}.{mb[3]}"
            elif (ma := re.match(r"mid\.attn_1\.(\w+)\.(weight|bias)$", rest)):
                nk = f"{side}.mid_block.attentions.0.{attn[ma[1]]}.{ma[2]}"
                if ma[1] != "norm" and v.dim() == 4:
                    v = v[:, :, 0, 0]
            elif rest.startswith("norm_out."):
                nk = f"{side}.conv_norm_out.{rest.split('.')[-1]}"
            elif rest.startswith(("conv_in.", "conv_out.")):
                nk = f"{side}.{rest}"
        elif k.startswith(("quant_conv.", "post_quant_conv.")):
            nk = k
        if nk is not None:
            out[nk] = v
    return out


def vae_config_from(sd: dict, scaling: float, shift: float):
    from .vae import VAEConfig
    lat = int(sd["decoder.conv_in.weight"].shape[1])
    levels = sorted({int(m.group(1)) for k in sd for m in [re.match(r"encoder\.down_blocks\.(\d+)\.resnets", k)] if m})
    ch = tuple(int(sd[f"encoder.down_blocks.{i}.resnets.0.conv1.weight"].shape[0]) for i in levels)
    layers = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"encoder\.down_blocks\.0\.resnets\.(\d+)\.", k)] if m)
    return VAEConfig(latent=lat, channels=ch, layers=layers, groups=32, scaling=scaling, shift=shift,
                     quant_conv="quant_conv.weight" in sd)


# ---------------------------------------------------------------- Flux (BFL names)
def bfl_flux_to_diffusers(sd: dict) -> dict:
    sd = strip(sd, "model.diffusion_model.") or sd
    d = int(sd["img_in.weight"].shape[0])
    top = {"img_in": "x_embedder", "txt_in": "context_embedder",
           "time_in.in_layer": "time_text_embed.timestep_embedder.linear_1",
           "time_in.out_layer": "time_text_embed.timestep_embedder.linear_2",
           "vector_in.in_layer": "time_text_embed.text_embedder.linear_1",
           "vector_in.out_layer": "time_text_embed.text_embedder.linear_2",
           "guidance_in.in_layer": "time_text_embed.guidance_embedder.linear_1",
           "guidance_in.out_layer": "time_text_embed.guidance_embedder.linear_2",
           "final_layer.linear": "proj_out"}
    dbl = {"img_mod.lin": "norm1.linear", "txt_mod.lin": "norm1_context.linear", "img_attn.proj": "attn.to_out.0",
           "txt_attn.proj": "attn.to_add_out", "img_mlp.0": "ff.net.0.proj", "img_mlp.2": "ff.net.2",
           "txt_mlp.0": "ff_context.net.0.proj", "txt_mlp.2": "ff_context.net.2",
           "img_attn.norm.query_norm.scale": "attn.norm_q.weight", "img_attn.norm.key_norm.scale": "attn.norm_k.weight",
           "txt_attn.norm.query_norm.scale": "attn.norm_added_q.weight",
           "txt_attn.norm.key_norm.scale": "attn.norm_added_k.weight"}
    sgl = {"linear2": "proj_out", "modulation.lin": "norm.linear", "norm.query_norm.scale": "attn.norm_q.weight",
           "norm.key_norm.scale": "attn.norm_k.weight"}
    out = {}
    for k, v in sd.items():
        stem, _, leaf = k.rpartition(".")
        if stem in top:
            out[f"{top[stem]}.{leaf}"] = v
        elif stem == "final_layer.adaLN_modulation.1":  # BFL (shift, scale) -> diffusers (scale, shift)
            out[f"norm_out.linear.{leaf}"] = torch.cat([v[d:], v[:d]], 0)
        elif (m := re.match(r"double_blocks\.(\d+)\.(.+)$", k)):
            i, rest = m.groups()
            b = f"transformer_blocks.{i}."
            if rest in dbl:
                out[b + dbl[rest]] = v
            elif rest.rpartition(".")[0] in dbl:
                s, _, lf = rest.rpartition(".")
                out[b + dbl[s] + "." + lf] = v
            elif rest.startswith(("img_attn.qkv.", "txt_attn.qkv.")):
                lf = rest.rpartition(".")[2]
                names = ("to_q", "to_k", "to_v") if rest.startswith("img") else ("add_q_proj", "add_k_proj", "add_v_proj")
                for j, nm in enumerate(names):
                    out[f"{b}attn.{nm}.{lf}"] = v[j * d:(j + 1) * d]
        elif (m := re.match(r"single_blocks\.(\d+)\.(.+)$", k)):
            i, rest = m.groups()
            b = f"single_transformer_blocks.{i}."
            if rest in sgl:
                out[b + sgl[rest]] = v
            elif rest.rpartition(".")[0] in sgl:
                s, _, lf = rest.rpartition(".")
                out[b + sgl[s] + "." + lf] = v
            elif rest.startswith("linear1."):
                lf = rest.rpartition(".")[2]
                for j, nm in enumerate(("attn.to_q", "attn.to_k", "attn.to_v")):
                    out[f"{b}{nm}.{lf}"] = v[j * d:(j + 1) * d]
                out[f"{b}proj_mlp.{lf}"] = v[3 * d:]
    return out


def flux_config_from(sd: dict):
    """Diffusers-named Flux state dict -> FluxConfig (block counts and widths from the shapes)."""
    from .flux import FluxConfig
    d = int(sd["x_embedder.weight"].shape[0])
    nd = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"transformer_blocks\.(\d+)\.", k)] if m)
    ns = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"single_transformer_blocks\.(\d+)\.", k)] if m)
    hd = int(sd["transformer_blocks.0.attn.norm_q.weight"].shape[0])
    return FluxConfig(in_channels=int(sd["x_embedder.weight"].shape[1]), layers=nd, single_layers=ns, head_dim=hd,
                      heads=d // hd, joint_dim=int(sd["context_embedder.weight"].shape[1]),
                      pooled_dim=int(sd["time_text_embed.text_embedder.linear_1.weight"].shape[1]),
                      guidance="time_text_embed.guidance_embedder.linear_1.weight" in sd)


# ---------------------------------------------------------------- SD3 / SD3.5 (Stability MMDiT names)
def sai_mmdit_to_diffusers(sd: dict) -> dict:
    """model.diffusion_model.* MMDiT (joint_blocks.i.{x,context}_block) -> SD3Transformer2DModel names.
    The last block's context stream is pre-only (adaLN with 2 vectors, no attention output / MLP)."""
    sd = strip(sd, "model.diffusion_model.") or sd
    d = int(sd["x_embedder.proj.weight"].shape[0])
    top = {"x_embedder.proj": "pos_embed.proj", "t_embedder.mlp.0": "time_text_embed.timestep_embedder.linear_1",
           "t_embedder.mlp.2": "time_text_embed.timestep_embedder.linear_2",
           "y_embedder.mlp.0": "time_text_embed.text_embedder.linear_1",
           "y_embedder.mlp.2": "time_text_embed.text_embedder.linear_2", "context_embedder": "context_embedder",
           "final_layer.linear": "proj_out"}
    blk = {"x_block.adaLN_modulation.1": "norm1.linear", "x_block.attn.proj": "attn.to_out.0",
           "x_block.mlp.fc1": "ff.net.0.proj", "x_block.mlp.fc2": "ff.net.2",
           "context_block.attn.proj": "attn.to_add_out", "context_block.mlp.fc1": "ff_context.net.0.proj",
           "context_block.mlp.fc2": "ff_context.net.2", "x_block.attn.ln_q": "attn.norm_q",
           "x_block.attn.ln_k": "attn.norm_k", "context_block.attn.ln_q": "attn.norm_added_q",
           "context_block.attn.ln_k": "attn.norm_added_k"}
    n = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"joint_blocks\.(\d+)\.", k)] if m)
    out = {}
    for k, v in sd.items():
        stem, _, leaf = k.rpartition(".")
        if k == "pos_embed":
            out["pos_embed.pos_embed"] = v
        elif stem in top:
            out[f"{top[stem]}.{leaf}"] = v
        elif stem == "final_layer.adaLN_modulation.1":  # (shift, scale) -> diffusers (scale, shift)
            out[f"norm_out.linear.{leaf}"] = torch.cat([v[d:], v[:d]], 0)
        elif (m := re.match(r"joint_blocks\.(\d+)\.(.+)$", stem)):
            i, rest = int(m.group(1)), m.group(2)
            b = f"transformer_blocks.{i}."
            if rest in blk:
                out[f"{b}{blk[rest]}.{leaf}"] = v
            elif rest == "context_block.adaLN_modulation.1":
                # last block: AdaLayerNormContinuous (2 vectors, swapped like norm_out)
                out[f"{b}norm1_context.linear.{leaf}"] = (torch.cat([v[d:], v[:d]], 0) if i == n - 1 and
                                                          v.shape[0] == 2 * d else v)
            elif rest in ("x_block.attn.qkv", "context_block.attn.qkv"):
                names = ("to_q", "to_k", "to_v") if rest.startswith("x_") else ("add_q_proj", "add_k_proj", "add_v_proj")
                for j, nm in enumerate(names):
                    out[f"{b}attn.{nm}.{leaf}"] = v[j * d:(j + 1) * d]
            elif rest == "x_block.attn2.qkv":  # MMDiT-X (SD3.5-medium) image-only second attention
                for j, nm in enumerate(("to_q", "to_k", "to_v")):
                    out[f"{b}attn2.{nm}.{leaf}"] = v[j * d:(j + 1) * d]
            elif rest in ("x_block.attn2.proj", "x_block.attn2.ln_q", "x_block.attn2.ln_k"):
                nm = {"proj": "to_out.0", "ln_q": "norm_q", "ln_k": "norm_k"}[rest.rsplit(".", 1)[1]]
                out[f"{b}attn2.{nm}.{leaf}"] = v
    return out


def mmdit_config_from(sd: dict):
    from .mmdit import MMDiTConfig
    w = sd["pos_embed.proj.weight"]
    d = int(w.shape[0])
    layers = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"transformer_blocks\.(\d+)\.", k)] if m)
    pos = sd.get("pos_embed.pos_embed")
    pos_max = int(round(float(pos.shape[1]) ** 0.5)) if pos is not None else 192
    return MMDiTConfig(patch=int(w.shape[2]), in_channels=int(w.shape[1]),
                       out_channels=int(sd["proj_out.weight"].shape[0]) // int(w.shape[2]) ** 2, layers=layers,
                       head_dim=64, heads=d // 64, joint_dim=int(sd["context_embedder.weight"].shape[1]),
                       caption_dim=d, pooled_dim=int(sd["time_text_embed.text_embedder.linear_1.weight"].shape[1]),
                       pos_max=pos_max, sample_size=128, qk_norm="transformer_blocks.0.attn.norm_q.weight" in sd,
                       dual_attention_layers=tuple(i for i in range(layers)
                                                   if f"transformer_blocks.{i}.attn2.to_q.weight" in sd))


# ---------------------------------------------------------------- text encoders
def openclip_to_hf(sd: dict) -> dict:
    """OpenCLIP text tower (SDXL conditioner.embedders.1.model.*) -> HF CLIPTextModelWithProjection names."""
    out = {}
    for k, v in sd.items():
        if k == "token_embedding.weight":
            out["text_model.embeddings.token_embedding.weight"] = v
        elif k == "positional_embedding":
            out["text_model.embeddings.position_embedding.weight"] = v
        elif k.startswith("ln_final."):
            out["text_model.final_layer_norm." + k.split(".")[-1]] = v
        elif k == "text_projection":
            out["text_projection.weight"] = v.t().contiguous()
        elif (m := re.match(r"transformer\.resblocks\.(\d+)\.(.+)$", k)):
            i, rest = m.groups()
            p = f"text_model.encoder.layers.{i}."
            if rest in ("attn.in_proj_weight", "attn.in_proj_bias"):
                lf = "weight" if rest.endswith("weight") else "bias"
                h = v.shape[0] // 3
                for j, nm in enumerate(("q_proj", "k_proj", "v_proj")):
                    out[f"{p}self_attn.{nm}.{lf}"] = v[j * h:(j + 1) * h]
            else:
                ren = {"attn.out_proj": "self_attn.out_proj", "ln_1": "layer_norm1", "ln_2": "layer_norm2",
                       "mlp.c_fc": "mlp.fc1", "mlp.c_proj": "mlp.fc2"}
                s, _, lf = rest.rpartition(".")
                if s in ren:
                    out[f"{p}{ren[s]}.{lf}"] = v
    return out


def clip_config_from(sd: dict):
    from .text_encoders import CLIPTextConfig
    te = sd["text_model.embeddings.token_embedding.weight"]
    hidden = int(te.shape[1])
    layers = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"text_model\.encoder\.layers\.(\d+)\.", k)] if m)
    proj = int(sd["text_projection.weight"].shape[0]) if "text_projection.weight" in sd else hidden
    # head width 64 in every released CLIP text tower (L: 12 x 64, H: 16 x 64, bigG: 20 x 64); the weights
    # do not carry it. Test-size towers (< 512 wide) use 16-wide heads.
    heads = hidden // 64 if hidden >= 512 else max(1, hidden // 16)
    return CLIPTextConfig(vocab=int(te.shape[0]), hidden=hidden, layers=layers, heads=heads,
                          ffn=int(sd["text_model.encoder.layers.0.mlp.fc1.weight"].shape[0]),
                          max_pos=int(sd["text_model.embeddings.position_embedding.weight"].shape[0]),
                          act="gelu" if hidden >= 1024 else "quick_gelu", proj=proj)


def t5_config_from(sd: dict):
    from .text_encoders import T5Config
    sd_ = sd
    emb = sd_.get("shared.weight", sd_.get("encoder.embed_tokens.weight"))
    layers = 1 + max(int(m.group(1)) for k in sd_ for m in [re.match(r"encoder\.block\.(\d+)\.", k)] if m)
    rab = sd_["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
    heads = int(rab.shape[1])
    q = sd_["encoder.block.0.layer.0.SelfAttention.q.weight"]
    return T5Config(vocab=int(emb.shape[0]), d_model=int(emb.shape[1]), heads=heads, d_kv=int(q.shape[0]) // heads,
                    d_ff=int(sd_["encoder.block.0.layer.1.DenseReluDense.wi_0.weight"].shape[0]), layers=layers,
                    buckets=int(rab.shape[0]))


# ---------------------------------------------------------------- tokenizers
def _clip_tokenizer(search: list[str], vocab: int, pad_token=None):
    from ...tokenizer.clip import CLIPTokenizer
    for d in search:
        for sub in ("", "tokenizer", "tokenizer_2" if pad_token else "tokenizer"):
            p = os.path.join(d, sub)
            if os.path.isfile(os.path.join(p, "vocab.json")) and os.path.isfile(os.path.join(p, "merges.txt")):
                return CLIPTokenizer.from_dir(p, pad_token=pad_token)
    log.warning("no CLIP vocab.json / merges.txt next to %s: byte-level prompt tokens (images will not follow "
                "the prompt)", search[:1])
    return CLIPTokenizer.synthetic(vocab, pad_token=pad_token)


def _t5_tokenizer(search: list[str], vocab: int, max_len: int):
    from ...tokenizer.clip import T5Tokenizer
    for d in search:
        for p in (os.path.join(d, "spiece.model"), os.path.join(d, "tokenizer_2", "spiece.model")):
            if os.path.isfile(p):
                return T5Tokenizer.from_file(p, max_len)
    log.warning("no T5 spiece.model next to %s: byte-level prompt tokens", search[:1])
    return T5Tokenizer(None, vocab, max_len)


def _dirs(*paths) -> list[str]:
    return [os.path.dirname(os.path.abspath(p)) for p in paths if p]


def _load(make, sd: dict, what: str, device, dtype, allow_missing=("position_ids",)):
    """Build the module directly on the target device (a 12B Flux transformer is not staged in host
    RAM twice), load the converted weights, cast to the pipeline dtype. GGMLTensor weights of nn.Linear
    layers become QParams (kept quantised); other GGMLTensors are dequantised."""
    from torch import nn as tnn
    from .nn import QParam, cast_module
    with torch.device(device):
        module = make()
    dense, quant = {}, {}
    for k, v in sd.items():
        if isinstance(v, GGMLTensor):
            mname, _, leaf = k.rpartition(".")
            try:
                mod = module.get_submodule(mname)
            except AttributeError:
                mod = None
            if leaf == "weight" and isinstance(mod, tnn.Linear) and tuple(mod.weight.shape) == tuple(v.shape):
                quant[k] = (mod, v)
                continue
            v = v.dense()
        dense[k] = v
    missing, _ = module.load_state_dict(dense, strict=False)
    missing = [k for k in missing if k not in quant and not any(a in k for a in allow_missing)]
    if missing:
        raise ValueError(f"{what}: missing weights {missing[:5]} ({len(missing)} in all)")
    module = cast_module(module, device, dtype).eval()
    nq = 0
    for k, (mod, v) in quant.items():
        qp = QParam.from_ggml(v.raw, v.qtype, v.n, v.k, device, dtype)
        del mod._parameters["weight"]
        if isinstance(qp, QParam):
            mod.weight = qp
            nq += 1
        else:
            mod.weight = tnn.Parameter(qp, requires_grad=False)
    if quant:
        log.info("%s: %d of %d linear weights kept block-quantised", what, nq, len(quant))
    return module


# ---------------------------------------------------------------- pipelines
def flux_from_single_file(model: str, device, clip_l_path: str = "", t5xxl_path: str = "", vae_path: str = "",
                          dtype=None):
    """Flux.1 transformer file (BFL names; safetensors or GGUF) + ae / clip_l / t5xxl component files."""
    from .flux import FluxPipeline, FluxTransformer
    from .text_encoders import CLIPTextEncoder, T5Encoder
    from .vae import AutoencoderKL
    dev = torch.device(device)
    dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
    raw = read_tensors(model, keep_quant=True)
    if not vae_path and any(k.startswith("vae.") for k in raw):
        vae_sd = ldm_vae_to_diffusers(strip(raw, "vae."))
    else:
        if not vae_path:
            raise ValueError("Flux needs the autoencoder: set the option vae_path:<ae.safetensors>")
        vae_sd = ldm_vae_to_diffusers(read_tensors(vae_path))
    tsd = bfl_flux_to_diffusers(raw)
    del raw
    fc = flux_config_from(tsd)
    tr = _load(lambda: FluxTransformer(fc), tsd, "flux transformer", dev, dtype)
    del tsd
    if not clip_l_path or not t5xxl_path:
        raise ValueError("Flux needs clip_l_path:<clip_l.safetensors> and t5xxl_path:<t5xxl.safetensors|gguf>")
    csd = read_tensors(clip_l_path, keep_quant=True)
    csd = strip(csd, "text_encoders.clip_l.transformer.") or csd
    cl = _load(lambda: CLIPTextEncoder(clip_config_from(csd)), csd, "clip_l", dev, dtype)
    t5sd = read_tensors(t5xxl_path, keep_quant=True)
    t5c = t5_config_from(t5sd)
    t5 = _load(lambda: T5Encoder(t5c), t5sd, "t5xxl", dev, dtype)
    vae = _load(lambda: AutoencoderKL(vae_config_from(vae_sd, 0.3611, 0.1159)), vae_sd, "vae", dev, dtype)
    nt = 512 if fc.guidance else 256
    search = _dirs(model, clip_l_path, t5xxl_path)
    return FluxPipeline(fc, tr, cl, t5, vae, _clip_tokenizer(search, cl.cfg.vocab), _t5_tokenizer(search, t5c.vocab, nt),
                        dev, t5_tokens=nt, dynamic_shift=fc.guidance)


def unet_from_single_file(model: str, device, kind: str, vae_path: str = "", clip_l_path: str = "",
                          clip_g_path: str = "", dtype=None):
    """SD1.x / SD2.x / SDXL single file (LDM/SGM names) -> UNetPipeline; component files override."""
    from .sd_pipeline import UNetPipeline, UNetPreset
    from .sgm_names import sgm_unet_path
    from .text_encoders import CLIPTextEncoder
    from .unet import SD15_UNET, SDXL_UNET, UNet2DConditionModel
    from .vae import AutoencoderKL
    import dataclasses
    dev = torch.device(device)
    dtype = dtype or (torch.float16 if dev.type == "cuda" else torch.float32)
    raw = read_tensors(model, keep_quant=True)
    usd_ldm = strip(raw, "model.diffusion_model.")
    xl = kind == "sdxl"
    if xl:
        uc = SDXL_UNET
    else:
        ctx = next(int(v.shape[1]) for k, v in usd_ldm.items() if k.endswith("attn2.to_k.weight"))
        lin = next(v for k, v in usd_ldm.items() if k.endswith("proj_in.weight")).dim() == 2
        # SD2.x: 1024-wide OpenCLIP-H context, linear projections, 64-channel heads
        uc = SD15_UNET if ctx == 768 else dataclasses.replace(SD15_UNET, cross_dim=ctx, linear_proj=lin,
                                                              heads=(5, 10, 20, 20), sample_size=96)
    with torch.device("meta"):  # the block numbering only (sgm_unet_path)
        shape_ref = UNet2DConditionModel(uc)
    usd = {}
    for k, v in usd_ldm.items():
        stem, _, leaf = k.rpartition(".")
        p = sgm_unet_path(stem, shape_ref)
        if p is not None:
            usd[f"{p}.{leaf}"] = v
    un = _load(lambda: UNet2DConditionModel(uc), usd, "unet", dev, dtype)
    del usd, usd_ldm
    vae_sd = ldm_vae_to_diffusers(read_tensors(vae_path) if vae_path else strip(raw, "first_stage_model."))
    scaling = 0.13025 if xl else 0.18215
    vae = _load(lambda: AutoencoderKL(vae_config_from(vae_sd, scaling, 0.0)), vae_sd, "vae", dev, dtype)
    if clip_l_path:
        lsd = read_tensors(clip_l_path, keep_quant=True)
    else:
        lsd = strip(raw, "conditioner.embedders.0.transformer.") if xl else strip(raw, "cond_stage_model.transformer.")
    if not lsd and not xl and any(k.startswith("cond_stage_model.model.") for k in raw):  # SD2.x OpenCLIP-H
        lsd = openclip_to_hf(strip(raw, "cond_stage_model.model."))
    t1 = _load(lambda: CLIPTextEncoder(clip_config_from(lsd), with_projection=False), lsd, "clip_l", dev, dtype,
               allow_missing=("position_ids", "text_projection"))
    t2 = None
    if xl:
        gsd = read_tensors(clip_g_path, keep_quant=True) if clip_g_path else openclip_to_hf(strip(raw, "conditioner.embedders.1.model."))
        t2 = _load(lambda: CLIPTextEncoder(clip_config_from(gsd), with_projection=True), gsd, "clip_g", dev, dtype)
    del raw
    search = _dirs(model, clip_l_path, clip_g_path)
    tk1 = _clip_tokenizer(search, t1.cfg.vocab)
    tk2 = _clip_tokenizer(search, t2.cfg.vocab, pad_token="!") if xl else None
    pr = UNetPreset(uc, t1.cfg, t2.cfg if t2 is not None else None, vae.cfg, uc.sample_size * 8)
    return UNetPipeline(pr, un, t1, t2, vae, tk1, tk2, dev)


def _component(raw: dict, path: str, prefixes: tuple) -> dict:
    """A text encoder from its own file (any of the known prefixes stripped) or from the model file."""
    src = read_tensors(path, keep_quant=True) if path else raw
    for p in prefixes:
        got = strip(src, p)
        if got:
            return got
    return src if path else {}


def sd3_from_single_file(model: str, device, clip_l_path: str = "", clip_g_path: str = "", t5xxl_path: str = "",
                         vae_path: str = "", dtype=None):
    """SD3 / SD3.5 (large) single file in Stability's names (+ optional component files)."""
    from .mmdit import MMDiT
    from .pipeline import SD3Pipeline, SD3Preset
    from .text_encoders import CLIPTextEncoder, T5Encoder
    from .vae import AutoencoderKL
    dev = torch.device(device)
    dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
    raw = read_tensors(model, keep_quant=True)
    msd = sai_mmdit_to_diffusers(raw)
    mc = mmdit_config_from(msd)
    mm = _load(lambda: MMDiT(mc), msd, "mmdit", dev, dtype, allow_missing=("pos_embed.pos_embed",))
    del msd
    vae_sd = ldm_vae_to_diffusers(read_tensors(vae_path) if vae_path else strip(raw, "first_stage_model."))
    if not vae_sd:
        raise ValueError("SD3 needs its VAE: bundled first_stage_model.* tensors or the option vae_path")
    vae = _load(lambda: AutoencoderKL(vae_config_from(vae_sd, 1.5305, 0.0609)), vae_sd, "vae", dev, dtype)
    lsd = _component(raw, clip_l_path, ("text_encoders.clip_l.transformer.", "cond_stage_model.transformer."))
    gsd = _component(raw, clip_g_path, ("text_encoders.clip_g.transformer.",))
    tsd = _component(raw, t5xxl_path, ("text_encoders.t5xxl.transformer.",))
    if not lsd or not gsd:
        raise ValueError("SD3 needs CLIP-L and CLIP-G: bundled text_encoders.* tensors or clip_l_path / clip_g_path")
    cl = _load(lambda: CLIPTextEncoder(clip_config_from(lsd)), lsd, "clip_l", dev, dtype,
               allow_missing=("position_ids", "text_projection"))
    cg = _load(lambda: CLIPTextEncoder(clip_config_from(gsd)), gsd, "clip_g", dev, dtype)
    t5 = None
    if tsd:
        t5c = t5_config_from(tsd)
        t5 = _load(lambda: T5Encoder(t5c), tsd, "t5xxl", dev, dtype)
    del raw
    search = _dirs(model, clip_l_path, clip_g_path, t5xxl_path)
    pr = SD3Preset(mc, cl.cfg, cg.cfg, t5.cfg if t5 is not None else None, vae.cfg)
    return SD3Pipeline(pr, mm, cl, cg, t5, vae, _clip_tokenizer(search, cl.cfg.vocab),
                       _clip_tokenizer(search, cg.cfg.vocab, pad_token="!"),
                       _t5_tokenizer(search, t5.cfg.vocab, 256) if t5 is not None else None, dev)


def from_single_file(model: str, device, opts: dict):
    """Entry point of the diffusion worker for a model FILE (gosd.cpp load_model)."""
    head = read_tensor_names(model)
    kind = detect(dict.fromkeys(head))
    if kind == "flux":
        return flux_from_single_file(model, device, opts.get("clip_l_path", ""), opts.get("t5xxl_path", ""),
                                     opts.get("vae_path", ""))
    if kind in ("sd1", "sdxl"):
        return unet_from_single_file(model, device, kind, opts.get("vae_path", ""), opts.get("clip_l_path", ""),
                                     opts.get("clip_g_path", ""))
    return sd3_from_single_file(model, device, opts.get("clip_l_path", ""), opts.get("clip_g_path", ""),
                                opts.get("t5xxl_path", ""), opts.get("vae_path", ""))


def read_tensor_names(path: str) -> list[str]:
    if path.endswith(".safetensors"):
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            return list(f.keys())
    if path.endswith(".gguf"):
        from ...formats.gguf import GGUFReader
        return list(GGUFReader(path).tensors)
    return list(read_tensors(path))
