"""LoRA adapters for the image pipelines, merged into the weights at load time.

Reference behaviour: the diffusers backend (backend/python/diffusers/backend.py:244-257) loads
`LoraAdapter` (one file, or a directory of attention processors) and `LoraAdapters` + `LoraScales`
(several named adapters with per-adapter weights); its kohya merge helper (backend.py:270-300)
adds `multiplier * alpha / rank * up @ down` into each targeted Linear / Conv2d weight.

Here every adapter is merged once into the resident weights (no per-step low-rank GEMMs: a
merged weight costs nothing per denoising step), then the fused-weight caches the MI355X forward
passes keep (MMDiT/Flux `_prep`, CLIP/UNet `_qkv`) are dropped so they are rebuilt from the
merged weights. Key layouts understood:

* kohya / sd-scripts:  `lora_unet_<path_with_underscores>.lora_down.weight|lora_up.weight|alpha`,
  `lora_te_` / `lora_te1_` / `lora_te2_` (text encoders), `lora_transformer_` (MMDiT / Flux);
* kohya over the original (SGM / LDM) UNet names, as SDXL LoRAs trained with sd-scripts ship:
  `lora_unet_input_blocks_4_1_transformer_blocks_0_attn1_to_q`, `..._middle_block_1_...`,
  `..._output_blocks_2_1_conv` — renamed onto the diffusers module tree (sgm_names.py);
* kohya over Black Forest Labs' Flux names: `lora_unet_double_blocks_<i>_img_attn_qkv` (split into
  to_q/to_k/to_v), `..._txt_attn_proj`, `..._img_mlp_0`, `lora_unet_single_blocks_<i>_linear1` (split
  into to_q/to_k/to_v/proj_mlp), `..._linear2`, `..._modulation_lin`;
* diffusers / PEFT:    `<root>.<dotted.path>.lora_A.weight|lora_B.weight` (optional `.alpha`),
  and the older `<root>.<dotted.path>.lora.down.weight|lora.up.weight`; `<root>` is `unet`,
  `transformer`, `text_encoder`, `text_encoder_2`, `text_encoder_3`, or absent (= the denoiser).

A denoiser (UNet / transformer) group that matches no layer fails the load: silently dropping the
denoiser half of an adapter would serve the base model under the adapter's name.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.nn as nn

from .sgm_names import bfl_flux_targets, sgm_unet_path

log = logging.getLogger("localai_tfp_amd.diffusion.lora")

_KOHYA_ROOTS = (("lora_unet_", "unet"), ("lora_transformer_", "transformer"), ("lora_te1_", "text_encoder"),
                ("lora_te2_", "text_encoder_2"), ("lora_te3_", "text_encoder_3"), ("lora_te_", "text_encoder"))
_SUFFIXES = ((".lora_down.weight", "down"), (".lora_up.weight", "up"), (".lora_A.weight", "down"),
             (".lora_B.weight", "up"), (".lora.down.weight", "down"), (".lora.up.weight", "up"), (".alpha", "alpha"))


def pipeline_roots(pipe) -> dict[str, nn.Module]:
    """Map the diffusers component names onto this framework's pipeline modules."""
    roots = {}
    for name, attrs in (("unet", ("unet", "mmdit", "tr")), ("transformer", ("mmdit", "tr", "unet")),
                        ("text_encoder", ("te1", "clip_l")), ("text_encoder_2", ("te2", "clip_g", "t5")),
                        ("text_encoder_3", ("t5",))):
        for a in attrs:
            m = getattr(pipe, a, None)
            if isinstance(m, nn.Module):
                roots[name] = m
                break
    if getattr(pipe, "clip_g", None) is None and getattr(pipe, "t5", None) is not None:
        roots["text_encoder_2"] = pipe.t5  # Flux: text_encoder_2 is the T5 encoder
    return roots


def load_lora_file(path: str) -> dict[str, torch.Tensor]:
    """A `.safetensors` file, or a directory holding one (diffusers `pytorch_lora_weights.safetensors`)."""
    from safetensors.torch import load_file
    if os.path.isdir(path):
        cands = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
        pref = [f for f in cands if f.startswith("pytorch_lora_weights")]
        if not cands:
            raise ValueError(f"{path}: no .safetensors LoRA file in directory")
        path = os.path.join(path, (pref or cands)[0])
    if not path.endswith(".safetensors"):
        raise ValueError(f"{path}: only safetensors LoRA files are loaded (no pickled checkpoints)")
    return load_file(path)


def _group(sd: dict[str, torch.Tensor]) -> dict[tuple[str, str, bool], dict[str, torch.Tensor]]:
    """(root, module path, kohya?) -> {"down", "up", "alpha"}."""
    out: dict[tuple[str, str, bool], dict[str, torch.Tensor]] = {}
    for k, v in sd.items():
        for suf, role in _SUFFIXES:
            if k.endswith(suf):
                stem = k[: -len(suf)]
                break
        else:
            continue
        root, kohya = None, False
        for pre, r in _KOHYA_ROOTS:
            if stem.startswith(pre):
                root, stem, kohya = r, stem[len(pre):], True
                break
        if root is None:
            head, _, rest = stem.partition(".")
            if head in ("unet", "transformer", "text_encoder", "text_encoder_2", "text_encoder_3") and rest:
                root, stem = head, rest
            else:
                root = "unet"
            stem = stem.replace(".processor.", ".").replace("_lora", "")  # attn-proc layout: to_q_lora -> to_q
        out.setdefault((root, stem, kohya), {})[role] = v
    return out


def _module_index(root: nn.Module) -> tuple[dict[str, nn.Module], dict[str, nn.Module]]:
    dotted, under = {}, {}
    for n, m in root.named_modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            dotted[n] = m
            under[n.replace(".", "_")] = m
    return dotted, under


def _targets(root: str, path: str, kohya: bool, mod_root: nn.Module):
    """-> [(module path, under?, up-row slice or None)] for one adapter group."""
    if kohya and root in ("unet", "transformer"):
        bfl = bfl_flux_targets(path, getattr(getattr(mod_root, "cfg", None), "dim", 0))
        if bfl is not None:
            return [(p, False, sl) for p, sl in bfl]
        sgm = sgm_unet_path(path, mod_root, underscore=True)
        if sgm is not None:
            return [(sgm, False, None)]
    return [(path, kohya, None)]


@torch.no_grad()
def merge_lora(roots: dict[str, nn.Module], sd: dict[str, torch.Tensor], scale: float = 1.0) -> int:
    """Merge one adapter into the modules under `roots`; returns the number of layers patched."""
    idx = {}
    n = 0
    missing = []
    for (root, path, kohya), t in _group(sd).items():
        if "down" not in t or "up" not in t:
            continue
        mod_root = roots.get(root) or (roots.get("transformer") if root == "unet" else roots.get("unet"))
        if mod_root is None:
            log.warning("LoRA: no %s component for %s", root, path)
            continue
        if id(mod_root) not in idx:
            idx[id(mod_root)] = _module_index(mod_root)
        dotted, under = idx[id(mod_root)]
        down = t["down"].float()
        up_all = t["up"].float()
        r = down.shape[0]
        alpha = float(t["alpha"]) if "alpha" in t else float(r)
        for tpath, tunder, rows in _targets(root, path, kohya, mod_root):
            mod = (under if tunder else dotted).get(tpath)
            if mod is None:
                if root in ("unet", "transformer"):
                    missing.append(f"{root}.{path}")
                else:
                    log.warning("LoRA: no layer %s.%s", root, path)
                break
            up = up_all.reshape(up_all.shape[0], -1)
            if rows is not None:
                up = up[rows[0]:rows[1]]
            w = mod.weight
            delta = up.reshape(up.shape[0], r) @ down.reshape(r, -1)
            if delta.numel() != w.numel():
                raise ValueError(f"LoRA {root}.{path}: delta {tuple(delta.shape)} vs weight {tuple(w.shape)}")
            w.add_((delta * (scale * alpha / r)).reshape(w.shape).to(device=w.device, dtype=w.dtype))
            n += 1
    if missing:
        raise ValueError(f"LoRA: {len(missing)} denoiser layer group(s) match no module of this model, e.g. "
                         + ", ".join(missing[:4]))
    for m in roots.values():  # fused caches rebuild from the merged weights on next use
        for sub in m.modules():
            if getattr(sub, "_prep", None) is not None:
                sub._prep = None
            if getattr(sub, "_qkv", None) is not None:
                sub._qkv = None
    return n


def apply_adapters(pipe, adapters: list[tuple[str, float]]) -> int:
    """Merge `[(path, scale), ...]` into a loaded pipeline; returns patched layer count."""
    roots = pipeline_roots(pipe)
    total = 0
    for path, scale in adapters:
        n = merge_lora(roots, load_lora_file(path), scale)
        if n == 0:
            raise ValueError(f"{path}: LoRA matched no layer of this model")
        log.info("LoRA %s (scale %.3g): %d layers merged", path, scale, n)
        total += n
    return total
