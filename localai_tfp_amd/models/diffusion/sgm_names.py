"""Original-checkpoint parameter names -> this framework's (diffusers-layout) module paths.

Stable Diffusion single-file checkpoints and kohya LoRAs use the names of the original training code
(Stability's "SGM" / CompVis LDM UNet: `input_blocks.<i>.<j>`, `middle_block.<j>`,
`output_blocks.<i>.<j>`, `in_layers` / `emb_layers` / `out_layers` resnets, `op` downsamplers) and
Black Forest Labs' Flux names (`double_blocks.<i>.img_attn.qkv`, `single_blocks.<i>.linear1`, ...).
The reference hands such files to stable-diffusion.cpp (backend/go/image/stablediffusion-ggml/
gosd.cpp:56-162) or to diffusers' single-file loaders (backend/python/diffusers/backend.py:139-270);
here both map onto the module tree built by unet.py / flux.py.

The UNet numbering follows from the model's config: `input_blocks.0` is conv_in, then per level
`layers` (resnet[, attention]) entries and one downsampler; `output_blocks` walk the up blocks with
`layers + 1` entries each, the upsampler being the last sub-index of a level's last entry.
"""
from __future__ import annotations

import re

_RES = {"in_layers.0": "norm1", "in_layers.2": "conv1", "emb_layers.1": "time_emb_proj", "out_layers.0": "norm2",
        "out_layers.3": "conv2", "skip_connection": "conv_shortcut"}
_TOP = {"time_embed.0": "time_embedding.linear_1", "time_embed.2": "time_embedding.linear_2",
        "label_emb.0.0": "add_embedding.linear_1", "label_emb.0.2": "add_embedding.linear_2",
        "input_blocks.0.0": "conv_in", "out.0": "conv_norm_out", "out.2": "conv_out"}
_UNDER_RES = {k.replace(".", "_"): v for k, v in _RES.items()}
_UNDER_TOP = {k.replace(".", "_"): v for k, v in _TOP.items()}


def _sub(rest: str, kind: str, underscore: bool) -> str:
    """Rename the part below a block entry: resnet layer names, downsampler `op`."""
    table = _UNDER_RES if underscore else _RES
    sep = "_" if underscore else "."
    if kind == "res":
        for k in sorted(table, key=len, reverse=True):
            if rest == k or rest.startswith(k + sep):
                return table[k] + rest[len(k):]
        return rest
    if kind == "down" and (rest == "op" or rest.startswith("op" + sep)):
        return "conv" + rest[2:]
    return rest


def sgm_unet_path(name: str, unet, underscore: bool = False) -> str | None:
    """SGM/LDM UNet module path (dotted, or kohya underscore form) -> diffusers dotted path; None if
    `name` is not an SGM UNet name. `unet`: a UNet2DConditionModel (its blocks give the numbering)."""
    if not hasattr(unet, "down_blocks") or not hasattr(unet, "up_blocks"):
        return None
    s = "_" if underscore else "."
    top = _UNDER_TOP if underscore else _TOP
    for k in sorted(top, key=len, reverse=True):
        if name == k or name.startswith(k + s):
            return (top[k] + name[len(k):].replace("_", ".")) if underscore else top[k] + name[len(k):]
    L = unet.cfg.layers
    m = re.match(rf"(input_blocks|output_blocks){re.escape(s)}(\d+){re.escape(s)}(\d+)(?:{re.escape(s)}(.*))?$", name)
    mm = re.match(rf"middle_block{re.escape(s)}(\d+)(?:{re.escape(s)}(.*))?$", name)
    if m:
        which, i, j, rest = m.group(1), int(m.group(2)), int(m.group(3)), m.group(4) or ""
        if which == "input_blocks":
            lvl, k = divmod(i - 1, L + 1)
            if i == 0 or lvl >= len(unet.down_blocks):
                return None
            blk = unet.down_blocks[lvl]
            if k == L:
                prefix, kind = f"down_blocks.{lvl}.downsamplers.0", "down"
            elif j == 0:
                prefix, kind = f"down_blocks.{lvl}.resnets.{k}", "res"
            else:
                if blk.attentions is None:
                    return None
                prefix, kind = f"down_blocks.{lvl}.attentions.{k}", "attn"
        else:
            lvl, k = divmod(i, L + 1)
            if lvl >= len(unet.up_blocks):
                return None
            blk = unet.up_blocks[lvl]
            has_attn = blk.attentions is not None
            if j == 0:
                prefix, kind = f"up_blocks.{lvl}.resnets.{k}", "res"
            elif j == 1 and has_attn:
                prefix, kind = f"up_blocks.{lvl}.attentions.{k}", "attn"
            else:
                prefix, kind = f"up_blocks.{lvl}.upsamplers.0", "up"
    elif mm:
        j, rest = int(mm.group(1)), mm.group(2) or ""
        prefix, kind = {0: ("mid_block.resnets.0", "res"), 1: ("mid_block.attentions.0", "attn"),
                        2: ("mid_block.resnets.1", "res")}.get(j, (None, None))
        if prefix is None:
            return None
    else:
        return None
    rest = _sub(rest, kind, underscore)
    if underscore:  # the module tree is looked up in dotted form: re-dot the known sub-paths
        rest = _redot(rest)
    return prefix + ("." + rest if rest else "")


_ATTN_PARTS = ("transformer_blocks", "attn1", "attn2", "to_q", "to_k", "to_v", "to_out", "ff", "net", "proj",
               "proj_in", "proj_out", "norm1", "norm2", "norm3", "norm", "conv1", "conv2", "conv_shortcut",
               "time_emb_proj", "conv")


def _redot(rest: str) -> str:
    """kohya underscore sub-path -> dotted (`transformer_blocks_0_attn1_to_out_0` ->
    `transformer_blocks.0.attn1.to_out.0`): greedy match of known component names and indices."""
    out, i = [], 0
    parts = sorted(_ATTN_PARTS, key=len, reverse=True)
    while i < len(rest):
        if rest[i] == "_":
            i += 1
            continue
        mnum = re.match(r"\d+", rest[i:])
        if mnum:
            out.append(mnum.group(0))
            i += len(mnum.group(0))
            continue
        for p in parts:
            if rest.startswith(p, i) and (i + len(p) == len(rest) or rest[i + len(p)] == "_"):
                out.append(p)
                i += len(p)
                break
        else:
            j = rest.find("_", i)
            j = len(rest) if j < 0 else j
            out.append(rest[i:j])
            i = j
    return ".".join(out)


def bfl_flux_targets(path: str, dim: int):
    """kohya BFL Flux stem -> [(diffusers dotted path, (row0, row1) of the fused up matrix or None)];
    None if `path` is not a BFL Flux name. `dim`: the transformer's hidden size (for qkv splits)."""
    m = re.match(r"(double|single)_blocks_(\d+)_(.+)$", path)
    if not m or not dim:
        return None
    kind, i, rest = m.group(1), int(m.group(2)), m.group(3)
    d = dim
    if kind == "double":
        b = f"transformer_blocks.{i}."
        table = {"img_attn_proj": [(b + "attn.to_out.0", None)], "txt_attn_proj": [(b + "attn.to_add_out", None)],
                 "img_mlp_0": [(b + "ff.net.0.proj", None)], "img_mlp_2": [(b + "ff.net.2", None)],
                 "txt_mlp_0": [(b + "ff_context.net.0.proj", None)], "txt_mlp_2": [(b + "ff_context.net.2", None)],
                 "img_mod_lin": [(b + "norm1.linear", None)], "txt_mod_lin": [(b + "norm1_context.linear", None)],
                 "img_attn_qkv": [(b + "attn.to_q", (0, d)), (b + "attn.to_k", (d, 2 * d)),
                                  (b + "attn.to_v", (2 * d, 3 * d))],
                 "txt_attn_qkv": [(b + "attn.add_q_proj", (0, d)), (b + "attn.add_k_proj", (d, 2 * d)),
                                  (b + "attn.add_v_proj", (2 * d, 3 * d))]}
    else:
        b = f"single_transformer_blocks.{i}."
        table = {"linear1": [(b + "attn.to_q", (0, d)), (b + "attn.to_k", (d, 2 * d)), (b + "attn.to_v", (2 * d, 3 * d)),
                             (b + "proj_mlp", (3 * d, 7 * d))],
                 "linear2": [(b + "proj_out", None)], "modulation_lin": [(b + "norm.linear", None)]}
    return table.get(rest)
