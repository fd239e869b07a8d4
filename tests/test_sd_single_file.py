"""stablediffusion-ggml checkpoint parity (gosd.cpp:56-162): single-file / GGUF diffusion models in their
original training-code names plus clip_l_path / clip_g_path / t5xxl_path / vae_path component files
(models/diffusion/single_file.py). No real checkpoint can be fetched here: the files are synthetic
weights written in the original layouts (Black Forest Labs Flux, LDM VAE, CompVis/SGM UNet, OpenCLIP,
HF CLIP / T5) and must load into exactly the weights of the diffusers-layout pipeline they came from;
parity with stable-diffusion.cpp's own output is unpinned."""
import re

import numpy as np
import pytest
import torch
from safetensors.torch import save_file

from localai_tfp_amd.models.diffusion import single_file as SF
from localai_tfp_amd.models.diffusion.nn import QParam


def _flux_to_bfl(sd, d):
    """diffusers Flux names -> BFL names (the layout city96 / BFL files use)."""
    out = {}
    inv_top = {"x_embedder": "img_in", "context_embedder": "txt_in",
               "time_text_embed.timestep_embedder.linear_1": "time_in.in_layer",
               "time_text_embed.timestep_embedder.linear_2": "time_in.out_layer",
               "time_text_embed.text_embedder.linear_1": "vector_in.in_layer",
               "time_text_embed.text_embedder.linear_2": "vector_in.out_layer",
               "time_text_embed.guidance_embedder.linear_1": "guidance_in.in_layer",
               "time_text_embed.guidance_embedder.linear_2": "guidance_in.out_layer", "proj_out": "final_layer.linear"}
    dbl = {"norm1.linear": "img_mod.lin", "norm1_context.linear": "txt_mod.lin", "attn.to_out.0": "img_attn.proj",
           "attn.to_add_out": "txt_attn.proj", "ff.net.0.proj": "img_mlp.0", "ff.net.2": "img_mlp.2",
           "ff_context.net.0.proj": "txt_mlp.0", "ff_context.net.2": "txt_mlp.2"}
    norms = {"attn.norm_q.weight": "img_attn.norm.query_norm.scale", "attn.norm_k.weight": "img_attn.norm.key_norm.scale",
             "attn.norm_added_q.weight": "txt_attn.norm.query_norm.scale",
             "attn.norm_added_k.weight": "txt_attn.norm.key_norm.scale"}
    for k, v in sd.items():
        stem, _, leaf = k.rpartition(".")
        if stem in inv_top:
            out[f"{inv_top[stem]}.{leaf}"] = v
        elif stem == "norm_out.linear":
            out[f"final_layer.adaLN_modulation.1.{leaf}"] = torch.cat([v[d:], v[:d]], 0)
    n = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"transformer_blocks\.(\d+)\.", k)] if m)
    for i in range(n):
        b = f"transformer_blocks.{i}."
        for src, dst in dbl.items():
            for lf in ("weight", "bias"):
                out[f"double_blocks.{i}.{dst}.{lf}"] = sd[f"{b}{src}.{lf}"]
        for src, dst in norms.items():
            out[f"double_blocks.{i}.{dst}"] = sd[b + src]
        for lf in ("weight", "bias"):
            out[f"double_blocks.{i}.img_attn.qkv.{lf}"] = torch.cat([sd[f"{b}attn.to_{x}.{lf}"] for x in "qkv"])
            out[f"double_blocks.{i}.txt_attn.qkv.{lf}"] = torch.cat([sd[f"{b}attn.add_{x}_proj.{lf}"] for x in "qkv"])
    ns = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"single_transformer_blocks\.(\d+)\.", k)] if m)
    for i in range(ns):
        b = f"single_transformer_blocks.{i}."
        for lf in ("weight", "bias"):
            out[f"single_blocks.{i}.linear1.{lf}"] = torch.cat(
                [sd[f"{b}attn.to_{x}.{lf}"] for x in "qkv"] + [sd[f"{b}proj_mlp.{lf}"]])
            out[f"single_blocks.{i}.linear2.{lf}"] = sd[f"{b}proj_out.{lf}"]
            out[f"single_blocks.{i}.modulation.lin.{lf}"] = sd[f"{b}norm.linear.{lf}"]
        out[f"single_blocks.{i}.norm.query_norm.scale"] = sd[b + "attn.norm_q.weight"]
        out[f"single_blocks.{i}.norm.key_norm.scale"] = sd[b + "attn.norm_k.weight"]
    return out


def _vae_to_ldm(sd):
    """diffusers AutoencoderKL names -> LDM names (up blocks reversed, attention as 1x1 convs)."""
    n_up = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"decoder\.up_blocks\.(\d+)\.", k)] if m)
    out = {}
    for k, v in sd.items():
        nk = k
        nk = re.sub(r"down_blocks\.(\d+)\.resnets\.(\d+)\.", r"down.\1.block.\2.", nk)
        nk = re.sub(r"up_blocks\.(\d+)\.resnets\.(\d+)\.",
                    lambda m: f"up.{n_up - 1 - int(m[1])}.block.{m[2]}.", nk)
        nk = re.sub(r"down_blocks\.(\d+)\.downsamplers\.0\.conv\.", r"down.\1.downsample.conv.", nk)
        nk = re.sub(r"up_blocks\.(\d+)\.upsamplers\.0\.conv\.", lambda m: f"up.{n_up - 1 - int(m[1])}.upsample.conv.", nk)
        nk = nk.replace("conv_shortcut", "nin_shortcut").replace("conv_norm_out", "norm_out")
        nk = re.sub(r"mid_block\.resnets\.(\d)\.", lambda m: f"mid.block_{int(m[1]) + 1}.", nk)
        if "mid_block.attentions.0." in nk:
            part = {"group_norm": "norm", "to_q": "q", "to_k": "k", "to_v": "v", "to_out.0": "proj_out"}
            for a, b in part.items():
                nk = nk.replace(f"mid_block.attentions.0.{a}.", f"mid.attn_1.{b}.")
            if v.dim() == 2:
                v = v[:, :, None, None]
        out[nk] = v
    return out


def _save_gguf(path, sd):
    """transformer weights as a GGUF with Q8_0 blocks for the 2-D matrices (city96-style file)."""
    from localai_tfp_amd.formats.gguf import GGUFWriter, QType
    from localai_tfp_amd.ops.quant import quantize_q8_0
    w = GGUFWriter(path)
    w.add("general.architecture", "flux")
    for k, v in sd.items():
        a = v.float().numpy()
        if a.ndim == 2 and a.shape[1] % 32 == 0:
            w.add_tensor(k, quantize_q8_0(a).tobytes(), shape=tuple(reversed(a.shape)), qtype=QType.Q8_0)
        else:
            w.add_tensor(k, np.ascontiguousarray(a))
    w.write()


@pytest.mark.parametrize("fmt", ["safetensors", "gguf"])
def test_flux_single_file_with_components(tmp_path, fmt):
    from localai_tfp_amd.models.diffusion.flux import FluxPipeline
    from localai_tfp_amd.models.diffusion.pipeline import GenParams
    ref = FluxPipeline.synthetic("flux-test", "cpu")
    d = ref.cfg.dim
    tsd = {k: v.contiguous() for k, v in ref.tr.state_dict().items()}
    bfl = _flux_to_bfl(tsd, d)
    mp = str(tmp_path / f"flux1-test.{fmt}")
    if fmt == "safetensors":
        save_file(bfl, mp)
    else:
        _save_gguf(mp, bfl)
    vp, cp, tp = (str(tmp_path / n) for n in ("ae.safetensors", "clip_l.safetensors", "t5xxl.safetensors"))
    save_file(_vae_to_ldm({k: v.contiguous() for k, v in ref.vae.state_dict().items()}), vp)
    save_file({k: v.contiguous() for k, v in ref.clip_l.state_dict().items()}, cp)
    save_file({k: v.contiguous() for k, v in ref.t5.state_dict().items()}, tp)
    assert SF.detect(dict.fromkeys(SF.read_tensor_names(mp))) == "flux"
    pipe = SF.from_single_file(mp, "cpu", {"clip_l_path": cp, "t5xxl_path": tp, "vae_path": vp})
    assert pipe.cfg == ref.cfg
    got = pipe.tr.state_dict()
    for k, v in tsd.items():
        tol = 0 if fmt == "safetensors" or v.dim() != 2 else float(v.abs().max()) / 100
        if k not in got:  # a GGUF block weight kept quantised (nn.QParam)
            assert fmt == "gguf"
            w = pipe.tr.get_submodule(k.rpartition(".")[0]).weight
            assert isinstance(w, QParam)
            got[k] = w.dense()
        assert torch.allclose(got[k].float(), v.float(), atol=tol), k
    for a, b in ((pipe.vae, ref.vae), (pipe.clip_l, ref.clip_l), (pipe.t5, ref.t5)):
        sa, sb = a.state_dict(), b.state_dict()
        assert sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sb)
    if fmt == "safetensors":  # identical weights + tokenizer stand-ins -> identical image
        pipe.tok_l, pipe.tok_t5, pipe.t5_tokens = ref.tok_l, ref.tok_t5, ref.t5_tokens
        # GroupNorm group count is not stored in a checkpoint (32 in every released VAE; 8 in this test
        # preset): the VAE weights were compared above, the image checks transformer + text encoders
        pipe.vae = ref.vae
        gp = GenParams(width=32, height=32, steps=2, seed=3, cfg_scale=3.5)
        assert torch.equal(pipe.generate("a cat", gp), ref.generate("a cat", gp))


def test_flux_single_file_needs_components(tmp_path):
    from localai_tfp_amd.models.diffusion.flux import FluxPipeline
    ref = FluxPipeline.synthetic("flux-test", "cpu")
    mp = str(tmp_path / "f.safetensors")
    save_file(_flux_to_bfl({k: v.contiguous() for k, v in ref.tr.state_dict().items()}, ref.cfg.dim), mp)
    with pytest.raises(ValueError, match="vae_path"):
        SF.from_single_file(mp, "cpu", {})


def _ldm_unet_names(unet):
    """diffusers UNet param name -> SGM name, by enumerating SGM stems through sgm_unet_path."""
    from localai_tfp_amd.models.diffusion.sgm_names import sgm_unet_path
    params = dict(unet.state_dict())
    inv = {}
    stems = ["time_embed.0", "time_embed.2", "label_emb.0.0", "label_emb.0.2", "input_blocks.0.0", "out.0", "out.2"]
    sub_res = ["in_layers.0", "in_layers.2", "emb_layers.1", "out_layers.0", "out_layers.3", "skip_connection"]
    for i in range(40):
        for j in range(3):
            for blk in ("input_blocks", "output_blocks"):
                base = f"{blk}.{i}.{j}"
                stems += [f"{base}.{s}" for s in sub_res] + [f"{base}.op", f"{base}.conv"]
                stems += [f"{base}.{s}" for s in ("norm", "proj_in", "proj_out")]
    for j in range(3):
        stems += [f"middle_block.{j}.{s}" for s in sub_res + ["norm", "proj_in", "proj_out"]]
    for s in stems:
        p = sgm_unet_path(s, unet)
        if p is not None:
            for lf in ("weight", "bias"):
                if f"{p}.{lf}" in params and f"{p}.{lf}" not in inv:  # lowest SGM index wins
                    inv[f"{p}.{lf}"] = f"{s}.{lf}"
    # transformer blocks keep their names below the attention entry
    for k in params:
        if k in inv:
            continue
        m = re.match(r"(down_blocks\.\d+\.attentions\.\d+|up_blocks\.\d+\.attentions\.\d+|mid_block\.attentions\.0)"
                     r"\.(transformer_blocks\..+)$", k)
        if m:
            owner = next(v for kk, v in inv.items() if kk.startswith(m[1] + ".norm."))
            inv[k] = owner.rsplit(".norm.", 1)[0] + "." + m[2]
    return inv


def test_sd15_single_file(tmp_path):
    """SD1.x single file: model.diffusion_model. (SGM UNet), first_stage_model. (LDM VAE),
    cond_stage_model.transformer. (HF CLIP) in one .safetensors."""
    from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline
    ref = UNetPipeline.synthetic("sd15-test", "cpu")
    usd = {k: v.contiguous() for k, v in ref.unet.state_dict().items()}
    inv = _ldm_unet_names(ref.unet)
    missing = [k for k in usd if k not in inv]
    assert not missing, missing[:5]
    f = {"model.diffusion_model." + inv[k]: v for k, v in usd.items()}
    f.update({"first_stage_model." + k: v for k, v in _vae_to_ldm(
        {k: v.contiguous() for k, v in ref.vae.state_dict().items()}).items()})
    f.update({"cond_stage_model.transformer." + k: v.contiguous() for k, v in ref.te1.state_dict().items()})
    mp = str(tmp_path / "sd15.safetensors")
    save_file(f, mp)
    # the test UNet preset is not an SD1.x size: map it through the same code path with its config
    import localai_tfp_amd.models.diffusion.unet as U
    old = U.SD15_UNET
    U.SD15_UNET = ref.p.unet
    try:
        pipe = SF.unet_from_single_file(mp, "cpu", "sd1")
    finally:
        U.SD15_UNET = old
    for a, b in ((pipe.unet, ref.unet), (pipe.vae, ref.vae), (pipe.te1, ref.te1)):
        sa, sb = a.state_dict(), b.state_dict()
        assert all(torch.equal(sa[k], sb[k]) for k in sb), [k for k in sb if not torch.equal(sa[k], sb[k])][:3]


def test_openclip_to_hf_matches_transformers_layout():
    """OpenCLIP text tower (SDXL conditioner.embedders.1.model.) -> HF CLIP names: fused in_proj split,
    c_fc / c_proj, transposed text_projection."""
    h, L = 16, 2
    rng = torch.Generator().manual_seed(0)
    oc = {"token_embedding.weight": torch.randn(50, h, generator=rng),
          "positional_embedding": torch.randn(8, h, generator=rng),
          "ln_final.weight": torch.randn(h, generator=rng), "ln_final.bias": torch.randn(h, generator=rng),
          "text_projection": torch.randn(h, 12, generator=rng)}
    for i in range(L):
        p = f"transformer.resblocks.{i}."
        oc[p + "attn.in_proj_weight"] = torch.randn(3 * h, h, generator=rng)
        oc[p + "attn.in_proj_bias"] = torch.randn(3 * h, generator=rng)
        for n, shp in (("attn.out_proj", (h, h)), ("mlp.c_fc", (4 * h, h)), ("mlp.c_proj", (h, 4 * h))):
            oc[p + n + ".weight"] = torch.randn(*shp, generator=rng)
            oc[p + n + ".bias"] = torch.randn(shp[0], generator=rng)
        for n in ("ln_1", "ln_2"):
            oc[p + n + ".weight"] = torch.randn(h, generator=rng)
            oc[p + n + ".bias"] = torch.randn(h, generator=rng)
    hf = SF.openclip_to_hf(oc)
    assert torch.equal(hf["text_model.encoder.layers.1.self_attn.k_proj.weight"],
                       oc["transformer.resblocks.1.attn.in_proj_weight"][h:2 * h])
    assert torch.equal(hf["text_projection.weight"], oc["text_projection"].t())
    c = SF.clip_config_from(hf)
    assert (c.hidden, c.layers, c.ffn, c.proj, c.max_pos) == (h, L, 4 * h, 12, 8)
    transformers = pytest.importorskip("transformers")
    hc = transformers.CLIPTextConfig(vocab_size=50, hidden_size=h, intermediate_size=4 * h, num_hidden_layers=L,
                                     num_attention_heads=2, max_position_embeddings=8, projection_dim=12)
    m = transformers.CLIPTextModelWithProjection(hc)
    missing, unexpected = m.load_state_dict(hf, strict=False)
    assert not unexpected and all("position_ids" in k for k in missing), (missing, unexpected)


def test_worker_loads_flux_ggml_gallery_layout(tmp_path):
    """The gallery flux-ggml config shape: model file + clip_l_path / t5xxl_path / vae_path options
    relative to the models directory, then GenerateImage writes a PNG."""
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.models.diffusion.flux import FluxPipeline
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    ref = FluxPipeline.synthetic("flux-test", "cpu")
    save_file(_flux_to_bfl({k: v.contiguous() for k, v in ref.tr.state_dict().items()}, ref.cfg.dim),
              str(tmp_path / "flux1-dev-Q2_K.safetensors"))
    save_file(_vae_to_ldm({k: v.contiguous() for k, v in ref.vae.state_dict().items()}), str(tmp_path / "ae.safetensors"))
    save_file({k: v.contiguous() for k, v in ref.clip_l.state_dict().items()}, str(tmp_path / "clip_l.safetensors"))
    save_file({k: v.contiguous() for k, v in ref.t5.state_dict().items()}, str(tmp_path / "t5xxl_fp16.safetensors"))
    s = DiffusionServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="flux1-dev-Q2_K.safetensors", ModelPath=str(tmp_path), Options=[
        "diffusion_model", "clip_l_path:clip_l.safetensors", "t5xxl_path:t5xxl_fp16.safetensors",
        "vae_path:ae.safetensors", "sampler:euler"]), None)
    assert r.success, r.message
    dst = str(tmp_path / "o.png")
    r = s.GenerateImage(pb.GenerateImageRequest(positive_prompt="a cat", width=32, height=32, step=2, seed=1,
                                                dst=dst), None)
    assert r.success, r.message
    with open(dst, "rb") as f:
        assert f.read(8) == b"\x89PNG\r\n\x1a\n"


def _mmdit_to_sai(sd, d, n):
    """diffusers SD3Transformer2DModel names -> Stability MMDiT names (inverse of the loader's map)."""
    out = {"pos_embed": sd["pos_embed.pos_embed"]}
    top = {"pos_embed.proj": "x_embedder.proj", "time_text_embed.timestep_embedder.linear_1": "t_embedder.mlp.0",
           "time_text_embed.timestep_embedder.linear_2": "t_embedder.mlp.2",
           "time_text_embed.text_embedder.linear_1": "y_embedder.mlp.0",
           "time_text_embed.text_embedder.linear_2": "y_embedder.mlp.2", "context_embedder": "context_embedder",
           "proj_out": "final_layer.linear"}
    blk = {"norm1.linear": "x_block.adaLN_modulation.1", "attn.to_out.0": "x_block.attn.proj",
           "ff.net.0.proj": "x_block.mlp.fc1", "ff.net.2": "x_block.mlp.fc2", "attn.to_add_out": "context_block.attn.proj",
           "ff_context.net.0.proj": "context_block.mlp.fc1", "ff_context.net.2": "context_block.mlp.fc2",
           "attn.norm_q": "x_block.attn.ln_q", "attn.norm_k": "x_block.attn.ln_k",
           "attn.norm_added_q": "context_block.attn.ln_q", "attn.norm_added_k": "context_block.attn.ln_k",
           "attn2.to_out.0": "x_block.attn2.proj", "attn2.norm_q": "x_block.attn2.ln_q",
           "attn2.norm_k": "x_block.attn2.ln_k"}
    for k, v in sd.items():
        stem, _, leaf = k.rpartition(".")
        if stem in top:
            out[f"{top[stem]}.{leaf}"] = v
        elif stem == "norm_out.linear":
            out[f"final_layer.adaLN_modulation.1.{leaf}"] = torch.cat([v[d:], v[:d]], 0)
        elif (m := re.match(r"transformer_blocks\.(\d+)\.(.+)$", stem)):
            i, rest = int(m[1]), m[2]
            b = f"joint_blocks.{i}."
            if rest in blk:
                out[f"{b}{blk[rest]}.{leaf}"] = v
            elif rest == "norm1_context.linear":
                out[f"{b}context_block.adaLN_modulation.1.{leaf}"] = (
                    torch.cat([v[d:], v[:d]], 0) if i == n - 1 and v.shape[0] == 2 * d else v)
    for i in range(n):
        for lf in ("weight", "bias"):
            p = f"transformer_blocks.{i}.attn."
            out[f"joint_blocks.{i}.x_block.attn.qkv.{lf}"] = torch.cat([sd[f"{p}to_{x}.{lf}"] for x in "qkv"])
            out[f"joint_blocks.{i}.context_block.attn.qkv.{lf}"] = torch.cat([sd[f"{p}add_{x}_proj.{lf}"] for x in "qkv"])
            p2 = f"transformer_blocks.{i}.attn2."
            if f"{p2}to_q.{lf}" in sd:
                out[f"joint_blocks.{i}.x_block.attn2.qkv.{lf}"] = torch.cat([sd[f"{p2}to_{x}.{lf}"] for x in "qkv"])
    return out


def test_sd35_medium_mmditx_single_file(tmp_path):
    """SD3.5-medium (MMDiT-X) Stability layout: x_block.attn2.{qkv,proj,ln_q,ln_k} and 9-vector adaLN map to
    diffusers attn2 names; the config recovers dual_attention_layers from the tensor names."""
    from localai_tfp_amd.models.diffusion.mmdit import MMDITX_TEST, MMDiT
    from localai_tfp_amd.models.diffusion.nn import init_synthetic
    m = init_synthetic(MMDiT(MMDITX_TEST), 5)
    msd = {k: v.contiguous() for k, v in m.state_dict().items()}
    f = {"model.diffusion_model." + k: v for k, v in _mmdit_to_sai(msd, MMDITX_TEST.dim, MMDITX_TEST.layers).items()}
    assert "model.diffusion_model.joint_blocks.1.x_block.attn2.qkv.weight" in f
    sd = SF.sai_mmdit_to_diffusers(f)
    cfg = SF.mmdit_config_from(sd)
    assert cfg.dual_attention_layers == (0, 1) and cfg.qk_norm
    import dataclasses
    assert dataclasses.replace(cfg, sample_size=MMDITX_TEST.sample_size) == MMDITX_TEST
    m2 = MMDiT(cfg)
    miss, unexp = m2.load_state_dict(sd, strict=False)
    assert not unexp and not miss
    assert all(torch.equal(m2.state_dict()[k], v) for k, v in msd.items())


def test_sd3_single_file_bundled(tmp_path):
    """SD3 single file with everything bundled (Stability layout): model.diffusion_model.*,
    first_stage_model.*, text_encoders.{clip_l,clip_g,t5xxl}.transformer.*"""
    from localai_tfp_amd.models.diffusion.pipeline import GenParams, SD3Pipeline
    ref = SD3Pipeline.synthetic("sd3-test", "cpu")
    msd = {k: v.contiguous() for k, v in ref.mmdit.state_dict().items()}
    n = ref.p.mmdit.layers
    f = {"model.diffusion_model." + k: v for k, v in _mmdit_to_sai(msd, ref.p.mmdit.dim, n).items()}
    f.update({"first_stage_model." + k: v for k, v in _vae_to_ldm(
        {k: v.contiguous() for k, v in ref.vae.state_dict().items()}).items()})
    for name, m in (("clip_l", ref.clip_l), ("clip_g", ref.clip_g), ("t5xxl", ref.t5)):
        f.update({f"text_encoders.{name}.transformer.{k}": v.contiguous() for k, v in m.state_dict().items()})
    mp = str(tmp_path / "sd3_test.safetensors")
    save_file(f, mp)
    pipe = SF.from_single_file(mp, "cpu", {})
    import dataclasses  # the default sample size is not stored in the weights (SD3: 128 latents)
    assert dataclasses.replace(pipe.p.mmdit, sample_size=ref.p.mmdit.sample_size) == ref.p.mmdit
    for a, b in ((pipe.mmdit, ref.mmdit), (pipe.clip_l, ref.clip_l), (pipe.clip_g, ref.clip_g), (pipe.t5, ref.t5),
                 (pipe.vae, ref.vae)):
        sa, sb = a.state_dict(), b.state_dict()
        bad = [k for k in sb if k not in sa or not torch.equal(sa[k], sb[k])]
        assert not bad, bad[:4]
