"""LoRA adapters for the image pipelines (reference: backend/python/diffusers/backend.py:244-300 —
`LoraAdapter`, `LoraAdapters` + `LoraScales`, kohya merge `W += multiplier * alpha/rank * up@down`).

Checked against a plain fp32 re-computation of that formula on the affected weights, and end to end:
an image generated after the merge (fused QKV / `_prep` caches built BEFORE the merge) must equal the
image of a fresh pipeline whose weights were edited by hand. diffusers/peft are not installed, so key
naming parity with real adapter files rests on the shared diffusers parameter names."""
import copy

import pytest
import torch
from safetensors.torch import save_file

from localai_tfp_amd.models.diffusion import lora as L
from localai_tfp_amd.models.diffusion.pipeline import GenParams


def _ud(out_f, in_f, r, g, conv=None):
    down = torch.randn(r, in_f, *(conv or ()), generator=g) * 0.05
    up = torch.randn(out_f, r, *((1, 1) if conv else ()), generator=g) * 0.05
    return up, down


def _delta(up, down, alpha, r, scale, shape):
    return (scale * alpha / r) * (up.reshape(up.shape[0], r).double() @ down.reshape(r, -1).double()).reshape(shape)


def test_kohya_unet_and_text_encoder(tmp_path):
    from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline
    p = UNetPipeline.synthetic("sd15-test", "cpu")
    ref = copy.deepcopy(p)
    gp = GenParams(width=64, height=64, steps=2, seed=3, cfg_scale=4.0)
    base = p.generate("a fox", gp)  # populates the fused-QKV caches before the merge
    g = torch.Generator().manual_seed(0)
    targets = {
        ("lora_unet_", "unet", "down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q", None),
        ("lora_unet_", "unet", "down_blocks.0.resnets.0.conv1", (3, 3)),
        ("lora_te_", "te1", "text_model.encoder.layers.0.self_attn.q_proj", None),
    }
    sd, expect = {}, {}
    for pre, comp, path, conv in targets:
        mod = dict(getattr(ref, comp).named_modules())[path]
        w = mod.weight
        up, down = _ud(w.shape[0], w.shape[1], 4, g, conv)
        key = pre + path.replace(".", "_")
        sd[key + ".lora_up.weight"], sd[key + ".lora_down.weight"] = up, down
        sd[key + ".alpha"] = torch.tensor(2.0)
        expect[(comp, path)] = w.double() + _delta(up, down, 2.0, 4, 0.7, w.shape)
    f = tmp_path / "k.safetensors"
    save_file(sd, str(f))
    assert L.apply_adapters(p, [(str(f), 0.7)]) == 3
    for (comp, path), want in expect.items():
        got = dict(getattr(p, comp).named_modules())[path].weight
        torch.testing.assert_close(got.double(), want, rtol=1e-6, atol=1e-6)
        dict(getattr(ref, comp).named_modules())[path].weight.data.copy_(want.float())
    out = p.generate("a fox", gp)
    assert not torch.equal(out, base)
    torch.testing.assert_close(out, ref.generate("a fox", gp), rtol=0, atol=1e-5)


def test_peft_flux_transformer_cache_invalidated(tmp_path):
    from localai_tfp_amd.models.diffusion import flux as FX
    p = FX.FluxPipeline.synthetic("flux-test", "cpu")
    ref = FX.FluxPipeline.synthetic("flux-test", "cpu")
    gp = GenParams(width=64, height=64, steps=2, seed=5, cfg_scale=3.5)
    base = p.generate("a boat", gp)
    assert p.tr._prep is not None
    g = torch.Generator().manual_seed(1)
    sd = {}
    for path in ("transformer_blocks.0.attn.to_k", "single_transformer_blocks.0.attn.to_q"):
        w = dict(p.tr.named_modules())[path].weight
        up, down = _ud(w.shape[0], w.shape[1], 8, g)
        sd[f"transformer.{path}.lora_A.weight"], sd[f"transformer.{path}.lora_B.weight"] = down, up
        rw = dict(ref.tr.named_modules())[path].weight
        rw.data.add_(_delta(up, down, 8, 8, 1.0, w.shape).float())
    ref.tr._prep = None
    d = tmp_path / "adapter"
    d.mkdir()
    save_file(sd, str(d / "pytorch_lora_weights.safetensors"))
    assert L.apply_adapters(p, [(str(d), 1.0)]) == 2
    assert p.tr._prep is None
    out = p.generate("a boat", gp)
    assert not torch.equal(out, base)
    torch.testing.assert_close(out, ref.generate("a boat", gp), rtol=0, atol=1e-5)


def test_worker_lora_options(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    sd = {}
    g = torch.Generator().manual_seed(2)
    up, down = _ud(64, 64, 2, g)  # sd15-test attn inner dim
    svc0 = DiffusionServicer("cpu")
    assert svc0.LoadModel(pb.ModelOptions(Model="synthetic:sd15-test"), None).success
    w0 = svc0.pipe.unet.mid_block.attentions[0].transformer_blocks[0].attn1.to_v.weight.clone()
    assert tuple(w0.shape) == (64, 64)
    sd["unet.mid_block.attentions.0.transformer_blocks.0.attn1.to_v.lora.down.weight"] = down
    sd["unet.mid_block.attentions.0.transformer_blocks.0.attn1.to_v.lora.up.weight"] = up
    save_file(sd, str(tmp_path / "a.safetensors"))
    svc = DiffusionServicer("cpu")
    r = svc.LoadModel(pb.ModelOptions(Model="synthetic:sd15-test", ModelPath=str(tmp_path),
                                      LoraAdapters=["a.safetensors", "a.safetensors"], LoraScales=[0.5, 0.25]), None)
    assert r.success, r.message
    w = svc.pipe.unet.mid_block.attentions[0].transformer_blocks[0].attn1.to_v.weight
    torch.testing.assert_close(w.double(), w0.double() + _delta(up, down, 2, 2, 0.75, w0.shape), rtol=1e-6, atol=1e-6)
    bad = DiffusionServicer("cpu")
    save_file({"lora_unet_nope.lora_up.weight": up, "lora_unet_nope.lora_down.weight": down},
              str(tmp_path / "bad.safetensors"))
    r = bad.LoadModel(pb.ModelOptions(Model="synthetic:sd15-test", ModelPath=str(tmp_path),
                                      LoraAdapter="bad.safetensors"), None)
    assert not r.success and ("matched no layer" in r.message or "match no module" in r.message)


@pytest.mark.gpu
def test_lora_merge_on_gpu(tmp_path):
    from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline
    p = UNetPipeline.synthetic("sd15-test", "cuda:0")
    mod = p.unet.down_blocks[0].attentions[0].transformer_blocks[0].attn1.to_q
    w0 = mod.weight.float().cpu()
    g = torch.Generator().manual_seed(4)
    up, down = _ud(w0.shape[0], w0.shape[1], 4, g)
    key = "lora_unet_down_blocks_0_attentions_0_transformer_blocks_0_attn1_to_q"
    save_file({key + ".lora_up.weight": up, key + ".lora_down.weight": down}, str(tmp_path / "g.safetensors"))
    gp = GenParams(width=64, height=64, steps=2, seed=3)
    p.generate("x", gp)
    assert L.apply_adapters(p, [(str(tmp_path / "g.safetensors"), 1.0)]) == 1
    want = w0.double() + _delta(up, down, 4, 4, 1.0, w0.shape)
    torch.testing.assert_close(mod.weight.double().cpu(), want, rtol=1e-2, atol=2e-3)
    img = p.generate("x", gp)
    assert torch.isfinite(img).all()


def test_sgm_unet_names_map_onto_diffusers_tree():
    """SDXL kohya LoRAs use the original SGM UNet numbering (they used to match nothing)."""
    from localai_tfp_amd.models.diffusion.sgm_names import sgm_unet_path
    from localai_tfp_amd.models.diffusion.unet import UNET_XL_TEST, UNet2DConditionModel
    unet = UNet2DConditionModel(UNET_XL_TEST)  # layers=1; level 0 plain, level 1 cross-attention
    mods = dict(unet.named_modules())
    cases = {
        "input_blocks_1_0_in_layers_2": "down_blocks.0.resnets.0.conv1",
        "input_blocks_2_0_op": "down_blocks.0.downsamplers.0.conv",
        "input_blocks_3_1_transformer_blocks_0_attn1_to_q": "down_blocks.1.attentions.0.transformer_blocks.0.attn1.to_q",
        "input_blocks_3_1_proj_in": "down_blocks.1.attentions.0.proj_in",
        "middle_block_0_emb_layers_1": "mid_block.resnets.0.time_emb_proj",
        "middle_block_1_transformer_blocks_1_ff_net_0_proj": "mid_block.attentions.0.transformer_blocks.1.ff.net.0.proj",
        "middle_block_2_out_layers_3": "mid_block.resnets.1.conv2",
        "output_blocks_0_1_transformer_blocks_0_attn2_to_out_0": "up_blocks.0.attentions.0.transformer_blocks.0.attn2.to_out.0",
        "output_blocks_1_0_skip_connection": "up_blocks.0.resnets.1.conv_shortcut",
        "output_blocks_1_2_conv": "up_blocks.0.upsamplers.0.conv",
        "output_blocks_3_0_in_layers_2": "up_blocks.1.resnets.1.conv1",
        "time_embed_0": "time_embedding.linear_1",
        "label_emb_0_2": "add_embedding.linear_2",
    }
    for k, want in cases.items():
        got = sgm_unet_path(k, unet, underscore=True)
        assert got == want, (k, got)
        assert want in mods
    assert sgm_unet_path("input_blocks.3.1.transformer_blocks.0.attn1.to_q", unet) == \
        "down_blocks.1.attentions.0.transformer_blocks.0.attn1.to_q"
    # merge through the kohya path
    g = torch.Generator().manual_seed(1)
    w = mods["down_blocks.1.attentions.0.transformer_blocks.0.attn1.to_q"].weight
    w0 = w.detach().clone()
    up, down = _ud(w.shape[0], w.shape[1], 2, g)
    sd = {"lora_unet_input_blocks_3_1_transformer_blocks_0_attn1_to_q.lora_up.weight": up,
          "lora_unet_input_blocks_3_1_transformer_blocks_0_attn1_to_q.lora_down.weight": down}
    assert L.merge_lora({"unet": unet}, sd, 1.0) == 1
    torch.testing.assert_close(w.double(), w0.double() + _delta(up, down, 2, 2, 1.0, w0.shape), rtol=1e-6, atol=1e-6)


def test_bfl_flux_lora_splits_fused_qkv():
    from localai_tfp_amd.models.diffusion import flux as FX
    tr = FX.FluxTransformer(FX.FLUX_TEST)
    d = FX.FLUX_TEST.dim
    mods = dict(tr.named_modules())
    g = torch.Generator().manual_seed(2)
    r = 4
    down = torch.randn(r, d, generator=g) * 0.05
    up_qkv = torch.randn(3 * d, r, generator=g) * 0.05
    up_l1 = torch.randn(7 * d, r, generator=g) * 0.05
    before = {k: mods[k].weight.detach().clone() for k in (
        "transformer_blocks.0.attn.to_q", "transformer_blocks.0.attn.to_v",
        "single_transformer_blocks.1.attn.to_k", "single_transformer_blocks.1.proj_mlp")}
    sd = {"lora_unet_double_blocks_0_img_attn_qkv.lora_up.weight": up_qkv,
          "lora_unet_double_blocks_0_img_attn_qkv.lora_down.weight": down,
          "lora_unet_single_blocks_1_linear1.lora_up.weight": up_l1,
          "lora_unet_single_blocks_1_linear1.lora_down.weight": down}
    assert L.merge_lora({"transformer": tr}, sd, 1.0) == 3 + 4
    chk = {"transformer_blocks.0.attn.to_q": up_qkv[:d], "transformer_blocks.0.attn.to_v": up_qkv[2 * d:],
           "single_transformer_blocks.1.attn.to_k": up_l1[d:2 * d], "single_transformer_blocks.1.proj_mlp": up_l1[3 * d:]}
    for k, u in chk.items():
        w0 = before[k]
        torch.testing.assert_close(mods[k].weight.double(), w0.double() + _delta(u, down, r, r, 1.0, w0.shape),
                                   rtol=1e-6, atol=1e-6)
