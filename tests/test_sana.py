"""Sana (diffusers SanaPipeline, backend/python/diffusers/backend.py:21,218-221).

* the transformer matches a float64 re-statement of diffusers' SanaTransformer2DModel written here
  independently (NCHW GLUMBConv through F.conv2d, ReLU linear attention with the padded-value trick,
  masked SDPA cross-attention, adaLN-single modulation);
* the DC-AE decoder matches a float64 re-statement of AutoencoderDC's decoder (ResBlock / EfficientViT
  multi-scale linear attention / interpolate up-blocks);
* a synthetic directory in diffusers' layout loads and generates through the diffusion worker.
diffusers is not installed: parity with its images stays unpinned."""
import json
import math

import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.models.diffusion import sana as SA

transformers = pytest.importorskip("transformers")


def _perturb(m, seed):
    from localai_tfp_amd.models.diffusion.nn import init_synthetic
    init_synthetic(m, seed, std=0.05)
    g = torch.Generator().manual_seed(seed + 100)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("norm.weight") or "norm_out.weight" in n or "caption_norm" in n:
                p.copy_(1 + 0.2 * torch.randn(p.shape, generator=g))
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(1 + 0.3 * torch.rand(mod.running_var.shape, generator=g))
    return m


def _ref_transformer(tr: SA.SanaTransformer, x, t, ctx, klen):
    c = tr.cfg
    sd = {k: v.double() for k, v in tr.state_dict().items()}
    D = c.dim
    B, C, H, W = x.shape
    N_ = H * W

    def linear(v, name, bias=True):
        y = v @ sd[name + ".weight"].reshape(sd[name + ".weight"].shape[0], -1).T
        return y + sd[name + ".bias"] if bias and name + ".bias" in sd else y
    silu = F.silu
    hs = F.conv2d(x.double(), sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"]).flatten(2).transpose(1, 2)
    half = 128
    fr = torch.exp(-math.log(10000.0) * torch.arange(half, dtype=torch.float64) / half)
    a = t.double()[:, None] * fr[None]
    tp = torch.cat([torch.cos(a), torch.sin(a)], -1)
    emb = linear(silu(linear(tp, "time_embed.emb.timestep_embedder.linear_1")), "time_embed.emb.timestep_embedder.linear_2")
    tmod = linear(silu(emb), "time_embed.linear")
    e = linear(F.gelu(linear(ctx.double(), "caption_projection.linear_1"), approximate="tanh"), "caption_projection.linear_2")
    e = e * torch.rsqrt(e.pow(2).mean(-1, keepdim=True) + 1e-5) * sd["caption_norm.weight"]
    T = ctx.shape[1]
    mask = torch.arange(T)[None, :] < klen[:, None].long()
    for i in range(c.layers):
        p = f"transformer_blocks.{i}."
        sh1, sc1, g1, sh2, sc2, g2 = (sd[p + "scale_shift_table"][None] + tmod.reshape(B, 6, -1)).chunk(6, dim=1)
        n = F.layer_norm(hs, (D,), eps=c.eps) * (1 + sc1) + sh1
        q = F.relu(linear(n, p + "attn1.to_q")).transpose(1, 2).unflatten(1, (c.heads, -1))       # B H hd N
        k = F.relu(linear(n, p + "attn1.to_k")).transpose(1, 2).unflatten(1, (c.heads, -1)).transpose(2, 3)
        v = linear(n, p + "attn1.to_v").transpose(1, 2).unflatten(1, (c.heads, -1))
        v = F.pad(v, (0, 0, 0, 1), value=1.0)
        o = torch.matmul(torch.matmul(v, k), q)
        o = (o[:, :, :-1] / (o[:, :, -1:] + 1e-15)).flatten(1, 2).transpose(1, 2)
        hs = hs + g1 * linear(o, p + "attn1.to_out.0")
        q2 = linear(hs, p + "attn2.to_q").view(B, N_, c.cross_heads, -1).transpose(1, 2)
        k2 = linear(e, p + "attn2.to_k").view(B, T, c.cross_heads, -1).transpose(1, 2)
        v2 = linear(e, p + "attn2.to_v").view(B, T, c.cross_heads, -1).transpose(1, 2)
        o2 = F.scaled_dot_product_attention(q2, k2, v2, attn_mask=mask[:, None, None, :])
        hs = hs + linear(o2.transpose(1, 2).reshape(B, N_, -1), p + "attn2.to_out.0")
        n = F.layer_norm(hs, (D,), eps=c.eps) * (1 + sc2) + sh2
        n = n.unflatten(1, (H, W)).permute(0, 3, 1, 2)
        y = silu(F.conv2d(n, sd[p + "ff.conv_inverted.weight"], sd[p + "ff.conv_inverted.bias"]))
        y = F.conv2d(y, sd[p + "ff.conv_depth.weight"], sd[p + "ff.conv_depth.bias"], padding=1, groups=y.shape[1])
        y, gate = y.chunk(2, 1)
        y = F.conv2d(y * silu(gate), sd[p + "ff.conv_point.weight"])
        hs = hs + g2 * y.flatten(2, 3).permute(0, 2, 1)
    shift, scale = (sd["scale_shift_table"][None] + emb[:, None]).chunk(2, dim=1)
    hs = F.layer_norm(hs, (D,), eps=1e-6) * (1 + scale) + shift
    out = linear(hs, "proj_out")
    return out.reshape(B, H, W, 1, 1, -1).permute(0, 5, 1, 3, 2, 4).reshape(B, -1, H, W)


def _tr(device="cpu", dtype=torch.float32):
    with torch.device(device):
        tr = SA.SanaTransformer(SA.SANA_TEST)
    _perturb(tr, 1)
    from localai_tfp_amd.models.diffusion.nn import cast_module
    return cast_module(tr, device, dtype).eval()


def _inputs():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 32, 6, 8, generator=g)
    ctx = torch.randn(2, 9, SA.SANA_TEST.caption_channels, generator=g)
    return x, torch.tensor([700.0, 250.0]), ctx, torch.tensor([9, 5], dtype=torch.int32)


def test_sana_transformer_matches_reference():
    tr = _tr()
    x, t, ctx, kl = _inputs()
    got = tr(x, t, ctx, kl)
    ref = _ref_transformer(tr, x, t, ctx, kl).float()
    assert float((got - ref).norm() / ref.norm()) < 1e-4


def _ref_decoder(vae: SA.AutoencoderDC, z):
    c = vae.cfg
    sd = {k: v.double() for k, v in vae.state_dict().items()}

    def norm(x, p, kind):
        if kind == "batch_norm":
            return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                                False, 0.0, 1e-5)
        y = x.movedim(1, -1)
        y = y * torch.rsqrt(y.pow(2).mean(-1, keepdim=True) + 1e-5) * sd[p + ".weight"] + sd[p + ".bias"]
        return y.movedim(-1, 1)

    def conv(x, p, **kw):
        return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), **kw)
    x = z.double() / c.scaling
    h = conv(x, "decoder.conv_in", padding=1) + x.repeat_interleave(c.channels[-1] // c.latent, 1)
    n = len(c.channels)
    for i in reversed(range(n)):
        j = 0
        pre = f"decoder.up_blocks.{i}."
        if i < n - 1:
            y = conv(F.interpolate(h, scale_factor=2, mode="nearest"), pre + "0.conv", padding=1)
            h = y + F.pixel_shuffle(h.repeat_interleave(c.channels[i] * 4 // c.channels[i + 1], 1), 2)
            j = 1
        for _ in range(c.layers[i]):
            p = pre + f"{j}."
            if c.block_types[i] == "ResBlock":
                y = conv({"relu": F.relu, "silu": F.silu}[c.acts[i]](conv(h, p + "conv1", padding=1)), p + "conv2", padding=1)
                h = norm(y, p + "norm", c.norms[i]) + h
            else:
                B, _, H, W = h.shape
                hl = h.movedim(1, -1)
                qkv = torch.cat([hl @ sd[p + f"attn.to_{t}.weight"].T for t in "qkv"], -1).movedim(-1, 1)
                ms = [qkv]
                for s, k in enumerate(c.scales[i]):
                    q = f"{p}attn.to_qkv_multiscale.{s}."
                    y = F.conv2d(qkv, sd[q + "proj_in.weight"], padding=k // 2, groups=qkv.shape[1])
                    ms.append(F.conv2d(y, sd[q + "proj_out.weight"], groups=3 * (c.channels[i] // c.head_dim)))
                a = torch.cat(ms, 1).reshape(B, -1, 3 * c.head_dim, H * W)
                q_, k_, v_ = a.chunk(3, dim=2)
                q_, k_ = F.relu(q_), F.relu(k_)
                v_ = F.pad(v_, (0, 0, 0, 1), value=1.0)
                o = torch.matmul(torch.matmul(v_, k_.transpose(-1, -2)), q_)
                o = (o[:, :, :-1] / (o[:, :, -1:] + 1e-15)).reshape(B, -1, H, W)
                o = (o.movedim(1, -1) @ sd[p + "attn.to_out.weight"].T).movedim(-1, 1)
                h = norm(o, p + "attn.norm_out", c.norms[i]) + h
                y = F.silu(conv(h, p + "conv_out.conv_inverted"))
                y = F.conv2d(y, sd[p + "conv_out.conv_depth.weight"], sd[p + "conv_out.conv_depth.bias"], padding=1,
                             groups=y.shape[1])
                y, g = y.chunk(2, 1)
                y = conv(y * F.silu(g), p + "conv_out.conv_point")
                h = norm(y, p + "conv_out.norm", "rms_norm") + h
            j += 1
    h = F.relu(norm(h, "decoder.norm_out", "rms_norm"))
    return conv(h, "decoder.conv_out", padding=1)


def test_dcae_decoder_matches_reference():
    with torch.device("cpu"):
        vae = SA.AutoencoderDC(SA.DCAE_TEST)
    _perturb(vae, 2)
    vae.eval()
    z = torch.randn(1, 32, 3, 4, generator=torch.Generator().manual_seed(1))
    got = vae.decode(z)
    ref = _ref_decoder(vae, z).float()
    assert got.shape == (1, 3, 12, 16)
    assert float((got - ref).norm() / ref.norm()) < 1e-4


def _write_dir(tmp_path):
    from safetensors.torch import save_file
    import test_lumina2 as TL
    root = tmp_path / "sana"
    root.mkdir()
    (root / "model_index.json").write_text(json.dumps({"_class_name": "SanaPipeline"}))
    tr = _perturb(SA.SanaTransformer(SA.SANA_TEST), 3)
    (root / "transformer").mkdir()
    save_file({k: v.contiguous() for k, v in tr.state_dict().items()}, str(root / "transformer" / "model.safetensors"))
    c = SA.SANA_TEST
    (root / "transformer" / "config.json").write_text(json.dumps({
        "_class_name": "SanaTransformer2DModel", "in_channels": 32, "out_channels": 32, "num_attention_heads": c.heads,
        "attention_head_dim": c.head_dim, "num_layers": c.layers, "num_cross_attention_heads": c.cross_heads,
        "cross_attention_head_dim": c.cross_head_dim, "cross_attention_dim": c.dim, "caption_channels": 64,
        "mlp_ratio": 2.5, "attention_bias": False, "sample_size": 32, "patch_size": 1, "norm_eps": 1e-6,
        "interpolation_scale": None}))
    TL._gemma_dir(root)  # hidden 64 == caption_channels
    TL._tokenizer_dir(root / "tokenizer")
    vae = _perturb(SA.AutoencoderDC(SA.DCAE_TEST), 4)
    sdv = {k: v.contiguous() for k, v in vae.state_dict().items()}
    sdv["encoder.conv_in.weight"] = torch.zeros(16, 3, 3, 3)  # encoder weights present in real files: ignored
    (root / "vae").mkdir()
    save_file(sdv, str(root / "vae" / "model.safetensors"))
    d = SA.DCAE_TEST
    (root / "vae" / "config.json").write_text(json.dumps({
        "_class_name": "AutoencoderDC", "in_channels": 3, "latent_channels": 32, "attention_head_dim": d.head_dim,
        "decoder_block_types": list(d.block_types), "decoder_block_out_channels": list(d.channels),
        "decoder_layers_per_block": list(d.layers), "decoder_qkv_multiscales": [list(s) for s in d.scales],
        "decoder_norm_types": list(d.norms), "decoder_act_fns": list(d.acts), "upsample_block_type": "interpolate",
        "scaling_factor": 0.41407}))
    (root / "scheduler").mkdir()
    (root / "scheduler" / "scheduler_config.json").write_text(json.dumps({
        "_class_name": "DPMSolverMultistepScheduler", "flow_shift": 3.0, "prediction_type": "flow_prediction"}))
    return root, tr, vae


def test_sana_diffusers_dir_through_worker(tmp_path):
    import sys
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).parent))
    root, tr, vae = _write_dir(tmp_path)
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    s = DiffusionServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model=str(root)), None)
    assert r.success, r.message
    assert type(s.pipe).__name__ == "SanaPipeline" and s.defaults["cfg_scale"] == 4.5
    got = s.pipe.vae.state_dict()
    assert all(torch.equal(got[k], v) for k, v in vae.state_dict().items())
    dst = str(tmp_path / "o.png")
    r = s.GenerateImage(pb.GenerateImageRequest(positive_prompt="a red fox", width=64, height=64, step=2, seed=3,
                                                dst=dst), None)
    assert r.success, r.message
    from PIL import Image
    with Image.open(dst) as im:
        assert im.size == (64, 64)


def test_sana_prompt_selection():
    """Complex-human-instruction prompts keep BOS + the last max_tokens-1 positions of the padded sequence."""
    p = SA.SanaPipeline.synthetic("sana-test", "cpu")
    p.chi = True
    rows, n = p.encode_prompt("a red fox", True)
    ids = p.tok.encode("\n".join(SA.COMPLEX_HUMAN_INSTRUCTION) + "a red fox")
    h = p.te.prompt_hidden(ids)
    n_pre = len(p.tok.encode("\n".join(SA.COMPLEX_HUMAN_INSTRUCTION)))
    L = n_pre + p.max_tokens - 2
    sel = [0] + [i for i in range(L - p.max_tokens + 1, L) if i < len(ids)]
    assert n == len(sel) and torch.allclose(rows[:n], h[sel]) and float(rows[n:].abs().sum()) == 0


@pytest.mark.gpu
def test_sana_transformer_gpu():
    import copy
    from localai_tfp_amd.models.diffusion.nn import cast_module
    tr = _tr()  # weights drawn on the CPU (a CUDA generator would draw different ones)
    trg = cast_module(copy.deepcopy(tr), "cuda", torch.bfloat16)
    x, t, ctx, kl = _inputs()
    ref = tr(x, t, ctx, kl)
    got = trg(x.cuda(), t.cuda(), ctx.cuda(), kl.cuda()).cpu()
    assert float((got - ref).norm() / ref.norm()) < 3e-2


@pytest.mark.gpu
def test_dwconv3_glu_kernel():
    torch.manual_seed(0)
    B, H, W, Ch = 2, 7, 9, 40
    conv = torch.nn.Conv2d(2 * Ch, 2 * Ch, 3, padding=1, groups=2 * Ch)
    x = torch.randn(B * H * W, 2 * Ch).bfloat16()
    ref = SA.dwconv3_glu(x.float(), conv, B, H, W, True)
    got = SA.dwconv3_glu(x.cuda(), conv.cuda(), B, H, W, True).cpu()
    assert float((got.float() - ref).norm() / ref.norm()) < 1e-2
