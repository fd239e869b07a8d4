"""Multimodal (LLaVA) path: CLIP vision tower + mlp2x projector vs transformers' CLIPVisionModel
(penultimate-layer features, CLS dropped) and LLaVA projector with the same weights; `[img-N]`
prompt splitting (grpc-server.cpp:900-944); embedding splicing through the engine (chunked prefill)
checked against the equivalent token prompt; the LLM worker Predict with Images and an mmproj."""
import base64
import io

import numpy as np
import pytest
import torch

from localai_tfp_amd.models import vision as V

transformers = pytest.importorskip("transformers")


def _png(seed=0, size=(40, 30)):
    from PIL import Image
    rng = np.random.default_rng(seed)
    im = Image.fromarray(rng.integers(0, 255, (size[1], size[0], 3), dtype=np.uint8))
    b = io.BytesIO()
    im.save(b, "PNG")
    return base64.b64encode(b.getvalue()).decode()


def test_clip_tower_matches_transformers():
    from transformers import CLIPVisionConfig, CLIPVisionModel
    cfg = V.CLIP_TEST
    hc = CLIPVisionConfig(hidden_size=cfg.hidden, intermediate_size=cfg.ffn, num_hidden_layers=cfg.layers + 1,
                          num_attention_heads=cfg.heads, image_size=cfg.image_size, patch_size=cfg.patch,
                          layer_norm_eps=cfg.eps, hidden_act="quick_gelu")
    torch.manual_seed(0)
    hm = CLIPVisionModel(hc).eval()
    hs = hm.state_dict()
    sd = {"v.patch_embd.weight": hs["embeddings.patch_embedding.weight"],
          "v.class_embd": hs["embeddings.class_embedding"],
          "v.position_embd.weight": hs["embeddings.position_embedding.weight"],
          "v.pre_ln.weight": hs["pre_layrnorm.weight"], "v.pre_ln.bias": hs["pre_layrnorm.bias"]}
    for i in range(cfg.layers):
        q, p = f"encoder.layers.{i}.", f"v.blk.{i}."
        for a, b in (("q_proj", "attn_q"), ("k_proj", "attn_k"), ("v_proj", "attn_v"), ("out_proj", "attn_out")):
            sd[p + b + ".weight"], sd[p + b + ".bias"] = hs[q + f"self_attn.{a}.weight"], hs[q + f"self_attn.{a}.bias"]
        for a, b in (("layer_norm1", "ln1"), ("layer_norm2", "ln2"), ("mlp.fc1", "ffn_down"), ("mlp.fc2", "ffn_up")):
            sd[p + b + ".weight"], sd[p + b + ".bias"] = hs[q + a + ".weight"], hs[q + a + ".bias"]
    g = torch.Generator().manual_seed(1)
    P = cfg.proj_hidden
    l1w, l1b = torch.randn(P, cfg.hidden, generator=g) * 0.05, torch.randn(P, generator=g) * 0.05
    l2w, l2b = torch.randn(P, P, generator=g) * 0.05, torch.randn(P, generator=g) * 0.05
    sd.update({"mm.0.weight": l1w, "mm.0.bias": l1b, "mm.2.weight": l2w, "mm.2.bias": l2b})
    ours = V.ClipVision(cfg, sd, "cpu")
    px = torch.stack([ours.preprocess(_png(i)) for i in range(2)])
    with torch.no_grad():
        feats = hm(pixel_values=px, output_hidden_states=True).hidden_states[-2][:, 1:]
        ref = torch.nn.functional.gelu(feats @ l1w.t() + l1b) @ l2w.t() + l2b
    got = ours.encode(px)
    assert got.shape == ref.shape == (2, cfg.n_patches, P)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4)


def test_split_prompt():
    assert V.split_prompt("a [img-0] b [img-1] c", 2) == ["a ", 0, " b ", 1, " c"]
    assert V.split_prompt("no images", 1) == ["no images"]
    with pytest.raises(ValueError):
        V.split_prompt("x [img-3]", 1)
    with pytest.raises(ValueError):
        V.split_prompt("x [img-a]", 1)


def test_engine_splices_embeddings_like_tokens():
    """Injecting the token-embedding rows of ids b, c at their positions must reproduce the plain
    token prompt exactly (exercises chunk boundaries: max_batched_tokens=8)."""
    from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
    from localai_tfp_amd.engine.sequence import Request
    from localai_tfp_amd.models.config import tiny_config
    from localai_tfp_amd.models.llama import LlamaModel
    from localai_tfp_amd.models.synthetic import synthetic_source
    from localai_tfp_amd.ops.sampling import SamplingParams
    from localai_tfp_amd.tokenizer import ByteTokenizer
    cfg = tiny_config(n_layers=2)
    m = LlamaModel.load(cfg, synthetic_source(cfg, "Q8_0", seed=4), "cpu")
    tok = ByteTokenizer(cfg.vocab)
    eng = LLMEngine(m, tok, EngineConfig(num_blocks=128, max_num_seqs=4, max_batched_tokens=8, max_model_len=256))
    prompt = [1, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51]
    ref = eng.generate(prompt, SamplingParams(temperature=0.0), max_tokens=6).token_ids
    E = m.tok_embd.dense_f32()
    span = prompt[3:11]
    ph = prompt[:3] + [0] * len(span) + prompt[11:]
    req = Request(ph, SamplingParams(temperature=0.0), 6)
    req.mm_embeds = [(3, E[torch.tensor(span)].float())]
    req.cache_prompt = False
    h = eng.submit(req)
    eng.run_until_done()
    got = [t for o in h for t in o.token_ids]
    assert got == ref
    # a plain request with the placeholder ids afterwards must not reuse the spliced KV blocks
    o = eng.generate(ph, SamplingParams(temperature=0.0), max_tokens=6)
    assert o.cached_tokens == 0


def test_worker_predict_with_image():
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    s = LLMServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:tiny", MMProj="synthetic:clip-test", Options=["lazy_graphs"]), None)
    assert r.success, r.message
    req = s._request(pb.PredictOptions(Prompt="USER: [img-0] what is this? ASSISTANT:", Images=[_png(3)], Tokens=4))
    assert len(req.mm_embeds) == 1 and req.mm_embeds[0][1].shape == (V.CLIP_TEST.n_patches, 256)
    p0 = req.mm_embeds[0][0]
    assert req.prompt_ids[p0:p0 + V.CLIP_TEST.n_patches] == [0] * V.CLIP_TEST.n_patches and not req.cache_prompt
    req2 = s._request(pb.PredictOptions(Prompt="describe", Images=[_png(1), _png(2)], Tokens=4))
    assert [p for p, _ in req2.mm_embeds] == [1, 1 + V.CLIP_TEST.n_patches]  # BOS, then both images, then text
    s.engine.shutdown()


@pytest.mark.gpu
def test_clip_tower_gpu_matches_cpu():
    sd = V.synthetic_clip(V.CLIP_TEST, 2)
    c, g = V.ClipVision(V.CLIP_TEST, sd, "cpu"), V.ClipVision(V.CLIP_TEST, sd, "cuda:0")
    px = torch.stack([c.preprocess(_png(i)) for i in range(3)])
    a, b = c.encode(px), g.encode(px).cpu()
    assert float((a - b).norm() / a.norm()) < 1e-2


# ------------------------------------------------------------------------------------------------ LLaVA-1.6 anyres
def test_select_best_resolution_matches_transformers():
    """clip.cpp's canvas choice == transformers' select_best_resolution (which takes (height, width) pairs)."""
    from transformers.image_processing_utils import select_best_resolution as hf_sel
    pins = V.LLAVA16.grid_pinpoints
    for w, h in ((640, 480), (480, 640), (336, 336), (1200, 300), (300, 1200), (1000, 1000), (50, 700), (700, 52)):
        hh, ww = hf_sel((h, w), [(ph, pw) for pw, ph in pins])
        assert V.select_best_resolution((w, h), pins) == (ww, hh), (w, h)


def test_anyres_crops_and_packing():
    """llava.cpp's LLaVA-1.6 path: whole-image crop + row-major grid crops of the best canvas, each through the tower
    and projector; grid features re-ordered into the canvas raster exactly as transformers' LlavaNext arranges them
    before its unpad step (view(nh, nw, h, w, C) -> permute(4, 0, 2, 1, 3)); no image_newline rows."""
    from PIL import Image
    cfg = V.CLIP_TEST_ANYRES
    vis = V.ClipVision(cfg, V.synthetic_clip(cfg, 5), "cpu")
    rng = np.random.default_rng(9)
    im = Image.fromarray(rng.integers(0, 255, (30, 70, 3), dtype=np.uint8))  # wide: the (112, 56) canvas
    crops, (gw, gh) = vis.anyres_crops(im)
    assert (gw, gh) == (2, 1) and len(crops) == 3 and all(c.shape == (3, 56, 56) for c in crops)
    canvas = V.resize_and_pad(im, (112, 56))
    assert torch.allclose(crops[2], vis.normalise(canvas.crop((56, 0, 112, 56))))
    out = vis.embed_anyres(im)
    side = 4
    assert out.shape == ((1 + gw * gh) * side * side, cfg.proj_hidden)
    feats = vis.encode(torch.stack(crops))
    assert torch.allclose(out[:16], feats[0])
    hf = feats[1:].view(gh, gw, side, side, -1).permute(4, 0, 2, 1, 3).flatten(1, 2).flatten(2, 3)  # [C, H, W]
    assert torch.allclose(out[16:], hf.flatten(1, 2).transpose(0, 1))


def test_worker_predict_with_anyres_image():
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    s = LLMServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:tiny", MMProj="synthetic:clip-test-anyres",
                                    Options=["lazy_graphs"]), None)
    assert r.success, r.message
    req = s._request(pb.PredictOptions(Prompt="USER: [img-0] what is this? ASSISTANT:", Images=[_png(3, (90, 40))],
                                       Tokens=3))
    n = req.mm_embeds[0][1].shape[0]
    assert n == 16 * 3  # whole image + a 2 x 1 grid of 4 x 4 patches
    import asyncio
    res = asyncio.run(s.Predict(pb.PredictOptions(Prompt="USER: [img-0] what is this? ASSISTANT:",
                                                  Images=[_png(3, (90, 40))], Tokens=3), None))
    assert res.tokens == 3
    s.engine.shutdown()


# ------------------------------------------------------------------------------------------------ Gemma-3 (SigLIP)
def _gemma3_hf(cfg, seed=0):
    from transformers import Gemma3Config, SiglipVisionConfig, SiglipVisionModel
    from transformers.models.gemma3.modeling_gemma3 import Gemma3MultiModalProjector
    vc = SiglipVisionConfig(hidden_size=cfg.hidden, intermediate_size=cfg.ffn, num_hidden_layers=cfg.layers,
                            num_attention_heads=cfg.heads, image_size=cfg.image_size, patch_size=cfg.patch,
                            layer_norm_eps=cfg.eps, hidden_act="gelu_pytorch_tanh")
    gc = Gemma3Config(vision_config=vc.to_dict(), text_config={"hidden_size": cfg.proj_hidden, "vocab_size": 64,
                                                                "num_hidden_layers": 1},
                      mm_tokens_per_image=cfg.tokens_per_image)
    torch.manual_seed(seed)
    tower = SiglipVisionModel(vc).eval()
    proj = Gemma3MultiModalProjector(gc).eval()
    with torch.no_grad():
        proj.mm_input_projection_weight.normal_(0, 0.05)
        proj.mm_soft_emb_norm.weight.normal_(0, 0.1)
        for p in tower.parameters():  # non-trivial LayerNorm / bias values
            p.add_(torch.randn_like(p) * 0.02)
    return tower, proj


def _gemma3_sd(tower, proj, cfg):
    """transformers state dicts -> the mmproj GGUF tensor names (convert_hf_to_gguf Gemma3 vision: fc1 -> ffn_up,
    soft_emb_norm stored as 1 + w, mm_input_projection as is)."""
    hs = tower.state_dict()
    pre = "vision_model." if any(k.startswith("vision_model.") for k in hs) else ""
    sd = {"v.patch_embd.weight": hs[pre + "embeddings.patch_embedding.weight"],
          "v.patch_embd.bias": hs[pre + "embeddings.patch_embedding.bias"],
          "v.position_embd.weight": hs[pre + "embeddings.position_embedding.weight"],
          "v.post_ln.weight": hs[pre + "post_layernorm.weight"], "v.post_ln.bias": hs[pre + "post_layernorm.bias"],
          "mm.soft_emb_norm.weight": proj.mm_soft_emb_norm.weight.detach() + 1,
          "mm.input_projection.weight": proj.mm_input_projection_weight.detach()}
    for i in range(cfg.layers):
        q, p = f"{pre}encoder.layers.{i}.", f"v.blk.{i}."
        for a, b in (("q_proj", "attn_q"), ("k_proj", "attn_k"), ("v_proj", "attn_v"), ("out_proj", "attn_out")):
            sd[p + b + ".weight"], sd[p + b + ".bias"] = hs[q + f"self_attn.{a}.weight"], hs[q + f"self_attn.{a}.bias"]
        for a, b in (("layer_norm1", "ln1"), ("layer_norm2", "ln2"), ("mlp.fc1", "ffn_up"), ("mlp.fc2", "ffn_down")):
            sd[p + b + ".weight"], sd[p + b + ".bias"] = hs[q + a + ".weight"], hs[q + a + ".bias"]
    return sd


def test_gemma3_projector_matches_transformers():
    """Gemma-3 image embeddings (clip.cpp PROJECTOR_TYPE_GEMMA3): SigLIP tower (patch bias, no CLS, post-LN, tanh
    GELU) -> average pool to tokens_per_image -> (1 + w) RMSNorm -> projection, against transformers'
    SiglipVisionModel + Gemma3MultiModalProjector with the same weights (get_image_features)."""
    cfg = V.GEMMA3_TEST
    tower, proj = _gemma3_hf(cfg)
    ours = V.ClipVision(cfg, _gemma3_sd(tower, proj, cfg), "cpu")
    px = torch.stack([ours.preprocess(_png(i)) for i in range(2)])
    with torch.no_grad():
        ref = proj(tower(pixel_values=px).last_hidden_state)
    got = ours.encode(px)
    assert got.shape == ref.shape == (2, cfg.tokens_per_image, cfg.proj_hidden)
    assert torch.allclose(got, ref, atol=2e-4, rtol=2e-4), float((got - ref).abs().max())


def test_gemma3_mmproj_gguf_roundtrip(tmp_path):
    """A gemma3 mmproj GGUF (projector_type gemma3, gguf-py tensor names, F16 weights) loads through load_mmproj and
    encodes like the in-memory tower."""
    from localai_tfp_amd.formats.gguf import GGUFWriter
    cfg = V.GEMMA3_TEST
    sd = V.synthetic_clip(cfg, 3)
    path = str(tmp_path / "mmproj-gemma3.gguf")
    w = GGUFWriter(path)
    for k, v in {"general.architecture": "clip", "clip.projector_type": "gemma3", "clip.has_vision_encoder": True,
                 "clip.vision.image_size": cfg.image_size, "clip.vision.patch_size": cfg.patch,
                 "clip.vision.embedding_length": cfg.hidden, "clip.vision.feed_forward_length": cfg.ffn,
                 "clip.vision.block_count": cfg.layers, "clip.vision.attention.head_count": cfg.heads,
                 "clip.vision.attention.layer_norm_epsilon": cfg.eps, "clip.vision.image_mean": list(cfg.mean),
                 "clip.vision.image_std": list(cfg.std), "clip.vision.projection_dim": cfg.proj_hidden,
                 "clip.vision.mm_tokens_per_image": cfg.tokens_per_image, "clip.use_gelu": True}.items():
        w.add(k, v)
    for k, t in sd.items():
        w.add_tensor(k, t.numpy().astype(np.float32))
    w.write()
    vis = V.load_mmproj(path)
    assert vis.cfg.projector == "gemma3" and vis.cfg.proj_hidden == cfg.proj_hidden
    ref = V.ClipVision(cfg, sd, "cpu")
    px = torch.stack([ref.preprocess(_png(7))])
    assert torch.allclose(vis.encode(px), ref.encode(px), atol=1e-5)
    assert vis.embed_images([_png(2)])[0].shape == (cfg.tokens_per_image, cfg.proj_hidden)


# ------------------------------------------------------------------------------------------------ Qwen2.5-VL
def _qwen_hf(cfg):
    from transformers.models.qwen2_5_vl.configuration_qwen2_5_vl import Qwen2_5_VLVisionConfig
    from transformers.models.qwen2_5_vl.modeling_qwen2_5_vl import Qwen2_5_VisionTransformerPretrainedModel
    vc = Qwen2_5_VLVisionConfig(depth=cfg.depth, hidden_size=cfg.hidden, intermediate_size=cfg.ffn,
                                num_heads=cfg.heads, out_hidden_size=cfg.out_hidden, window_size=cfg.window,
                                fullatt_block_indexes=list(cfg.fullatt), patch_size=cfg.patch,
                                spatial_merge_size=cfg.merge, temporal_patch_size=cfg.temporal, hidden_act="silu")
    vc._attn_implementation = "eager"
    torch.manual_seed(0)
    m = Qwen2_5_VisionTransformerPretrainedModel(vc).eval()
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.02)
    return m


@pytest.mark.parametrize("size", [(84, 56), (140, 100)])
def test_qwen25vl_vision_matches_transformers(size):
    """Qwen2.5-VL image embeddings: patch GEMM, 2-D RoPE, window / full attention blocks, SwiGLU MLP, patch merger
    and the window-order round trip against transformers' Qwen2_5_VisionTransformerPretrainedModel (same weights,
    same flattened patches); the preprocessing against Qwen2VLImageProcessor's pixel values and grid."""
    from PIL import Image
    from localai_tfp_amd.models import qwen_vl as QV
    cfg = QV.QWEN25VL_TEST
    hm = _qwen_hf(cfg)
    ours = QV.QwenVLVision(cfg, hm.state_dict(), "cpu")
    rng = np.random.default_rng(size[0])
    im = Image.fromarray(rng.integers(0, 255, (size[1], size[0], 3), dtype=np.uint8))
    px, grid = ours.patches([im])
    try:
        from transformers import Qwen2VLImageProcessor
        pr = Qwen2VLImageProcessor(min_pixels=cfg.min_pixels, max_pixels=cfg.max_pixels, patch_size=cfg.patch,
                                   merge_size=cfg.merge, temporal_patch_size=cfg.temporal)
        ref_in = pr(images=[im], return_tensors="pt")
        assert tuple(ref_in["image_grid_thw"][0].tolist()) == grid
        assert float((ref_in["pixel_values"] - px).abs().max()) < 0.05  # resize implementations differ slightly
    except ImportError:
        pass
    with torch.no_grad():
        out = hm(px, grid_thw=torch.tensor([grid]))
    ref = out.pooler_output if hasattr(out, "pooler_output") else out
    got = ours.encode_patches(px, grid)
    assert got.shape == ref.shape == (grid[0] * grid[1] * grid[2] // 4, cfg.out_hidden)
    assert torch.allclose(got, ref, atol=2e-4, rtol=2e-4), float((got - ref).abs().max())


def test_qwen25vl_video_frames_and_gguf_names():
    """A video as a frame list: frame pairs become temporal patches (grid_t = frames / 2), matching transformers on the
    same patches; and the clip.cpp-style tensor names map onto the same tower."""
    from PIL import Image
    from localai_tfp_amd.models import qwen_vl as QV
    cfg = QV.QWEN25VL_TEST
    hm = _qwen_hf(cfg)
    hs = hm.state_dict()
    ours = QV.QwenVLVision(cfg, hs, "cpu")
    rng = np.random.default_rng(3)
    frames = [Image.fromarray(rng.integers(0, 255, (56, 84, 3), dtype=np.uint8)) for _ in range(4)]
    px, grid = ours.patches(frames)
    assert grid == (2, 4, 6)
    with torch.no_grad():
        out = hm(px, grid_thw=torch.tensor([grid]))
    ref = out.pooler_output if hasattr(out, "pooler_output") else out
    assert torch.allclose(ours.embed_video(frames), ref, atol=2e-4, rtol=2e-4)
    # clip.cpp names: split q / k / v, the Conv3d's two temporal halves, merger as mm.0 / mm.2 + v.post_ln
    gg = {"v.patch_embd.weight": hs["patch_embed.proj.weight"][:, :, 0], "v.patch_embd.weight.1":
          hs["patch_embed.proj.weight"][:, :, 1], "v.post_ln.weight": hs["merger.ln_q.weight"],
          "mm.0.weight": hs["merger.mlp.0.weight"], "mm.0.bias": hs["merger.mlp.0.bias"],
          "mm.2.weight": hs["merger.mlp.2.weight"], "mm.2.bias": hs["merger.mlp.2.bias"]}
    H = cfg.hidden
    for i in range(cfg.depth):
        p, q = f"v.blk.{i}.", f"blocks.{i}."
        for j, n in enumerate(("attn_q", "attn_k", "attn_v")):
            gg[p + n + ".weight"] = hs[q + "attn.qkv.weight"][j * H:(j + 1) * H]
            gg[p + n + ".bias"] = hs[q + "attn.qkv.bias"][j * H:(j + 1) * H]
        for a, b in (("attn.proj", "attn_out"), ("mlp.gate_proj", "ffn_gate"), ("mlp.up_proj", "ffn_up"),
                     ("mlp.down_proj", "ffn_down")):
            gg[p + b + ".weight"], gg[p + b + ".bias"] = hs[q + a + ".weight"], hs[q + a + ".bias"]
        gg[p + "ln1.weight"], gg[p + "ln2.weight"] = hs[q + "norm1.weight"], hs[q + "norm2.weight"]
    o2 = QV.QwenVLVision(cfg, QV.from_gguf_names(gg), "cpu")
    assert torch.allclose(o2.embed_video(frames), ref, atol=2e-4, rtol=2e-4)


def test_split_media_markers():
    assert V.split_media("a [img-1] b [vid-0] c", 2, 1) == ["a ", ("img", 1), " b ", ("vid", 0), " c"]
    assert V.split_media("<|vision_start|><|image_pad|><|vision_end|>x<|video_pad|>", 1, 1) == \
        ["<|vision_start|>", ("img", 0), "<|vision_end|>x", ("vid", 0), ""]
    assert V.split_media("text", 1, 1) == ["", ("img", 0), "", ("vid", 0), "text"]
    with pytest.raises(ValueError):
        V.split_media("[vid-2]", 0, 1)


def _gif(n=4, size=(60, 40)):
    from PIL import Image
    rng = np.random.default_rng(n)
    frames = [Image.fromarray(rng.integers(0, 255, (size[1], size[0], 3), dtype=np.uint8)) for _ in range(n)]
    b = io.BytesIO()
    frames[0].save(b, "GIF", save_all=True, append_images=frames[1:], duration=40)
    return base64.b64encode(b.getvalue()).decode()


@pytest.mark.parametrize("proj", ["gemma3-test", "qwen25vl-test"])
def test_worker_predict_with_projectors(proj):
    """The LLM worker with a Gemma-3 (SigLIP) or Qwen2.5-VL mmproj: images spliced at [img-N] / the Qwen image pad,
    a video (animated GIF frames, vLLM's multi_modal_data["video"]) at the video pad, generation runs."""
    import asyncio
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    s = LLMServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:tiny", MMProj=f"synthetic:{proj}", Options=["lazy_graphs"]), None)
    assert r.success, r.message
    if proj == "gemma3-test":
        req = s._request(pb.PredictOptions(Prompt="USER: [img-0] what? ASSISTANT:", Images=[_png(4)], Tokens=3))
        assert [e.shape[0] for _, e in req.mm_embeds] == [V.GEMMA3_TEST.tokens_per_image]
        po = pb.PredictOptions(Prompt="[img-0] hi", Images=[_png(4)], Tokens=3)
    else:
        prompt = "<|vision_start|><|image_pad|><|vision_end|> and <|vision_start|><|video_pad|><|vision_end|>?"
        req = s._request(pb.PredictOptions(Prompt=prompt, Images=[_png(4, (70, 50))], Videos=[_gif()], Tokens=3))
        (p0, e0), (p1, e1) = req.mm_embeds
        assert p1 > p0 + e0.shape[0] and e1.shape[0] == 2 * 1 * 2  # 2 frame pairs x (28/28) x (56/28) merge groups
        po = pb.PredictOptions(Prompt=prompt, Images=[_png(4, (70, 50))], Videos=[_gif()], Tokens=3)
    res = asyncio.run(s.Predict(po, None))
    assert res.tokens == 3
    s.engine.shutdown()


@pytest.mark.gpu
def test_projectors_gpu_match_cpu():
    """Gemma-3 SigLIP + projector, LLaVA-1.6 anyres and Qwen2.5-VL (window attention through attention_dense.hip with
    per-window lengths) on the GPU against their fp32 CPU path."""
    from localai_tfp_amd.models import qwen_vl as QV
    for cfg in (V.GEMMA3_TEST, V.CLIP_TEST_ANYRES):
        sd = V.synthetic_clip(cfg, 2)
        c, g = V.ClipVision(cfg, sd, "cpu"), V.ClipVision(cfg, sd, "cuda:0")
        a = c.embed_images([_png(5, (90, 40))])[0]
        b = g.embed_images([_png(5, (90, 40))])[0].cpu()
        assert float((a - b).norm() / a.norm()) < 1e-2, cfg.name
    sd = QV.synthetic_qwen_vl(QV.QWEN25VL_TEST, 1)
    c, g = QV.QwenVLVision(QV.QWEN25VL_TEST, sd, "cpu"), QV.QwenVLVision(QV.QWEN25VL_TEST, sd, "cuda:0")
    a, b = c.embed_images([_png(6, (140, 100))])[0], g.embed_images([_png(6, (140, 100))])[0].cpu()
    assert float((a - b).norm() / a.norm()) < 1e-2
    from localai_tfp_amd.models import minicpmv as MC
    sd = MC.synthetic_minicpmv(MC.MINICPMV_TEST, 2)
    c, g = MC.MiniCPMVVision(MC.MINICPMV_TEST, sd, "cpu"), MC.MiniCPMVVision(MC.MINICPMV_TEST, sd, "cuda:0")
    a, b = c.embed_images([_png(7, (170, 60))])[0], g.embed_images([_png(7, (170, 60))])[0].cpu()
    assert float((a - b).norm() / a.norm()) < 1e-2


# ------------------------------------------------------------------------------------------------ MiniCPM-V
def test_minicpmv_slicing():
    """MiniCPM-V's slice grid / refine size (the published processor, as clip.cpp uhd_slice_image): small images are
    not sliced, wide ones get a log-aspect-matched grid, every piece is a multiple of the patch size."""
    from PIL import Image
    from localai_tfp_amd.models import minicpmv as MC
    assert MC.get_sliced_grid((448, 448), 448, 9) is None
    assert MC.get_sliced_grid((1344, 448), 448, 9) == [3, 1]
    assert MC.get_sliced_grid((896, 896), 448, 9) == [2, 2]
    assert MC.find_best_resize((1000, 500), 448, 14) == (630, 322)
    cfg = MC.MINICPMV_TEST
    parts = MC.slice_image(Image.new("RGB", (170, 60)), cfg)
    assert len(parts) == 1 + 3 and all(p.width % 14 == 0 and p.height % 14 == 0 for p in parts)
    assert len({p.size for p in parts[1:]}) == 1


def test_minicpmv_tower_and_resampler():
    """Tower at the native slice size == transformers' SiglipVisionModel (bucketed position ids are then the identity);
    the resampler == a torch.nn.MultiheadAttention re-statement (learned queries, ln_kv / ln_q / ln_post, sin-cos key
    positions, proj)."""
    from transformers import SiglipVisionConfig, SiglipVisionModel
    from localai_tfp_amd.models import minicpmv as MC
    cfg = MC.MINICPMV_TEST
    vc = cfg.vision
    hc = SiglipVisionConfig(hidden_size=vc.hidden, intermediate_size=vc.ffn, num_hidden_layers=vc.layers,
                            num_attention_heads=vc.heads, image_size=vc.image_size, patch_size=vc.patch,
                            layer_norm_eps=vc.eps, hidden_act="gelu_pytorch_tanh")
    torch.manual_seed(0)
    tower = SiglipVisionModel(hc).eval()
    with torch.no_grad():
        for p in tower.parameters():
            p.add_(torch.randn_like(p) * 0.02)
    proj = type("P", (), {})()
    proj.mm_soft_emb_norm = type("N", (), {"weight": torch.zeros(vc.hidden)})()
    proj.mm_input_projection_weight = torch.zeros(vc.hidden, 4)
    sd = {k: v for k, v in _gemma3_sd(tower, proj, vc).items() if not k.startswith("mm.")}
    sd.update({k: v for k, v in MC.synthetic_minicpmv(cfg, 1).items() if k.startswith("resampler.")})
    ours = MC.MiniCPMVVision(cfg, sd, "cpu")
    from PIL import Image
    im = Image.fromarray(np.random.default_rng(2).integers(0, 255, (56, 56, 3), dtype=np.uint8))
    px = ours.normalise(im)
    feats, hw = ours._tower(px)
    with torch.no_grad():
        ref = tower(pixel_values=px[None]).last_hidden_state[0]
    assert hw == (4, 4) and torch.allclose(feats, ref, atol=2e-4, rtol=2e-4)
    # resampler oracle
    E = cfg.embed_dim
    mha = torch.nn.MultiheadAttention(E, cfg.heads)
    with torch.no_grad():
        mha.in_proj_weight.copy_(torch.cat([sd[f"resampler.attn.{x}.weight"] for x in "qkv"]))
        mha.in_proj_bias.copy_(torch.cat([sd[f"resampler.attn.{x}.bias"] for x in "qkv"]))
        mha.out_proj.weight.copy_(sd["resampler.attn.out.weight"])
        mha.out_proj.bias.copy_(sd["resampler.attn.out.bias"])
        ln = lambda x, n: torch.nn.functional.layer_norm(x, (E,), sd[f"resampler.ln_{n}.weight"],  # noqa: E731
                                                        sd[f"resampler.ln_{n}.bias"], 1e-6)
        x = ln(feats @ sd["resampler.kv.weight"].t(), "kv")
        q = ln(sd["resampler.query"], "q")
        pos = MC.sincos_2d(E, 4, 4).reshape(16, E)
        o = mha(q[:, None], (x + pos)[:, None], x[:, None])[0][:, 0]
        want = ln(o, "post") @ sd["resampler.proj.weight"]
    got = ours._resample(feats, hw)
    assert torch.allclose(got, want, atol=2e-4, rtol=2e-4)


def test_worker_predict_with_minicpmv():
    import asyncio
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    s = LLMServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:tiny", MMProj="synthetic:minicpmv-test", Options=["lazy_graphs"]),
                    None)
    assert r.success, r.message
    req = s._request(pb.PredictOptions(Prompt="[img-0] what?", Images=[_png(4, (170, 60))], Tokens=3))
    assert req.mm_embeds[0][1].shape == (8 * 4, 256)  # source + 3 slices x 8 queries
    res = asyncio.run(s.Predict(pb.PredictOptions(Prompt="[img-0] what?", Images=[_png(4, (170, 60))], Tokens=3), None))
    assert res.tokens == 3
    s.engine.shutdown()
