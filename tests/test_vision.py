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
