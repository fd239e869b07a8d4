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
