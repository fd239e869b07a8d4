"""Kokoro-82M (the reference's kokoro backend, backend/python/kokoro/backend.py:47-99; model code in
kokoro/models.py, istftnet.py, kokoro.py, plbert.py).

* the PL-BERT tower (ALBERT, shared layers) equals transformers' AlbertModel on the same weights;
* checkpoint loading: {"net": {...}} with "module." prefixes and weight-norm (weight_g / weight_v) pairs
  folds to the plain weights;
* text normalisation / tokenisation follow kokoro.py's rules and symbol table;
* the full synthesis path runs end to end and the worker writes a 24 kHz WAV with single and averaged
  (`a+b`) voice packs.
No Kokoro weights / espeak-ng here: audio parity is unpinned."""
import math
import wave

import numpy as np
import pytest
import torch

from localai_tfp_amd.models import kokoro as KK

transformers = pytest.importorskip("transformers")


def test_albert_matches_transformers():
    c = KK.KOKORO_TEST
    P = KK.synthetic_params(c, 3)
    T = transformers
    hc = T.AlbertConfig(vocab_size=c.n_token, embedding_size=c.bert_emb, hidden_size=c.bert_hidden,
                        num_attention_heads=c.bert_heads, intermediate_size=c.bert_inter,
                        num_hidden_layers=c.bert_layers, max_position_embeddings=c.bert_max_pos,
                        hidden_act="gelu_new")
    hm = T.AlbertModel(hc, add_pooling_layer=False).eval()
    sd = {k[len("bert."):]: v for k, v in P.items() if k.startswith("bert.")}
    missing, unexpected = hm.load_state_dict(sd, strict=False)
    assert not unexpected and all("position_ids" in m or "token_type_ids" in m for m in missing), (missing, unexpected)
    ids = torch.tensor([0, 5, 17, 43, 100, 2, 150, 0])
    with torch.no_grad():
        ref = hm(ids[None]).last_hidden_state[0]
    got = KK.Kokoro(c, P).bert(ids)
    assert float((got - ref).norm() / ref.norm()) < 1e-5


def test_weight_norm_folding_and_prefix(tmp_path):
    g = torch.Generator().manual_seed(0)
    v = torch.randn(6, 4, 3, generator=g)
    gg = torch.rand(6, 1, 1, generator=g) + 0.5
    ck = {"net": {"decoder": {"module.F0_conv.weight_g": gg, "module.F0_conv.weight_v": v,
                              "module.F0_conv.bias": torch.ones(6)}}}
    p = tmp_path / "k.pth"
    torch.save(ck, str(p))
    got = KK.load_checkpoint(str(p))
    want = gg * v / v.norm(dim=(1, 2), keepdim=True)
    assert set(got) == {"decoder.F0_conv.weight", "decoder.F0_conv.bias"}
    assert torch.allclose(got["decoder.F0_conv.weight"], want, atol=1e-6)


def test_text_rules():
    assert KK.normalize_text("Dr. Smith met Mr. Jones at 10:05 in 1985.") == \
        "Doctor Smith met Mister Jones at 10 oh 5 in 19 85."
    assert KK.normalize_text("It costs 3.14, from 5-7") == "It costs 3 point 1 4, from 5 to 7"
    assert KK.VOCAB["$"] == 0 and KK.VOCAB[";"] == 1 and KK.VOCAB["A"] == 17 and max(KK.VOCAB.values()) < 178
    ps = KK.phonemize("Hello there.")
    assert ps and all(ch in KK.VOCAB for ch in ps)
    assert KK.tokenize("ab$") == [KK.VOCAB["a"], KK.VOCAB["b"], 0]


def _write_model(tmp_path, seed=2):
    c = KK.KOKORO_TEST
    P = KK.synthetic_params(c, seed)
    net = {}
    for k, v in P.items():
        part, rest = k.split(".", 1)
        net.setdefault(part, {})["module." + rest] = v
    torch.save({"net": net}, str(tmp_path / "kokoro-test.pth"))
    gv = torch.Generator().manual_seed(5)
    torch.save(torch.randn(511, 1, 2 * c.style, generator=gv), str(tmp_path / "af.pt"))
    torch.save(torch.randn(511, 1, 2 * c.style, generator=gv), str(tmp_path / "am.pt"))
    return c, P


def test_kokoro_worker_end_to_end(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.kokoro import KokoroServicer
    c, P = _write_model(tmp_path)
    s = KokoroServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="kokoro", ModelFile=str(tmp_path / "kokoro-test.pth"),
                                    ModelPath=str(tmp_path), Options=["voice:af"]), None)
    assert r.success, r.message
    assert s.model.cfg == KK.config_for(s.model.p) and s.model.cfg.upsample_rates == c.upsample_rates
    dst = str(tmp_path / "o.wav")
    r = s.TTS(pb.TTSRequest(text="Hello world.", model="kokoro", dst=dst), None)
    assert r.success, r.message
    with wave.open(dst) as w:
        assert w.getframerate() == 24000 and w.getnframes() > 0
    # averaged voice packs; missing voice refused as in the reference
    r = s.LoadModel(pb.ModelOptions(Model="kokoro", ModelFile=str(tmp_path / "kokoro-test.pth"),
                                    ModelPath=str(tmp_path), Options=["voice:af+am"]), None)
    assert r.success
    a = torch.load(str(tmp_path / "af.pt"), weights_only=True)
    b = torch.load(str(tmp_path / "am.pt"), weights_only=True)
    assert torch.allclose(s.voice, (a + b) / 2)
    r = s.LoadModel(pb.ModelOptions(Model="kokoro", ModelFile=str(tmp_path / "kokoro-test.pth"),
                                    ModelPath=str(tmp_path)), None)
    assert not r.success and "voice" in r.message


def test_kokoro_durations_and_length():
    """Audio length = (2 x aligned frames) x prod(upsample rates) x hop; deterministic per seed."""
    c = KK.KOKORO_TEST
    m = KK.Kokoro(c, KK.synthetic_params(c, 4))
    toks = KK.tokenize(KK.phonemize("A short test."))
    ref = torch.randn(1, 2 * c.style, generator=torch.Generator().manual_seed(1))
    a1, a2 = m.synthesize(toks, ref, seed=3), m.synthesize(toks, ref, seed=3)
    assert np.array_equal(a1, a2) and np.isfinite(a1).all()
    L = len(toks) + 2
    ids = torch.tensor([0, *toks, 0])
    with torch.no_grad():
        d_en = m._lin(m.bert(ids), "bert_encoder")
    assert d_en.shape == (L, c.hidden)
    per_frame = 2 * int(np.prod(c.upsample_rates)) * c.hop
    assert len(a1) % per_frame == 0


@pytest.mark.gpu
def test_kokoro_gpu_matches_cpu():
    c = KK.KOKORO_TEST
    P = KK.synthetic_params(c, 6)
    toks = KK.tokenize(KK.phonemize("Testing the GPU path."))
    ids = torch.tensor([0, *toks, 0])
    cpu, gpu = KK.Kokoro(c, P, "cpu"), KK.Kokoro(c, P, "cuda")
    a = cpu.bert(ids)
    b = gpu.bert(ids.cuda()).cpu()
    assert float((a - b).norm() / a.norm()) < 2e-2  # bf16 flash attention inside
    ref = torch.randn(1, 2 * c.style, generator=torch.Generator().manual_seed(2))
    wav = gpu.synthesize(toks, ref, seed=1)
    assert np.isfinite(wav).all() and len(wav) > 0


def test_kokoro_pool_up2_matches_conv_transpose():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 6, 11, generator=g)
    w = torch.randn(6, 1, 3, generator=g)
    b = torch.randn(6, generator=g)
    want = torch.nn.functional.conv_transpose1d(x, w, b, stride=2, padding=1, output_padding=1, groups=6)
    assert torch.allclose(KK.Kokoro._pool_up2(x, w, b), want, atol=1e-6)
