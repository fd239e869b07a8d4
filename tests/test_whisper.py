"""Whisper backend: front end (log-mel vs torch.stft), encoder/decoder numerics vs a plain fp32
PyTorch Whisper, KV-cached decoding vs full recompute, timestamp segmentation, ggml container
round trip, the worker RPC and /v1/audio/transcriptions (reference coverage: core/http/app_test.go
transcription case, backend/go/transcribe/whisper)."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F
import yaml

from localai_tfp_amd.models import whisper as W
from localai_tfp_amd.tokenizer.whisper import WhisperTokenizer
from localai_tfp_amd.utils import audio as A

CFG = W.WHISPER_TEST


def ref_logmel(audio, filters):
    a = torch.from_numpy(np.concatenate([audio, np.zeros(W.N_SAMPLES, np.float32)]))
    st = torch.stft(a, W.N_FFT, W.HOP, window=torch.hann_window(W.N_FFT), return_complex=True)
    mag = st[..., :-1].abs() ** 2
    mel = torch.from_numpy(filters) @ mag
    log = mel.clamp(min=1e-10).log10()
    log = torch.maximum(log, log.max() - 8.0)
    return (log + 4.0) / 4.0


def ref_attn(x, xa, w, p, H, mask):
    q = x @ w[p + "query.weight"].T + w[p + "query.bias"]
    k = xa @ w[p + "key.weight"].T
    v = xa @ w[p + "value.weight"].T + w[p + "value.bias"]
    T, d = q.shape
    S = k.shape[0]
    hd = d // H
    q, k, v = (z.view(-1, H, hd).transpose(0, 1) for z in (q, k, v))
    s = q @ k.transpose(1, 2) / math.sqrt(hd)
    if mask:
        s = s + torch.triu(torch.full((T, S), float("-inf")), 1)
    o = (s.softmax(-1) @ v).transpose(0, 1).reshape(T, d)
    return o @ w[p + "out.weight"].T + w[p + "out.bias"]


def ln(x, w, p):
    return F.layer_norm(x, (x.shape[-1],), w[p + ".weight"], w[p + ".bias"], 1e-5)


def ref_encoder(mel, w):
    x = F.gelu(F.conv1d(mel[None], w["encoder.conv1.weight"], w["encoder.conv1.bias"], padding=1))
    x = F.gelu(F.conv1d(x, w["encoder.conv2.weight"], w["encoder.conv2.bias"], stride=2, padding=1))[0].T
    x = x + w["encoder.positional_embedding"]
    for i in range(CFG.n_audio_layer):
        p = f"encoder.blocks.{i}."
        h = ln(x, w, p + "attn_ln")
        x = x + ref_attn(h, h, w, p + "attn.", CFG.n_audio_head, False)
        h = ln(x, w, p + "mlp_ln")
        x = x + F.gelu(h @ w[p + "mlp.0.weight"].T + w[p + "mlp.0.bias"]) @ w[p + "mlp.2.weight"].T + w[p + "mlp.2.bias"]
    return ln(x, w, "encoder.ln_post")


def ref_decoder(tokens, xa, w):
    x = w["decoder.token_embedding.weight"][tokens] + w["decoder.positional_embedding"][:len(tokens)]
    for i in range(CFG.n_text_layer):
        p = f"decoder.blocks.{i}."
        h = ln(x, w, p + "attn_ln")
        x = x + ref_attn(h, h, w, p + "attn.", CFG.n_text_head, True)
        h = ln(x, w, p + "cross_attn_ln")
        x = x + ref_attn(h, xa, w, p + "cross_attn.", CFG.n_text_head, False)
        h = ln(x, w, p + "mlp_ln")
        x = x + F.gelu(h @ w[p + "mlp.0.weight"].T + w[p + "mlp.0.bias"]) @ w[p + "mlp.2.weight"].T + w[p + "mlp.2.bias"]
    return ln(x, w, "decoder.ln") @ w["decoder.token_embedding.weight"].T


@pytest.fixture(scope="module")
def weights():
    return W.synthetic_whisper(CFG, 7)


@pytest.fixture(scope="module")
def tw(weights):
    return {k: torch.from_numpy(v) for k, v in weights.items()}


def test_logmel_matches_stft():
    f = W.mel_filterbank()
    rng = np.random.default_rng(0)
    audio = (rng.standard_normal(16000 * 3) * 0.1).astype(np.float32)
    got = W.LogMel(f, "cpu")(torch.from_numpy(np.concatenate([audio, np.zeros(W.N_SAMPLES, np.float32)])))
    ref = ref_logmel(audio, f)
    assert got.shape == ref.shape
    assert (got - ref).abs().max() < 1e-3
    # filterbank rows are area-normalised triangles over 0..8 kHz
    assert f.shape == (80, 201) and (f >= 0).all() and (f.sum(1) > 0).all()


def test_encoder_decoder_match_reference(weights, tw):
    m = W.WhisperModel(CFG, weights.get, "cpu")
    rng = np.random.default_rng(1)
    mel = torch.from_numpy(rng.standard_normal((CFG.n_mels, W.N_FRAMES)).astype(np.float32) * 0.5)
    xa = m.encode(mel[None])
    ref = ref_encoder(mel, tw)
    assert (xa - ref).abs().max() < 2e-3
    toks = [50258, 50259, 50360, 400, 1234, 77]
    st = m.new_state(1)
    st.set_audio(xa)
    last = m.decode_prefix(st, [toks[:3]])
    full = ref_decoder(torch.tensor(toks), ref, tw)
    assert (last[0] - full[2]).abs().max() < 2e-3
    for i in range(3, len(toks)):  # KV-cached single steps == full recompute
        lg = m.decode_step(st, torch.tensor([toks[i]]))
        assert (lg[0] - full[i]).abs().max() < 2e-3, i


def test_beam_reorder_and_batch(weights):
    m = W.WhisperModel(CFG, weights.get, "cpu")
    mel = torch.zeros(1, CFG.n_mels, W.N_FRAMES)
    xa = m.encode(mel)
    st = m.new_state(2)
    st.set_audio(xa.repeat(2, 1))
    m.decode_prefix(st, [[50258, 50259], [50258, 50259]])
    a = m.decode_step(st, torch.tensor([10, 20]))
    st.reorder(torch.tensor([1, 1]))
    b = m.decode_step(st, torch.tensor([5, 5]))
    assert torch.allclose(b[0], b[1], atol=1e-6) and not torch.allclose(a[0], a[1])


def test_segments_from_timestamps():
    tok = WhisperTokenizer.synthetic()
    tr = W.Transcriber.__new__(W.Transcriber)
    tr.tok = tok
    tb = tok.timestamp_begin
    segs = []
    adv = tr._segments([tb + 0, 72, 105, tb + 50, tb + 50, 104, 105, tb + 120], 0.0, 3000, segs)
    assert [(s.start, s.end, s.text) for s in segs] == [(0.0, 1.0, "Hi"), (1.0, 2.4, "hi")]
    assert adv == 3000  # ends on a single timestamp after text -> whole window consumed
    segs = []
    adv = tr._segments([tb + 0, 72, tb + 50, tb + 50, 104, tb + 60, tb + 60], 0.0, 3000, segs)
    assert adv == 120 and len(segs) == 2


def test_timestamp_rules():
    tok = WhisperTokenizer.synthetic()
    tr = W.Transcriber.__new__(W.Transcriber)
    tr.tok = tok
    tr.suppress, tr.blank = [tok.sot], [tok.eot]
    tb = tok.timestamp_begin
    opt = W.DecodeOptions()
    lg = tr._apply_rules(np.zeros(tok.n_vocab), [], opt, True)
    assert np.isinf(lg[:tb]).all() and np.isfinite(lg[tb:tb + 51]).all() and np.isinf(lg[tb + 51:]).all()
    lg = tr._apply_rules(np.zeros(tok.n_vocab), [tb + 3, 100], opt, False)  # after text: ts >= last allowed
    assert np.isinf(lg[tb:tb + 4]).all() and np.isfinite(lg[tb + 4])
    lg = tr._apply_rules(np.zeros(tok.n_vocab), [tb + 3, 100, tb + 9], opt, False)  # open pair -> ts or eot
    assert np.isinf(lg[:tok.eot]).all()


def test_ggml_roundtrip_and_tokenizer(tmp_path, weights):
    from localai_tfp_amd.formats.ggml_whisper import write_ggml_whisper
    tok = WhisperTokenizer.synthetic()
    hp = dict(n_vocab=CFG.n_vocab, n_audio_ctx=CFG.n_audio_ctx, n_audio_state=CFG.n_audio_state,
              n_audio_head=CFG.n_audio_head, n_audio_layer=CFG.n_audio_layer, n_text_ctx=CFG.n_text_ctx,
              n_text_state=CFG.n_text_state, n_text_head=CFG.n_text_head, n_text_layer=CFG.n_text_layer,
              n_mels=CFG.n_mels, ftype=1)
    p = tmp_path / "ggml-test.bin"
    write_ggml_whisper(str(p), hp, W.mel_filterbank(), tok.pieces, weights)
    m, t2 = W.load_whisper(str(p), "cpu")
    assert m.cfg.n_text_state == CFG.n_text_state and t2.sot == 50258 and t2.timestamp_begin == 50364
    a = W.WhisperModel(CFG, weights.get, "cpu")
    mel = torch.zeros(1, CFG.n_mels, W.N_FRAMES)
    assert (m.encode(mel) - a.encode(mel)).abs().max() < 5e-2  # fp16-stored weights
    assert t2.decode(t2.encode("hello world")) == "hello world"


def test_transcribe_and_worker(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.whisper import WhisperServicer
    sr = 16000
    x = (0.3 * np.sin(2 * np.pi * 220 * np.arange(int(2.5 * sr)) / sr)).astype(np.float32)
    wav = tmp_path / "a.wav"
    A.write_wav(str(wav), x, 44100 if False else sr)
    s = WhisperServicer(device="cpu")
    assert s.LoadModel(pb.ModelOptions(Model="synthetic:whisper-test", Options=["temperatures:0"]), None).success
    r = s.AudioTranscription(pb.TranscriptRequest(dst=str(wav), language="en"), None)
    assert isinstance(r.text, str)
    for seg in r.segments:
        assert 0 <= seg.start <= seg.end


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    from fastapi.testclient import TestClient
    from localai_tfp_amd.config.app_config import ApplicationConfig
    from localai_tfp_amd.gateway.app import create_app
    d = tmp_path_factory.mktemp("wh")
    models = d / "models"
    models.mkdir()
    (models / "whisper-1.yaml").write_text(yaml.safe_dump({
        "name": "whisper-1", "backend": "whisper", "parameters": {"model": "synthetic:whisper-test"},
        "options": ["temperatures:0"]}))
    cfg = ApplicationConfig(models_path=str(models), generated_content_dir=str(d / "gen"),
                            upload_dir=str(d / "up"), config_dir=str(d / "cfg"), api_keys=[])
    app = create_app(cfg, inproc=True)
    with TestClient(app) as c:
        yield c
    app.state.localai.shutdown()


def test_http_transcription(client):
    x = (0.2 * np.sin(np.arange(16000) / 10)).astype(np.float32)
    r = client.post("/v1/audio/transcriptions", files={"file": ("a.wav", A.wav_bytes(x), "audio/wav")},
                    data={"model": "whisper-1"})
    assert r.status_code == 200, r.text
    j = r.json()
    assert "text" in j and isinstance(j["segments"], list)


@pytest.mark.gpu
def test_whisper_gpu_matches_cpu(weights):
    """GPU path (DFT-GEMM mel, im2col conv GEMMs, attention_dense.hip, norm.hip, hipGraph decode step)
    vs the fp32 CPU model."""
    cfg = W.WhisperConfig(n_audio_state=256, n_audio_head=4, n_audio_layer=2, n_text_state=256, n_text_head=4,
                          n_text_layer=2, name="t")
    w = W.synthetic_whisper(cfg, 3)
    c = W.WhisperModel(cfg, w.get, "cpu")
    g = W.WhisperModel(cfg, w.get, "cuda:0")
    rng = np.random.default_rng(2)
    audio = (rng.standard_normal(16000 * 4) * 0.1).astype(np.float32)
    mc, mg = c.log_mel(audio), g.log_mel(audio)
    assert (mg.cpu() - mc).abs().max() < 1e-2
    mel = mc[:, :W.N_FRAMES][None]
    xc, xg = c.encode(mel), g.encode(mel.cuda())
    assert ((xg.float().cpu() - xc).abs().max() / xc.abs().max()) < 3e-2
    toks = [50258, 50259, 50360, 400, 1234, 77, 5, 9]
    sc, sg = c.new_state(1), g.new_state(1)
    sc.set_audio(xc)
    sg.set_audio(xc.to("cuda:0", g.dtype))
    a, b = c.decode_prefix(sc, [toks[:3]]), g.decode_prefix(sg, [toks[:3]])
    assert (b.cpu() - a).abs().max() < 5e-2
    for t in toks[3:]:
        a = c.decode_step(sc, torch.tensor([t]))
        b = g.decode_step(sg, torch.tensor([t], device="cuda:0"))
        assert (b.cpu() - a).abs().max() < 5e-2
    assert sg.graph is not None


def _openai_to_ct2(w: dict, cfg, int8: bool) -> dict:
    """OpenAI names -> CTranslate2 WhisperSpec variables (written independently of the loader's map)."""
    v = {"encoder/num_heads": np.int16(cfg.n_audio_head), "decoder/num_heads": np.int16(cfg.n_text_head)}

    def q8(name, a):  # CTranslate2 int8: per-row scale 127 / amax, q = round(w * scale)
        if not int8 or a.ndim != 2 or "embedding" in name or "position" in name:
            v[name] = a.astype(np.float16) if int8 and a.ndim >= 2 else a
            return
        sc = 127.0 / np.maximum(np.abs(a).max(1), 1e-8)
        v[name] = np.clip(np.rint(a * sc[:, None]), -127, 127).astype(np.int8)
        v[name + "_scale"] = sc.astype(np.float32)
    for n in ("conv1", "conv2"):
        q8(f"encoder/{n}/weight", w[f"encoder.{n}.weight"])
        v[f"encoder/{n}/bias"] = w[f"encoder.{n}.bias"]
    v["encoder/position_encodings/encodings"] = w["encoder.positional_embedding"]
    v["decoder/position_encodings/encodings"] = w["decoder.positional_embedding"]
    v["decoder/embeddings/weight"] = w["decoder.token_embedding.weight"]
    for side, ln_ in (("encoder", "ln_post"), ("decoder", "ln")):
        v[f"{side}/layer_norm/gamma"], v[f"{side}/layer_norm/beta"] = w[f"{side}.{ln_}.weight"], w[f"{side}.{ln_}.bias"]
    for side, n in (("encoder", cfg.n_audio_layer), ("decoder", cfg.n_text_layer)):
        for i in range(n):
            p, o = f"{side}/layer_{i}", f"{side}.blocks.{i}."
            d = w[o + "attn.query.weight"].shape[0]
            v[f"{p}/self_attention/layer_norm/gamma"] = w[o + "attn_ln.weight"]
            v[f"{p}/self_attention/layer_norm/beta"] = w[o + "attn_ln.bias"]
            q8(f"{p}/self_attention/linear_0/weight", np.concatenate([w[o + f"attn.{x}.weight"] for x in ("query", "key", "value")]))
            v[f"{p}/self_attention/linear_0/bias"] = np.concatenate([w[o + "attn.query.bias"], np.zeros(d, np.float32), w[o + "attn.value.bias"]])
            q8(f"{p}/self_attention/linear_1/weight", w[o + "attn.out.weight"])
            v[f"{p}/self_attention/linear_1/bias"] = w[o + "attn.out.bias"]
            if side == "decoder":
                v[f"{p}/attention/layer_norm/gamma"] = w[o + "cross_attn_ln.weight"]
                v[f"{p}/attention/layer_norm/beta"] = w[o + "cross_attn_ln.bias"]
                q8(f"{p}/attention/linear_0/weight", w[o + "cross_attn.query.weight"])
                v[f"{p}/attention/linear_0/bias"] = w[o + "cross_attn.query.bias"]
                q8(f"{p}/attention/linear_1/weight", np.concatenate([w[o + "cross_attn.key.weight"], w[o + "cross_attn.value.weight"]]))
                v[f"{p}/attention/linear_1/bias"] = np.concatenate([np.zeros(d, np.float32), w[o + "cross_attn.value.bias"]])
                q8(f"{p}/attention/linear_2/weight", w[o + "cross_attn.out.weight"])
                v[f"{p}/attention/linear_2/bias"] = w[o + "cross_attn.out.bias"]
            v[f"{p}/ffn/layer_norm/gamma"], v[f"{p}/ffn/layer_norm/beta"] = w[o + "mlp_ln.weight"], w[o + "mlp_ln.bias"]
            q8(f"{p}/ffn/linear_0/weight", w[o + "mlp.0.weight"])
            v[f"{p}/ffn/linear_0/bias"] = w[o + "mlp.0.bias"]
            q8(f"{p}/ffn/linear_1/weight", w[o + "mlp.2.weight"])
            v[f"{p}/ffn/linear_1/bias"] = w[o + "mlp.2.bias"]
    return v


@pytest.mark.parametrize("int8", [False, True])
def test_ctranslate2_faster_whisper_dir(tmp_path, weights, int8):
    """faster-whisper (backend/python/faster-whisper/backend.py:26-62) model directories: CTranslate2 model.bin
    (float32 or int8 + per-row scales, fused QKV / KV linears, projection aliased to the embeddings) +
    config.json + tokenizer.json load into the same model as the OpenAI-named weights; parity with
    ctranslate2 itself is unpinned (no ctranslate2 here, synthetic file)."""
    import json as _json
    from localai_tfp_amd.formats.ctranslate2 import read_model_bin, write_model_bin
    d = tmp_path / "faster-whisper-test"
    d.mkdir()
    v = _openai_to_ct2(weights, CFG, int8)
    write_model_bin(str(d / "model.bin"), v, "WhisperSpec", revision=3,
                    aliases={"decoder/projection/weight": "decoder/embeddings/weight"})
    back, meta = read_model_bin(str(d / "model.bin"))
    assert meta["spec"] == "WhisperSpec" and back["decoder/projection/weight"].shape == v["decoder/embeddings/weight"].shape
    (d / "config.json").write_text(_json.dumps({"suppress_ids": [], "suppress_ids_begin": [220, 50257]}))
    tok = WhisperTokenizer.synthetic()
    from localai_tfp_amd.tokenizer.whisper import _bytes_to_unicode
    b2u = _bytes_to_unicode()
    vocab = {"".join(b2u[b] for b in p): i for i, p in enumerate(tok.pieces)}
    (d / "tokenizer.json").write_text(_json.dumps({"model": {"type": "BPE", "vocab": vocab}}), encoding="utf-8")
    m, t2 = W.load_whisper(str(d), "cpu")
    assert (m.cfg.n_audio_head, m.cfg.n_text_layer, m.cfg.n_vocab) == (CFG.n_audio_head, CFG.n_text_layer, CFG.n_vocab)
    a = W.WhisperModel(CFG, weights.get, "cpu")
    mel = torch.from_numpy(np.random.default_rng(2).standard_normal((1, CFG.n_mels, W.N_FRAMES)).astype(np.float32) * 0.5)
    xa, xb = m.encode(mel), a.encode(mel)
    assert (xa - xb).abs().max() < (5e-2 if int8 else 1e-4)
    assert t2.decode(t2.encode("hello world")) == "hello world"
