"""VITS TTS backend: numerics vs a transformers VitsModel oracle built from the same random weights
(stochastic and deterministic duration predictors, multi-speaker conditioning), the rational-quadratic
spline inverse, the tokenizer, HF-directory loading, the worker RPC and the /v1/audio/speech, /tts and
/v1/sound-generation routes (reference coverage: core/http/app_test.go "tts" label, the AIO e2e TTS
case; piper .onnx voices: tests/test_piper.py)."""
import io
import json
import os

import numpy as np
import pytest
import torch
import yaml

from localai_tfp_amd.models import tts as T

transformers = pytest.importorskip("transformers")


def hf_pair(cfg, seed=1):
    from transformers import VitsConfig as HC, VitsModel as HM
    torch.manual_seed(seed)
    hm = HM(HC(**cfg.to_hf())).eval()
    with torch.no_grad():
        for n, p in hm.named_parameters():
            if "translate" in n or "log_scale" in n:
                p.normal_(0, 0.1)  # non-trivial elementwise-affine flow (zero-init in HF)
    hm.noise_scale = 0.0
    hm.noise_scale_duration = 0.0
    sd = T.fold_weight_norm({k: v.detach().clone() for k, v in hm.state_dict().items()})
    return hm, sd


IDS = [0, 5, 0, 12, 0, 7, 0, 3, 0, 19, 0, 22, 0, 1, 0]


@pytest.mark.parametrize("sdp,speakers", [(True, 1), (False, 1), (True, 3)])
def test_vits_matches_transformers(sdp, speakers):
    cfg = T.VitsConfig(**{**T.VITS_TEST.__dict__, "sdp": sdp, "n_speakers": speakers,
                          "spk_dim": 16 if speakers > 1 else 0})
    hm, sd = hf_pair(cfg)
    m = T.VitsModel(cfg, sd, "cpu")
    spk = 2 if speakers > 1 else None
    with torch.no_grad():
        ref = hm(torch.tensor([IDS]), speaker_id=spk).waveform[0].numpy()
    got = m.synthesize(IDS, speaker=spk, noise_scale=0.0, noise_scale_duration=0.0)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, atol=5e-5)


def test_speaking_rate_scales_length():
    hm, sd = hf_pair(T.VITS_TEST)
    m = T.VitsModel(T.VITS_TEST, sd, "cpu")
    a = m.synthesize(IDS, noise_scale=0.0, noise_scale_duration=0.0)
    b = m.synthesize(IDS, noise_scale=0.0, noise_scale_duration=0.0, speaking_rate=0.5)
    assert b.size > a.size
    hm.speaking_rate = 0.5
    with torch.no_grad():
        ref = hm(torch.tensor([IDS])).waveform[0].numpy()
    np.testing.assert_allclose(b, ref, atol=5e-5)


def test_spline_inverse_roundtrip():
    from transformers.models.vits.modeling_vits import _unconstrained_rational_quadratic_spline as fwd
    torch.manual_seed(0)
    x = torch.randn(2, 1, 9) * 3
    uw, uh, ud = torch.randn(2, 1, 9, 10), torch.randn(2, 1, 9, 10), torch.randn(2, 1, 9, 9)
    y, _ = fwd(x, uw, uh, ud, reverse=False, tail_bound=5.0)
    back = T.rq_spline_inverse(y, uw, uh, ud, 5.0)
    assert torch.allclose(back, x, atol=1e-4)


def test_tokenizer_and_hf_dir(tmp_path):
    tok = T.CharTokenizer({"_": 0, "h": 1, "i": 2, " ": 3}, add_blank=True)
    assert tok.encode("Hi !") == [0, 1, 0, 2, 0, 3, 0]
    from safetensors.torch import save_file
    hm, _ = hf_pair(T.VITS_TEST)
    d = tmp_path / "voice"
    d.mkdir()
    hm.config.to_json_file(str(d / "config.json"))
    save_file({k: v.contiguous() for k, v in hm.state_dict().items()}, str(d / "model.safetensors"))
    (d / "vocab.json").write_text(json.dumps({c: i for i, c in enumerate("_ abcdefghijklmnopqrstuvwxyz")}))
    m, t = T.load_vits(str(d), "cpu")
    ids = t.encode("hello")
    with torch.no_grad():
        ref = hm(torch.tensor([ids])).waveform[0].numpy()
    np.testing.assert_allclose(m.synthesize(ids, noise_scale=0.0, noise_scale_duration=0.0), ref, atol=5e-5)


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    from fastapi.testclient import TestClient

    from localai_tfp_amd.config.app_config import ApplicationConfig
    from localai_tfp_amd.gateway.app import create_app
    d = tmp_path_factory.mktemp("tts")
    models = d / "models"
    models.mkdir()
    (models / "voice.yaml").write_text(yaml.safe_dump({
        "name": "voice", "backend": "piper", "parameters": {"model": "synthetic:vits-test"},
        "options": ["noise_scale:0", "noise_w:0"]}))
    (models / "sfx.yaml").write_text(yaml.safe_dump({
        "name": "sfx", "backend": "transformers-tts", "parameters": {"model": "synthetic:vits-test"}}))
    cfg = ApplicationConfig(models_path=str(models), generated_content_dir=str(d / "gen"),
                            upload_dir=str(d / "up"), config_dir=str(d / "cfg"), api_keys=[])
    app = create_app(cfg, inproc=True)
    with TestClient(app) as c:
        yield c
    app.state.localai.shutdown()


def _wav(content: bytes):
    from localai_tfp_amd.utils.audio import _parse_wav
    return _parse_wav(content)


def test_worker_tts(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.tts import TTSServicer
    s = TTSServicer(device="cpu")
    assert s.LoadModel(pb.ModelOptions(Model="synthetic:vits-test", Options=["speaking_rate:1.0"]), None).success
    dst = str(tmp_path / "o.wav")
    r = s.TTS(pb.TTSRequest(text="hello world", dst=dst), None)
    assert r.success, r.message
    x, sr = _wav(open(dst, "rb").read())
    assert sr == 16000 and x.size > 100
    # a speech model does not generate sound effects (MusicGen's job in the reference): explicit refusal
    r = s.SoundGeneration(pb.SoundGenerationRequest(text="rain", dst=dst, duration=0.5), None)
    assert not r.success and "MusicGen" in r.message
    assert not s.TTS(pb.TTSRequest(text="", dst=dst), None).success


def test_http_speech_routes(client):
    for route, body in (("/v1/audio/speech", {"model": "voice", "input": "good morning"}),
                        ("/tts", {"model": "voice", "input": "good morning"}),
                        ("/v1/text-to-speech/0", {"model_id": "voice", "text": "good morning"})):
        r = client.post(route, json=body)
        assert r.status_code == 200, (route, r.text)
        x, sr = _wav(r.content)
        assert sr == 16000 and x.size > 100
    # /v1/sound-generation on a speech model: the backend's explicit refusal surfaces as a server error
    with pytest.raises(RuntimeError, match="MusicGen"):
        client.post("/v1/sound-generation", json={"model_id": "sfx", "text": "thunder", "duration_seconds": 0.25})


@pytest.mark.gpu
def test_vits_gpu_matches_cpu():
    """GPU path (HiFi-GAN on conv.hip, audio.hip wavenet_gate) vs the fp32 CPU model."""
    from localai_tfp_amd.ops import core as K
    x = torch.randn(2, 64, 37)
    g = K.wavenet_gate(x.cuda(), 32).cpu()
    assert torch.allclose(g, torch.tanh(x[:, :32]) * torch.sigmoid(x[:, 32:]), atol=1e-5)
    x = torch.randn(1, 128, 400)
    g = K.wavenet_gate(x.cuda(), 64).cpu()
    assert torch.allclose(g, torch.tanh(x[:, :64]) * torch.sigmoid(x[:, 64:]), atol=1e-5)
    _, sd = hf_pair(T.VITS_TEST)
    c = T.VitsModel(T.VITS_TEST, sd, "cpu").synthesize(IDS, noise_scale=0.0, noise_scale_duration=0.0)
    m = T.VitsModel(T.VITS_TEST, sd, "cuda:0")
    gm = m.synthesize(IDS, noise_scale=0.0, noise_scale_duration=0.0)
    assert m._vplan is not None  # the HiFi-GAN ran on conv.hip (f16 rows, fused leaky / residual / tanh)
    assert gm.shape == c.shape
    assert np.linalg.norm(gm - c) / np.linalg.norm(c) < 2e-2 and np.abs(gm - c).max() < 3e-2


def test_coqui_backend_routes_to_the_vits_worker():
    """The reference's `coqui` backend name is served by the VITS worker (Coqui VITS checkpoints,
    tests/test_coqui.py); XTTS is refused there, never silently replaced by another speech model."""
    from localai_tfp_amd.workers import WORKERS
    assert WORKERS["coqui"].endswith(".tts")
