"""Silero VAD backend: batched STFT/encoder + fused LSTM scan vs a plain per-window PyTorch silero
module (the way the ONNX graph is driven by silero-vad-go), the Detect hysteresis, the worker RPC and
/v1/vad (reference: backend/go/vad/silero/vad.go, core/http/endpoints/localai/vad.go; the AIO e2e
suite's VAD case uses hard-coded samples, tests/e2e-aio/sample_data_test.go — not loadable here, so
synthetic tone/noise clips are used and parity with real silero weights is unpinned)."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F
import yaml

from localai_tfp_amd.models import vad as V


class RefSilero(nn.Module):
    """Per-window silero v5 forward (ReflectionPad -> conv STFT -> 4 conv blocks -> LSTMCell ->
    ReLU/conv1x1/sigmoid), one call per 512-sample window with a carried state + 64-sample context."""

    def __init__(self, sd):
        super().__init__()
        self.sd = sd
        self.cell = nn.LSTMCell(128, 128)
        with torch.no_grad():
            for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                getattr(self.cell, n).copy_(sd[f"decoder.rnn.{n}"])

    def step(self, x, state):
        sd = self.sd
        x = F.pad(x[None, None], (0, 64), mode="reflect")
        spec = F.conv1d(x, sd["stft.forward_basis_buffer"], stride=128)
        mag = torch.sqrt(spec[:, :129] ** 2 + spec[:, 129:] ** 2)
        h = mag
        for i, (_, _, s) in enumerate(V.ENC):
            h = F.relu(F.conv1d(h, sd[f"encoder.{i}.reparam_conv.weight"], sd[f"encoder.{i}.reparam_conv.bias"],
                                stride=s, padding=1))
        hh, cc = self.cell(h[:, :, 0], state)
        p = torch.sigmoid(F.conv1d(F.relu(hh)[:, :, None], sd["decoder.decoder.2.weight"], sd["decoder.decoder.2.bias"]))
        return float(p.reshape(-1)[0]), (hh, cc)

    def run(self, audio):
        state = (torch.zeros(1, 128), torch.zeros(1, 128))
        ctx = torch.zeros(64)
        out = []
        a = torch.as_tensor(audio)
        for i in range(0, len(a) - 512, 512):
            w = a[i:i + 512]
            p, state = self.step(torch.cat([ctx, w]), state)
            ctx = w[-64:]
            out.append(p)
        return np.array(out, np.float32)


def clip(seconds=3.0, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(int(seconds * V.SR)) / V.SR
    x = 0.01 * rng.standard_normal(t.size)
    on = (t > 0.8) & (t < 2.0)
    x[on] += 0.4 * np.sin(2 * np.pi * 180 * t[on]) * (1 + 0.5 * np.sin(2 * np.pi * 3 * t[on]))
    return x.astype(np.float32)


def test_dft_basis_is_hann_stft():
    x = torch.randn(256, dtype=torch.float64)
    st = torch.stft(x, 256, 256, window=torch.hann_window(256, dtype=torch.float64), center=False,
                    return_complex=True)[:, 0]
    b = V.dft_basis().double()[:, 0]
    got = b @ x
    assert torch.allclose(got[:129], st.real, atol=1e-4) and torch.allclose(got[129:], st.imag, atol=1e-4)


def test_batched_model_matches_per_window_reference():
    sd = V.synthetic_state_dict(3)
    m = V.SileroVAD(sd, "cpu")
    audio = clip(2.0, 1)
    ref = RefSilero(sd).run(audio)
    got = m.probs(audio).numpy()
    assert got.shape == ref.shape == ((len(audio) - 1) // 512,)
    np.testing.assert_allclose(got, ref, atol=2e-5)


def test_segments_hysteresis():
    p = V.VADParams()
    probs = np.array([0.1, 0.6, 0.7, 0.4, 0.2, 0.1, 0.9, 0.8], np.float32)
    segs = V.segments(probs, p)
    w = 512 / V.SR
    assert segs == [(pytest.approx(1 * w), pytest.approx(5 * w)), (pytest.approx(6 * w), 0.0)]
    # min-silence keeps a short dip inside the segment
    segs = V.segments(np.array([0.9, 0.1, 0.9, 0.1, 0.1, 0.1], np.float32), V.VADParams(min_silence_ms=40))
    assert len(segs) == 1 and segs[0][0] == 0.0 and segs[0][1] == pytest.approx(4 * w)
    assert V.segments(np.zeros(0, np.float32), p) == []


def test_worker_and_http(tmp_path):
    from fastapi.testclient import TestClient

    from localai_tfp_amd.config.app_config import ApplicationConfig
    from localai_tfp_amd.gateway.app import create_app
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.vad import VADServicer
    s = VADServicer(device="cpu")
    assert s.LoadModel(pb.ModelOptions(Model="synthetic:silero-vad", Options=["threshold:0.0"]), None).success
    r = s.VAD(pb.VADRequest(audio=clip(1.0).tolist()), None)
    assert len(r.segments) == 1 and r.segments[0].start == 0.0  # threshold 0 -> speech from the first window

    models = tmp_path / "models"
    models.mkdir()
    (models / "vad.yaml").write_text(yaml.safe_dump({
        "name": "silero", "backend": "silero-vad", "parameters": {"model": "synthetic:silero-vad"},
        "options": ["threshold:0.0"]}))
    cfg = ApplicationConfig(models_path=str(models), generated_content_dir=str(tmp_path / "gen"),
                            upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"), api_keys=[])
    app = create_app(cfg, inproc=True)
    with TestClient(app) as c:
        r = c.post("/v1/vad", json={"model": "silero", "audio": clip(1.0).tolist()})
        assert r.status_code == 200, r.text
        assert r.json()["segments"][0]["start"] == 0.0
    app.state.localai.shutdown()


@pytest.mark.gpu
def test_lstm_scan_kernel_matches_fp32():
    """audio.hip lstm_scan (fused decoder head, and the plain hidden-sequence mode) vs fp32 PyTorch."""
    from localai_tfp_amd import _native as N
    torch.manual_seed(0)
    for H, T, B in ((128, 700, 1), (64, 300, 3)):
        gx = torch.randn(B, T, 4 * H) * 0.5
        whh = torch.randn(4 * H, H) / H ** 0.5
        hw = torch.randn(H) / H ** 0.5
        d = "cuda:0"
        out = torch.empty(B, T, device=d)
        h = torch.zeros(B, H, device=d)
        c = torch.zeros(B, H, device=d)
        gxd, whd, hwd = gx.to(d), whh.to(d), hw.to(d)
        N.kcall("mxk_lstm_scan", gxd.data_ptr(), whd.data_ptr(), h.data_ptr(), c.data_ptr(), hwd.data_ptr(), 0.1,
                out.data_ptr(), B, T, H, N.stream_ptr())
        for b in range(B):
            ref = V.lstm_scan_ref(gx[b], whh, hw, 0.1)
            assert (out[b].cpu() - ref).abs().max() < 1e-4
        hs = torch.empty(B, T, H, device=d)
        h.zero_()
        c.zero_()
        N.kcall("mxk_lstm_scan", gxd.data_ptr(), whd.data_ptr(), h.data_ptr(), c.data_ptr(), None, 0.0,
                hs.data_ptr(), B, T, H, N.stream_ptr())
        st = (torch.zeros(1, H), torch.zeros(1, H))
        with torch.no_grad():
            for t in range(T):
                g = gx[0, t] + whh @ st[0][0]
                i, f, gg, o = g[:H].sigmoid(), g[H:2 * H].sigmoid(), g[2 * H:3 * H].tanh(), g[3 * H:].sigmoid()
                cn = f * st[1][0] + i * gg
                hn = o * cn.tanh()
                st = (hn[None], cn[None])
                if t in (0, T // 2, T - 1):
                    assert (hs[0, t].cpu() - hn).abs().max() < 1e-4
        assert (h[0].cpu() - st[0][0]).abs().max() < 1e-4


@pytest.mark.gpu
def test_vad_gpu_matches_cpu():
    sd = V.synthetic_state_dict(5)
    audio = clip(4.0, 2)
    pc = V.SileroVAD(sd, "cpu").probs(audio).numpy()
    pg = V.SileroVAD(sd, "cuda:0").probs(audio).cpu().numpy()
    np.testing.assert_allclose(pg, pc, atol=1e-3)


def test_onnx_reader_and_silero_onnx(tmp_path):
    """The protobuf-only ONNX reader (formats/onnx.py) and the silero-vad .onnx loading path: weights
    inside an If branch (v5 layout, 16 kHz branch preferred over an 8 kHz decoy) reproduce the
    safetensors-loaded detector exactly. Parity against onnxruntime itself is unpinned."""
    from localai_tfp_amd.formats import onnx as O
    from localai_tfp_amd.models import vad as V
    sd = V.synthetic_state_dict(seed=3)
    top = {"_model.stft.forward_basis_buffer": sd["stft.forward_basis_buffer"].numpy()}
    sub = {"_model." + k: v.numpy() for k, v in sd.items() if k != "stft.forward_basis_buffer"}
    decoy = {"_model_8k." + k: np.zeros_like(v.numpy()) for k, v in sd.items() if k.startswith("decoder")}
    blob = O.make_model(top, {**sub, **decoy})
    p = tmp_path / "silero_vad.onnx"
    p.write_bytes(blob)
    tensors, nodes = O.initializers(str(p))
    assert any(n.op_type == "If" for _, n in nodes)
    assert "If_0/then_branch/_model.encoder.0.reparam_conv.weight" in tensors
    got = V.load_state_dict(str(p))
    for k, v in sd.items():
        assert torch.equal(got[k], v.float()), k
    bad = tmp_path / "other.onnx"
    bad.write_bytes(O.make_model({"onnx::Conv_12": np.zeros((3, 3), np.float32)}))
    with pytest.raises(ValueError, match="not found in the ONNX"):
        V.load_state_dict(str(bad))
