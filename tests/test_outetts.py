"""OuteTTS (transformers backend type OuteTTS, backend/python/transformers/backend.py:205-243, 509-531):
prompt format of the outetts v0.2 / v0.3 interfaces, code extraction, the WavTokenizer decoder (checkpoint
names, Vocos "same" iSTFT against a direct overlap-add) and the TTS RPC path. No OuteTTS / WavTokenizer
weights or the outetts package exist here: audio parity is unpinned."""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.models import outetts as O
from localai_tfp_amd.models import wavtokenizer as WT

SPK = {"text": "Hello, there.", "words": [{"word": "hello", "duration": 0.4, "codes": [5, 17, 9]},
                                          {"word": "there", "duration": 0.3333, "codes": [1, 2]}]}


def test_prompt_v03_and_v02():
    sp = O.Speaker(SPK["text"], SPK["words"])
    p = O.PromptV2("0.3").completion("It's 5 o'clock!", sp)
    assert p == ("<|im_start|>\n<|text_start|>hello<|text_sep|>there<|text_sep|>it's<|text_sep|>5<|text_sep|>"
                 "o'clock<|text_end|>\n<|audio_start|>\nhello<|t_0.40|><|code_start|><|c_5|><|c_17|><|c_9|>"
                 "<|code_end|>\nthere<|t_0.33|><|code_start|><|c_1|><|c_2|><|code_end|>\n")
    p2 = O.PromptV2("0.2").completion("hi", sp)
    assert p2.endswith("hello<|t_0.40|><|5|><|17|><|9|>\nthere<|t_0.33|><|1|><|2|>\n")
    assert O.PromptV2("0.2").completion("hi") == "<|im_start|>\n<|text_start|>hi<|text_end|>\n<|audio_start|>\n"
    gen = "world<|t_0.50|><|code_start|><|c_100|><|c_4095|><|code_end|>\n<|audio_end|>"
    assert O.PromptV2("0.3").codes(gen) == [100, 4095]
    assert O.PromptV2("0.2").codes("x<|t_0.10|><|7|><|8|>") == [7, 8]


def test_istft_same_matches_overlap_add():
    n_fft, hop, T = 64, 16, 12
    g = torch.Generator().manual_seed(0)
    spec = torch.polar(torch.rand(1, n_fft // 2 + 1, T, generator=g) + 0.1, torch.randn(1, n_fft // 2 + 1, T, generator=g))
    got = WT.istft_same(spec, n_fft, hop)[0].numpy()
    win = np.hanning(n_fft + 1)[:-1]  # periodic Hann
    frames = np.fft.irfft(spec[0].numpy(), n_fft, axis=0) * win[:, None]
    size = (T - 1) * hop + n_fft
    y, env = np.zeros(size), np.zeros(size)
    for t in range(T):
        y[t * hop:t * hop + n_fft] += frames[:, t]
        env[t * hop:t * hop + n_fft] += win ** 2
    pad = (n_fft - hop) // 2
    ref = y[pad:size - pad] / env[pad:size - pad]
    assert got.shape == (T * hop,)
    assert np.allclose(got, ref, atol=1e-5)


def _codec(seed=3):
    from localai_tfp_amd.models.diffusion.nn import init_synthetic
    m = WT.WavTokenizerDecoder(WT.WAVTOKENIZER_TEST)
    init_synthetic(m, seed, std=0.05)
    with torch.no_grad():
        m.codebook.normal_(generator=torch.Generator().manual_seed(seed))
    return m.eval()


def test_wavtokenizer_checkpoint_names(tmp_path):
    m = _codec()
    sd = {("feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed" if k == "codebook" else k):
          (v[None] if k == "codebook" else v) for k, v in m.state_dict().items()}
    sd["feature_extractor.encodec.encoder.model.0.conv.conv.weight"] = torch.zeros(4, 1, 7)  # encoder: ignored
    p = tmp_path / "wavtokenizer.ckpt"
    torch.save({"state_dict": sd, "epoch": 3}, str(p))
    m2 = WT.load_wavtokenizer(str(p))
    assert m2.cfg.layers == 2 and m2.cfg.n_fft == 64 and m2.cfg.hop == 16 and m2.cfg.codebook == 64
    codes = torch.tensor([3, 9, 60, 1, 1, 7, 22, 5])
    a, b = m.decode(codes), m2.decode(codes)
    assert a.shape == (8 * 16,) and torch.equal(a, b) and torch.isfinite(a).all()


def test_outetts_tts_through_llm_worker(tmp_path, monkeypatch):
    (tmp_path / "spk.json").write_text(json.dumps(SPK))
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    seen = {}

    def fake(self, prompt, max_tokens, seed=0):
        seen["prompt"] = prompt
        return "from<|t_0.20|><|code_start|><|c_3|><|c_9|><|c_60|><|code_end|>\nme<|t_0.10|><|code_start|><|c_1|><|code_end|>"
    monkeypatch.setattr(O.OuteTTS, "generate_text", fake)
    s = LLMServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:outetts-test", Type="OuteTTS", ModelPath=str(tmp_path),
                                    Options=["speaker:spk.json", "version:0.3"]), None)
    assert r.success, r.message
    dst = str(tmp_path / "o.wav")
    r = s.TTS(pb.TTSRequest(text="From me.", dst=dst), None)
    assert r.success, r.message
    assert seen["prompt"].startswith("<|im_start|>\n<|text_start|>hello<|text_sep|>there<|text_sep|>from<|text_sep|>me")
    import wave
    with wave.open(dst) as w:
        assert w.getframerate() == 24000 and w.getnframes() == 4 * 16


def test_outetts_generate_text_on_engine():
    """The LM side runs on the engine: a synthetic model produces some continuation of the prompt ids."""
    t = O.load_outetts("synthetic:outetts-test", "cpu", {})
    out = t.generate_text("<|im_start|>\nhello", 6)
    assert isinstance(out, str) and len(out) > 0


def _encoder(seed=0):
    sd = WT.synthetic_encoder_state(WT.WAVTOKENIZER_TEST, ratios=(2, 2, 2, 2), seed=seed)
    return WT.WavTokenizerEncoder({"state_dict": sd}, torch.zeros(64, 32))


def test_wavtokenizer_encoder_frames_and_codes():
    """SEANet encoder: one feature frame per hop (16 = 2*2*2*2 samples), codes = nearest codebook entry. With the
    codebook built from the clip's own (permuted) features the codes recover the permutation exactly."""
    enc = _encoder()
    assert [k for k, _, _ in enc.layers].count("res") == 4 and any(k == "lstm" for k, _, _ in enc.layers)
    assert [s for k, _, s in enc.layers if k == "conv"] == [1, 2, 2, 2, 2, 1]
    audio = torch.randn(16 * 20, generator=torch.Generator().manual_seed(1)) * 0.3
    f = enc.features(audio)
    assert f.shape == (20, 32) and torch.isfinite(f).all()
    assert enc.features(audio[:16 * 20 - 5]).shape == (20, 32)  # partial last frame padded, not dropped
    perm = torch.randperm(20, generator=torch.Generator().manual_seed(2))
    enc.codebook = torch.cat([f[perm], f[:1] + 100.0])  # + one far-away decoy
    assert enc.encode(audio) == torch.argsort(perm).tolist()


def test_wavtokenizer_encoder_residual_math():
    """One residual block against the plain formula: shortcut(x) + conv1(elu(conv3(elu(x)))), reflect padding."""
    enc = _encoder()
    x = torch.randn(1, 8, 12, generator=torch.Generator().manual_seed(4))
    w = enc.w
    p = "1."
    h = F.conv1d(F.pad(F.elu(x), (1, 1), mode="reflect"), w[p + "block.1.conv.conv.weight"], w[p + "block.1.conv.conv.bias"])
    h = F.conv1d(F.elu(h), w[p + "block.3.conv.conv.weight"], w[p + "block.3.conv.conv.bias"])
    ref = F.conv1d(x, w[p + "shortcut.conv.conv.weight"], w[p + "shortcut.conv.conv.bias"]) + h
    assert torch.allclose(enc._res(x, p), ref, atol=1e-5)


def test_create_speaker_word_split():
    class Enc:
        def encode(self, a):
            return list(range(100, 100 + len(a) // 16))
    audio = np.zeros(16 * 30, np.float32)  # 30 frames at 1500 fps
    sp = O.create_speaker(Enc(), audio, 24000, 1500.0, "Hi, everybody here!")
    assert [w["word"] for w in sp.words] == ["hi", "everybody", "here"]
    codes = [c for w in sp.words for c in w["codes"]]
    assert codes == list(range(100, 130))  # every code, in order, once
    lens = [len(w["codes"]) for w in sp.words]
    assert lens[1] > lens[2] > lens[0]  # proportional to word length
    assert sp.words[1]["duration"] == round(lens[1] / 1500.0, 2)
    # segments (Whisper timestamps): each word stays inside its segment
    sp = O.create_speaker(Enc(), audio, 24000, 1500.0, segments=[(0.0, 0.01, "one two"), (0.01, 0.02, "three")])
    assert [w["word"] for w in sp.words] == ["one", "two", "three"]
    assert sp.words[2]["codes"] == list(range(115, 130)) and sp.text == "one two three"
    with pytest.raises(ValueError, match="no words"):
        O.create_speaker(Enc(), audio, 24000, 1500.0, "")


def test_outetts_speaker_from_audio_path(tmp_path):
    """LoadModel AudioPath: the clip is encoded by the codec's encoder and becomes the prompt's speaker."""
    from localai_tfp_amd.utils.audio import write_wav
    sr = 24000
    t = np.arange(sr // 10) / sr
    write_wav(str(tmp_path / "ref.wav"), (0.3 * np.sin(2 * np.pi * 220 * t)).astype(np.float32), sr)
    with pytest.raises(ValueError, match="transcript"):
        O.load_outetts("synthetic:outetts-test", "cpu", {}, model_path=str(tmp_path), audio_path="ref.wav")
    tts = O.load_outetts("synthetic:outetts-test", "cpu", {"speaker_text": "Hello there."},
                         model_path=str(tmp_path), audio_path="ref.wav")
    sp = tts.speaker
    assert sp.text == "Hello there." and [w["word"] for w in sp.words] == ["hello", "there"]
    codes = [c for w in sp.words for c in w["codes"]]
    assert len(codes) == sr // 10 // 16 and all(0 <= c < 64 for c in codes)
    p = O.PromptV2("0.3").completion("Go.", sp)
    assert "hello<|t_" in p and f"<|c_{codes[0]}|>" in p
