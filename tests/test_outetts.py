"""OuteTTS (transformers backend type OuteTTS, backend/python/transformers/backend.py:205-243, 509-531):
prompt format of the outetts v0.2 / v0.3 interfaces, code extraction, the WavTokenizer decoder (checkpoint
names, Vocos "same" iSTFT against a direct overlap-add) and the TTS RPC path. No OuteTTS / WavTokenizer
weights or the outetts package exist here: audio parity is unpinned."""
import json

import numpy as np
import pytest
import torch

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


def test_outetts_audio_path_refused():
    with pytest.raises(NotImplementedError, match="AudioPath"):
        O.load_outetts("synthetic:outetts-test", "cpu", {}, audio_path="/x.wav")
