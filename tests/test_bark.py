"""Bark (models/bark.py) vs transformers BarkModel (random-init tiny config, greedy), the worker, GPU path."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.models import bark as BK

pytest.importorskip("transformers")


def _tiny_hf(seed=0):
    from transformers import BarkConfig, BarkModel, EncodecConfig
    from transformers.models.bark.configuration_bark import BarkCoarseConfig, BarkFineConfig, BarkSemanticConfig
    torch.manual_seed(seed)
    g = dict(num_layers=2, num_heads=2, hidden_size=16, block_size=1024)
    sem = BarkSemanticConfig(**g, input_vocab_size=129_600, output_vocab_size=10_048, bias=False)
    coa = BarkCoarseConfig(**g, input_vocab_size=12_096, output_vocab_size=12_096, bias=False)
    fin = BarkFineConfig(**g, input_vocab_size=1056, output_vocab_size=1056, n_codes_total=8, n_codes_given=1)
    codec = EncodecConfig(num_filters=4, upsampling_ratios=[8, 5, 4, 2], hidden_size=16, codebook_size=1024)
    cfg = BarkConfig(semantic_config=sem.to_dict(), coarse_acoustics_config=coa.to_dict(),
                     fine_acoustics_config=fin.to_dict(), codec_config=codec.to_dict())
    m = BarkModel(cfg).eval()
    from transformers.models.bark.generation_configuration_bark import BarkGenerationConfig
    gc = BarkGenerationConfig()
    for k in ("semantic_config", "coarse_acoustics_config", "fine_acoustics_config"):
        v = getattr(gc, k)
        if not isinstance(v, dict):
            setattr(gc, k, v.to_dict())
    m.generation_config = gc
    with torch.no_grad():  # spread the tiny model's logits so greedy picks are well separated
        for n, p in m.named_parameters():
            if "embeds" in n or "lm_head" in n:
                p.mul_(25.0)
    return cfg, m


@pytest.mark.parametrize("n_sem", [12, 40])
def test_bark_greedy_matches_transformers(n_sem):
    cfg, m = _tiny_hf()
    text = torch.tensor([[101, 2054, 2003, 1037, 4937, 102]])
    L = 256
    ids = torch.full((1, L), 0, dtype=torch.long)
    ids[0, :text.shape[1]] = text
    mask = torch.zeros_like(ids)
    mask[0, :text.shape[1]] = 1
    with torch.no_grad():
        ref = m.generate(input_ids=ids, attention_mask=mask, do_sample=False, semantic_max_new_tokens=n_sem)
    mine = BK.Bark(cfg.to_dict(), m.state_dict(), "cpu")
    sem = mine.semantic_tokens(text[0].tolist(), None, None, None, None, n_sem)
    co = mine.coarse_tokens(sem, None, None, None)
    fi = mine.fine_tokens(co, None, None, None)
    audio = mine.codec.decode(torch.from_numpy(fi)[None])[0, 0]
    assert audio.shape[-1] == ref.shape[-1], (audio.shape, ref.shape)
    torch.testing.assert_close(audio, ref[0], rtol=1e-3, atol=1e-4)


def test_bark_voice_preset_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    p = tmp_path / "v.npz"
    np.savez(p, semantic_prompt=rng.integers(0, 10000, 300), coarse_prompt=rng.integers(0, 1024, (2, 450)),
             fine_prompt=rng.integers(0, 1024, (8, 450)))
    v = BK.load_voice(str(p))
    m = BK.synthetic_bark("bark-test", "cpu")
    wav = m.generate(m.tokenize("hello"), history=v, seed=1, max_semantic=10)
    assert wav.dtype == np.float32 and wav.size > 0 and np.isfinite(wav).all()


def test_bark_worker_tts(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers import WORKERS, resolve
    from localai_tfp_amd.workers.bark import BarkServicer
    assert WORKERS[resolve("bark")] == WORKERS[resolve("bark-cpp")] == "localai_tfp_amd.workers.bark"
    s = BarkServicer("cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:bark-test", Options=["max_semantic_tokens:8"]), None)
    assert r.success, r.message
    dst = str(tmp_path / "o.wav")
    r = s.TTS(pb.TTSRequest(text="hi there", dst=dst), None)
    assert r.success, r.message
    import wave
    with wave.open(dst) as w:
        assert w.getframerate() == 24000 and w.getnframes() > 0


@pytest.mark.gpu
def test_bark_gpu_matches_cpu_codes():
    cfg, m = _tiny_hf(seed=2)
    cpu = BK.Bark(cfg.to_dict(), m.state_dict(), "cpu")
    gpu = BK.Bark(cfg.to_dict(), m.state_dict(), "cuda")
    text = [101, 7592, 2088, 102]
    s_c = cpu.semantic_tokens(text, None, None, None, None, 16)
    s_g = gpu.semantic_tokens(text, None, None, None, None, 16)
    assert np.mean(np.array(s_c) == np.array(s_g[:len(s_c)])) > 0.8
    co = cpu.coarse_tokens(s_c, None, None, None)
    co_g = gpu.coarse_tokens(s_c, None, None, None)  # HIP-graph decode loop (Bark._ar_graph)
    assert co_g.shape == co.shape and np.mean(co_g == co) > 0.8
    fi = cpu.fine_tokens(co, None, None, None)
    a_c = cpu.codec.decode(torch.from_numpy(fi)[None])
    a_g = gpu.codec.decode(torch.from_numpy(fi)[None].cuda()).cpu()
    assert float((a_g - a_c).norm() / a_c.norm()) < 3e-2
