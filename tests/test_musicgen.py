"""MusicGen (models/musicgen.py) + EnCodec decoder (models/encodec.py) vs the transformers implementations
(random-init tiny configs: no checkpoint download), the SoundGeneration worker, and the GPU path
(implicit-GEMM conv kernels for every Conv1d / ConvTranspose1d, hipGraph-captured decode step)."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.models import encodec as E
from localai_tfp_amd.models import musicgen as MG

tf = pytest.importorskip("transformers")


def _tiny_hf(seed=0, causal=True):
    from transformers import EncodecConfig, MusicgenConfig, MusicgenForConditionalGeneration, T5Config
    from transformers.models.musicgen.configuration_musicgen import MusicgenDecoderConfig
    torch.manual_seed(seed)
    t5 = T5Config(vocab_size=100, d_model=32, d_kv=8, d_ff=64, num_layers=2, num_heads=4, feed_forward_proj="relu")
    enc = EncodecConfig(num_filters=4, upsampling_ratios=[2, 2], hidden_size=16, codebook_size=64,
                        num_lstm_layers=2, sampling_rate=1000, use_causal_conv=causal)
    dec = MusicgenDecoderConfig(vocab_size=64, hidden_size=48, num_hidden_layers=2, num_attention_heads=4,
                                ffn_dim=64, num_codebooks=4, pad_token_id=64, bos_token_id=64,
                                decoder_start_token_id=64)
    cfg = MusicgenConfig(text_encoder=t5.to_dict(), audio_encoder=enc.to_dict(), decoder=dec.to_dict())
    m = MusicgenForConditionalGeneration(cfg).eval()
    gc = m.generation_config
    gc.pad_token_id = gc.decoder_start_token_id = gc.bos_token_id = 64
    return cfg, m


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("res_layers", [1, 2])
def test_encodec_decoder_matches_transformers(causal, res_layers):
    from transformers import EncodecConfig, EncodecModel
    torch.manual_seed(res_layers)
    cfg = EncodecConfig(num_filters=4, upsampling_ratios=[4, 2], hidden_size=16, codebook_size=64,
                        num_lstm_layers=2, sampling_rate=8000, use_causal_conv=causal,
                        num_residual_layers=res_layers)
    m = EncodecModel(cfg).eval()
    codes = torch.randint(0, 64, (2, 4, 13))
    with torch.no_grad():
        ref = m.decode(codes[None], [None]).audio_values
    got = E.from_state_dict(cfg.to_dict(), m.state_dict()).decode(codes)
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("guidance", [1.0, 3.0])
def test_musicgen_greedy_matches_transformers(guidance):
    cfg, m = _tiny_hf()
    ids = torch.tensor([[5, 17, 42, 9, 1]])
    with torch.no_grad():
        ref = m.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False,
                         guidance_scale=guidance, max_new_tokens=12)
    mine = MG.MusicGen(cfg.to_dict(), m.state_dict(), "cpu")
    codes = mine.generate_codes(ids, None, 12, guidance, do_sample=False)
    assert codes.shape == (1, 4, 12 + 1 - 4)
    audio = mine.decode_audio(codes)
    assert audio.shape == ref.shape
    torch.testing.assert_close(audio, ref, rtol=1e-4, atol=1e-5)


def test_musicgen_cfg_changes_output_and_delay_pattern():
    mine = MG.synthetic_musicgen("musicgen-test", "cpu", seed=3)  # unit-scale weights: CFG moves argmax
    ids = torch.tensor([[7, 3, 99, 1]])
    a = mine.generate_codes(ids, None, 16, 1.0, do_sample=False)
    b = mine.generate_codes(ids, None, 16, 8.0, do_sample=False)
    assert not torch.equal(a, b)  # guidance reaches the logits
    pat = MG.delay_pattern(mine.dc, 10)
    for k in range(4):  # codebook k: pads at positions <= k and >= 10 - 4 + 1 + k
        assert (pat[k, :k + 1] == mine.dc.pad_id).all() and (pat[k, k + 1:10 - 4 + 1 + k] == -1).all()
        assert (pat[k, 10 - 4 + 1 + k:] == mine.dc.pad_id).all()


def test_musicgen_unconditional_and_sampling_seeded():
    m = MG.synthetic_musicgen("musicgen-test", "cpu")
    c1 = m.generate_codes(None, None, 10, 1.0, do_sample=True, seed=5)
    c2 = m.generate_codes(None, None, 10, 1.0, do_sample=True, seed=5)
    assert torch.equal(c1, c2) and c1.shape == (1, 4, 7)


def test_musicgen_worker_sound_generation(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.musicgen import MusicgenServicer
    s = MusicgenServicer("cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:musicgen-test"), None)
    assert r.success, r.message
    dst = str(tmp_path / "out.wav")
    req = pb.SoundGenerationRequest(text="lofi beat", dst=dst, duration=0.5, sample=False)
    r = s.SoundGeneration(req, None)
    assert r.success, r.message
    import wave
    with wave.open(dst) as w:
        assert w.getframerate() == 4000 and w.getnframes() > 0
    r = s.SoundGeneration(pb.SoundGenerationRequest(text="", dst=dst, duration=0.5), None)  # unconditional
    assert r.success, r.message


def test_musicgen_backend_routes_to_worker():
    from localai_tfp_amd.workers import WORKERS, resolve
    assert WORKERS[resolve("transformers-musicgen")] == "localai_tfp_amd.workers.musicgen"


@pytest.mark.gpu
def test_musicgen_gpu_graph_matches_cpu():
    cfg, m = _tiny_hf(seed=1, causal=False)
    ids = torch.tensor([[5, 17, 42, 9, 1]])
    cpu = MG.MusicGen(cfg.to_dict(), m.state_dict(), "cpu")
    gpu = MG.MusicGen(cfg.to_dict(), m.state_dict(), "cuda")
    ref = cpu.generate_codes(ids, None, 16, 3.0, do_sample=False)
    eager = gpu.generate_codes(ids, None, 16, 3.0, do_sample=False, use_graph=False)
    graph = gpu.generate_codes(ids, None, 16, 3.0, do_sample=False, use_graph=True)
    assert torch.equal(eager.cpu(), graph.cpu())  # replaying the captured step == eager
    assert (eager.cpu() == ref).float().mean().item() > 0.8  # f16 vs fp32 greedy: near-identical tokens
    a_gpu = gpu.decode_audio(ref.cuda()).cpu()
    a_cpu = cpu.decode_audio(ref)
    err = (a_gpu - a_cpu).norm() / a_cpu.norm()
    assert err < 2e-2, float(err)


@pytest.mark.gpu
def test_musicgen_small_synthetic_gpu_runs():
    m = MG.synthetic_musicgen("musicgen-small", "cuda")
    codes = m.generate_codes(m.tokenize("80s synthwave"), None, 16, 3.0, do_sample=True, seed=0)
    wav = m.decode_audio(codes)
    assert codes.shape == (1, 4, 13) and torch.isfinite(wav).all()
    assert wav.shape[-1] == 13 * 640


def test_transformers_backend_serves_musicgen_type(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    s = LLMServicer("cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:musicgen-test", Type="MusicgenForConditionalGeneration"), None)
    assert r.success, r.message
    dst = str(tmp_path / "a.wav")
    r = s.SoundGeneration(pb.SoundGenerationRequest(text="drums", dst=dst, duration=0.4, sample=True), None)
    assert r.success, r.message
