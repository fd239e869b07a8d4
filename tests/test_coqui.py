"""Coqui TTS VITS checkpoints (the reference's `coqui` backend: backend/python/coqui/backend.py:26-80; its
test loads "tts_models/en/vctk/vits", test.py:55). A synthetic model directory in Coqui's layout —
config.json (model / model_args / audio / characters) + model_file.pth holding {"model": state dict} in
Coqui's module names with weight-norm pairs on the decoder and coupling convs — loads into exactly the
weights it was written from, tokenises with Coqui's vocabulary order + blank interspersing, resolves the
Coqui model name through the local cache layout, maps speaker names, and synthesises through the TTS worker.
No Coqui TTS package or real checkpoint exists here: parity with Coqui's audio is unpinned."""
import json
import re

import numpy as np
import pytest
import torch

from localai_tfp_amd.models import tts as T
from localai_tfp_amd.models.coqui import CoquiTokenizer, load_coqui

_INV_ATT = {"q_proj": "q", "k_proj": "k", "v_proj": "v", "out_proj": "o"}


def hf_to_coqui(sd: dict) -> dict:
    """HF VitsModel names -> Coqui VITS names (written independently of the loader)."""
    out = {}
    for k, v in sd.items():
        a = v.float().clone()
        m = re.match(r"text_encoder\.encoder\.layers\.(\d+)\.(.+)$", k)
        if m:
            i, rest = m[1], m[2]
            if rest.startswith("attention."):
                _, nm, *lf = rest.split(".")
                if nm.startswith("emb_rel"):
                    out[f"text_encoder.encoder.attn_layers.{i}.{nm}"] = a
                else:
                    out[f"text_encoder.encoder.attn_layers.{i}.conv_{_INV_ATT[nm]}.{lf[0]}"] = a[..., None] if lf[0] == "weight" else a
            elif rest.startswith(("layer_norm.", "final_layer_norm.")):
                n = "1" if rest.startswith("layer_norm.") else "2"
                out[f"text_encoder.encoder.norm_layers_{n}.{i}.{'gamma' if rest.endswith('weight') else 'beta'}"] = a
            elif rest.startswith("feed_forward."):
                out[f"text_encoder.encoder.ffn_layers.{i}.{rest[len('feed_forward.'):]}"] = a
            continue
        if k == "text_encoder.embed_tokens.weight":
            out["text_encoder.emb.weight"] = a
        elif k.startswith("text_encoder.project."):
            out["text_encoder.proj." + k.rsplit(".", 1)[1]] = a
        elif k.startswith("duration_predictor."):
            r = k[len("duration_predictor."):]
            r = re.sub(r"^(post_)?flows\.0\.translate$", lambda m: f"{m[1] or ''}flows.0.translation", r)
            r = r.replace("post_conv_pre", "post_pre").replace("post_conv_proj", "post_proj")
            r = r.replace("post_conv_dds.", "post_convs.").replace("conv_dds.", "convs.")
            r = r.replace("conv_pre", "pre").replace("conv_proj", "proj")
            r = r.replace("convs_dilated", "convs_sep").replace("convs_pointwise", "convs_1x1")
            if re.search(r"norms_[12]\.\d+\.(weight|bias)$", r):
                r = r[:-6] + "gamma" if r.endswith("weight") else r[:-4] + "beta"
            out["duration_predictor." + r] = a
        elif k.startswith("flow.flows."):
            m = re.match(r"flow\.flows\.(\d+)\.(.+)$", k)
            r = m[2].replace("conv_pre", "pre").replace("conv_post", "post").replace("wavenet.", "enc.")
            out[f"flow.flows.{m[1]}.{r}"] = a
        elif k.startswith("decoder."):
            r = k[len("decoder."):].replace("upsampler.", "ups.")
            r = re.sub(r"^cond\.", "cond_layer.", r)
            out["waveform_decoder." + r] = a
        elif k == "embed_speaker.weight":
            out["emb_g.weight"] = a
    # weight norm as torch.nn.utils.weight_norm leaves it (g = ||v|| over all but dim 0): decoder + coupling convs
    for k in [k for k in out if k.endswith(".weight") and re.search(r"(waveform_decoder\.(ups|resblocks)|\.enc\.in_layers)", k)]:
        w = out.pop(k)
        g = w.flatten(1).norm(dim=1).view(-1, *([1] * (w.dim() - 1)))
        out[k[:-len("weight")] + "weight_g"] = g
        out[k[:-len("weight")] + "weight_v"] = w * 2.0  # any scale: folding divides it out
    out["posterior_encoder.pre.weight"] = torch.zeros(4, 4, 1)  # training-only, dropped
    return out


CHARS = "abcdefghijklmnopqrstuvwxyzæçðøħŋœǀǁǂǃɐɑɒɓɔɕɖɗɘəɚɛɜɞɟɠɡɢɣɤɥɦɧɨɪɫɬɭɮɯɰɱɲɳɴɵɶɸɹɺɻɽɾʀʁʂʃʄʈʉʊʋʌʍʎʏʐʑʒʔʕʘʙʛʜʝʟʡʢˈˌːˑ̃"


def coqui_config(cfg: T.VitsConfig, use_phonemes=True):
    return {"model": "vits", "run_name": "vits_vctk", "use_phonemes": use_phonemes, "phoneme_language": "en-us",
            "phonemizer": "espeak", "add_blank": True, "text_cleaner": "english_cleaners",
            "audio": {"sample_rate": 22050},
            "characters": {"characters_class": "TTS.tts.models.vits.VitsCharacters", "pad": "_", "eos": "", "bos": "",
                           "blank": " " if False else "<BLNK>", "characters": CHARS,
                           "punctuations": ";:,.!?¡¿—…\"«»“” ", "phonemes": None, "is_unique": False, "is_sorted": True},
            "model_args": {"num_chars": cfg.vocab, "hidden_channels": cfg.hidden, "use_sdp": cfg.sdp,
                           "upsample_rates_decoder": list(cfg.upsample_rates),
                           "upsample_kernel_sizes_decoder": list(cfg.upsample_kernels),
                           "resblock_kernel_sizes_decoder": list(cfg.resblock_kernels),
                           "resblock_dilation_sizes_decoder": [list(d) for d in cfg.resblock_dilations],
                           "resblock_type_decoder": "1", "num_heads_text_encoder": cfg.n_heads,
                           "inference_noise_scale": 0.0, "inference_noise_scale_dp": 0.0, "length_scale": 1.25,
                           "speakers_file": "/some/training/path/speakers.json",
                           "use_speaker_embedding": cfg.n_speakers > 1}}


def make_model(tmp_path, name="tts_models--en--vctk--vits", n_speakers=3):
    base = T.VITS_TEST.__dict__
    tokv = len(CoquiTokenizer(coqui_config(T.VITS_TEST)).vocab)
    cfg = T.VitsConfig(**{**base, "vocab": tokv, "n_speakers": n_speakers, "spk_dim": 16 if n_speakers > 1 else 0})
    sd = T.synthetic_vits(cfg, seed=3)
    d = tmp_path / name
    d.mkdir(parents=True)
    torch.save({"model": hf_to_coqui(sd), "step": 1000}, d / "model_file.pth")
    (d / "config.json").write_text(json.dumps(coqui_config(cfg)), encoding="utf-8")
    (d / "speakers.json").write_text(json.dumps({"p225": 0, "p226": 1, "p227": 2}), encoding="utf-8")
    return d, sd, cfg


def test_coqui_weights_and_config(tmp_path):
    d, sd, cfg = make_model(tmp_path)
    m, tok, spk = load_coqui(str(d))
    sd = {k: v for k, v in sd.items() if not k.startswith("posterior_encoder.")}
    assert set(m.w) == set(sd)
    for k, v in sd.items():
        torch.testing.assert_close(m.w[k], v.float(), rtol=1e-6, atol=1e-6, msg=k)
    c = m.cfg
    for f in ("vocab", "hidden", "n_layers", "n_heads", "ffn", "ffn_kernel", "window", "flow_size", "sdp", "dp_filter",
              "dp_kernel", "dds_layers", "flow_bins", "dp_flows", "prior_flows", "prior_wn_layers", "wn_kernel",
              "upsample_initial", "upsample_rates", "upsample_kernels", "resblock_kernels", "resblock_dilations",
              "n_speakers", "spk_dim"):
        assert getattr(c, f) == getattr(cfg, f), f
    assert c.sample_rate == 22050 and c.speaking_rate == pytest.approx(0.8) and c.noise_scale == 0.0
    assert spk == {"p225": 0, "p226": 1, "p227": 2}


def test_coqui_tokenizer_vocab_order_and_blanks():
    tok = CoquiTokenizer(coqui_config(T.VITS_TEST, use_phonemes=False))
    punc = ";:,.!?¡¿—…\"«»“” "
    # VitsCharacters: pad, punctuations, characters, blank
    assert tok.vocab[0] == "_" and tok.vocab[1:1 + len(punc)] == list(punc) and tok.vocab[-1] == "<BLNK>"
    assert tok.vocab[1 + len(punc):-1] == sorted(CHARS)
    blank = len(tok.vocab) - 1
    ids = tok.encode("Hi, yo")
    core = [tok.ids[c] for c in "hi, yo"]
    assert ids == [blank, core[0], blank, core[1], blank, core[2], blank, core[3], blank, core[4], blank, core[5], blank]
    # the other character classes: pad, eos, bos, blank, characters, punctuations
    c2 = coqui_config(T.VITS_TEST, use_phonemes=False)
    c2["characters"].update(characters_class="TTS.tts.utils.text.characters.Graphemes", eos="&", bos="*", characters="cba")
    t2 = CoquiTokenizer(c2)
    assert t2.vocab[:7] == ["_", "&", "*", "<BLNK>", "a", "b", "c"] and t2.vocab[7:] == list(punc)
    # phonemes: built-in English rules when no espeak-ng is installed
    tp = CoquiTokenizer(coqui_config(T.VITS_TEST))
    tp._espeak = None
    assert len(tp.encode("hello world")) > 5


def test_coqui_synthesises_through_worker(tmp_path, monkeypatch):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.tts import TTSServicer
    d, sd, cfg = make_model(tmp_path)
    monkeypatch.setenv("MX_BACKEND_NAME", "coqui")
    s = TTSServicer(device="cpu")
    # the reference's model name, resolved through Coqui's cache layout under the models directory
    r = s.LoadModel(pb.ModelOptions(Model="tts_models/en/vctk/vits", ModelPath=str(tmp_path)), None)
    assert r.success, r.message
    s.tok._espeak = None
    dst = str(tmp_path / "o.wav")
    r = s.TTS(pb.TTSRequest(text="Hello from the GPU.", model="tts_models/en/vctk/vits", dst=dst, voice="p226"), None)
    assert r.success, r.message
    import wave
    with wave.open(dst) as w:
        assert w.getframerate() == 22050 and w.getnframes() > 0
    ids = s.tok.encode("Hello from the GPU.")
    ref = T.VitsModel(s.model.cfg, sd, "cpu").synthesize(ids, speaker=1, seed=0)
    got = s.model.synthesize(ids, speaker=1, seed=0)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    r = s.TTS(pb.TTSRequest(text="Hello.", dst=dst, voice="nobody"), None)
    assert not r.success and "unknown speaker" in r.message


def test_coqui_missing_and_xtts_incomplete(tmp_path, monkeypatch):
    """A missing model reports 'not found locally'; an XTTS directory whose checkpoint lacks the XTTS modules is
    refused with the missing names (full XTTS: tests/test_xtts.py)."""
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.tts import TTSServicer
    monkeypatch.setenv("MX_BACKEND_NAME", "coqui")
    monkeypatch.setenv("TTS_HOME", str(tmp_path / "nohome"))
    s = TTSServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="tts_models/en/ljspeech/glow-tts", ModelPath=str(tmp_path)), None)
    assert not r.success and "not found locally" in r.message
    d = tmp_path / "xtts"
    d.mkdir()
    (d / "config.json").write_text(json.dumps({"model": "xtts", "model_args": {}, "audio": {}}), encoding="utf-8")
    torch.save({"model": {}}, d / "model.pth")
    r = s.LoadModel(pb.ModelOptions(Model=str(d)), None)
    assert not r.success and "XTTS checkpoint" in r.message and "lacks" in r.message
