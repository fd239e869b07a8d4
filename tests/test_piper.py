"""Piper voices (backend/go/tts/piper.go:16-49, pkg/model/initializers.go:451-453): a synthetic
`<voice>.onnx` whose initializers carry piper's original-VITS module names (enc_p / dp / flow / dec /
emb_g, kernel-1 attention convs, Flip-interleaved flow indices, LayerNorm gamma/beta) plus the
`<voice>.onnx.json` config loads into exactly the weights it was written from, the phoneme-id layout
follows piper-phonemize (BOS, PAD, phoneme + PAD ..., EOS), and the voice synthesises through the TTS
worker. No real piper voice, espeak-ng or onnxruntime exists here: parity with piper's audio is unpinned."""
import json
import re

import numpy as np
import pytest
import torch

from localai_tfp_amd.models import tts as T
from localai_tfp_amd.models.piper import BOS, EOS, PAD, PiperPhonemes, english_to_ipa, load_piper

pytest.importorskip("transformers")

_INV_ATT = {"q_proj": "q", "k_proj": "k", "v_proj": "v", "out_proj": "o"}


def hf_to_original(sd: dict) -> dict:
    """HF VitsModel names -> original VITS (piper training code) names, written independently of the loader."""
    out = {}
    for k, v in sd.items():
        a = v.numpy().astype(np.float32)
        m = re.match(r"text_encoder\.encoder\.layers\.(\d+)\.(.+)$", k)
        if m:
            i, rest = m[1], m[2]
            if rest.startswith("attention."):
                _, nm, *lf = rest.split(".")
                if nm.startswith("emb_rel"):
                    out[f"enc_p.encoder.attn_layers.{i}.{nm}"] = a
                else:
                    out[f"enc_p.encoder.attn_layers.{i}.conv_{_INV_ATT[nm]}.{lf[0]}"] = a[..., None] if lf[0] == "weight" else a
            elif rest.startswith(("layer_norm.", "final_layer_norm.")):
                n = "1" if rest.startswith("layer_norm.") else "2"
                out[f"enc_p.encoder.norm_layers_{n}.{i}.{'gamma' if rest.endswith('weight') else 'beta'}"] = a
            elif rest.startswith("feed_forward."):
                out[f"enc_p.encoder.ffn_layers.{i}.{rest[len('feed_forward.'):]}"] = a
            continue
        if k == "text_encoder.embed_tokens.weight":
            out["enc_p.emb.weight"] = a
        elif k.startswith("text_encoder.project."):
            out["enc_p.proj." + k.rsplit(".", 1)[1]] = a
        elif k.startswith("duration_predictor."):
            r = k[len("duration_predictor."):]
            r = re.sub(r"^(post_)?flows\.0\.translate$", lambda m: f"{m[1] or ''}flows.0.m", r)
            r = re.sub(r"^(post_)?flows\.0\.log_scale$", lambda m: f"{m[1] or ''}flows.0.logs", r)
            r = re.sub(r"^(post_)?flows\.(\d+)\.", lambda m: f"{m[1] or ''}flows.{2 * int(m[2]) - 1}." if m[2] != "0"
                       else m[0], r)
            r = r.replace("post_conv_pre", "post_pre").replace("post_conv_proj", "post_proj")
            r = r.replace("post_conv_dds.", "post_convs.").replace("conv_dds.", "convs.")
            r = r.replace("conv_pre", "pre").replace("conv_proj", "proj")
            r = r.replace("convs_dilated", "convs_sep").replace("convs_pointwise", "convs_1x1")
            if re.search(r"norms_[12]\.\d+\.(weight|bias)$", r):
                r = r[:-6] + "gamma" if r.endswith("weight") else r[:-4] + "beta"
            out["dp." + r] = a
        elif k.startswith("flow.flows."):
            m = re.match(r"flow\.flows\.(\d+)\.(.+)$", k)
            r = m[2].replace("conv_pre", "pre").replace("conv_post", "post").replace("wavenet.", "enc.")
            out[f"flow.flows.{2 * int(m[1])}.{r}"] = a
        elif k.startswith("decoder."):
            out["dec." + k[len("decoder."):].replace("upsampler.", "ups.")] = a
        elif k == "embed_speaker.weight":
            out["emb_g.weight"] = a
    out["enc_q.pre.weight"] = np.zeros((4, 4, 1), np.float32)  # posterior encoder: present in exports, unused
    return out


PHONES = list(" ,.!?abdefhijklmnoprstuvwzæðŋɑɔəɚɛɜɡɪɹʃʊʌʒθˈˌː") + ["ɐ", "oʊ"]


def voice_json(kind="espeak", sr=22050):
    ids = {PAD: [0], BOS: [1], EOS: [2]}
    for i, p in enumerate(PHONES):
        ids.setdefault(p, [3 + i])
    return {"audio": {"sample_rate": sr}, "espeak": {"voice": "en-us"}, "phoneme_type": kind,
            "inference": {"noise_scale": 0.0, "length_scale": 1.25, "noise_w": 0.0},
            "phoneme_id_map": ids, "num_symbols": 64, "num_speakers": 1, "speaker_id_map": {}, "dataset": "test"}


def make_voice(tmp_path, cfg=None, kind="espeak", name="en_US-test-medium.onnx"):
    from localai_tfp_amd.formats import onnx as O
    cfg = cfg or T.VitsConfig(**{**T.VITS_TEST.__dict__, "vocab": 64})
    sd = T.synthetic_vits(cfg, seed=2)
    p = tmp_path / name
    p.write_bytes(O.make_model(hf_to_original(sd)))
    (tmp_path / (name + ".json")).write_text(json.dumps(voice_json(kind)), encoding="utf-8")
    return str(p), sd, cfg


def test_piper_onnx_weights_and_config(tmp_path):
    path, sd, cfg = make_voice(tmp_path)
    m, tok = load_piper(path)
    sd = {k: v for k, v in sd.items() if not k.startswith("posterior_encoder.")}  # training-only
    assert set(m.w) == set(sd)
    for k, v in sd.items():
        assert torch.equal(m.w[k], v.float()), k
    c = m.cfg
    for f in ("vocab", "hidden", "n_layers", "n_heads", "ffn", "ffn_kernel", "window", "flow_size", "sdp", "dp_filter",
              "dp_kernel", "dds_layers", "flow_bins", "dp_flows", "prior_flows", "prior_wn_layers", "wn_kernel",
              "upsample_initial", "upsample_rates", "upsample_kernels", "resblock_kernels", "resblock_dilations"):
        assert getattr(c, f) == getattr(cfg, f), f
    assert c.sample_rate == 22050 and c.speaking_rate == pytest.approx(0.8) and c.noise_scale == 0.0


def test_piper_phoneme_ids():
    ph = PiperPhonemes(voice_json("text"))
    assert ph.encode("ab") == [1, 0, PHONES.index("a") + 3, 0, PHONES.index("b") + 3, 0, 2]
    ph = PiperPhonemes(voice_json("espeak"))
    ph._espeak = None  # no espeak-ng in this image: the built-in English rules
    ipa = english_to_ipa("Hello world, this is a test.")
    assert ipa.startswith("həlˈoʊ wˈɜːld,") and ipa.endswith(".")
    ids = ph.encode("Hello world, this is a test.")
    assert ids[:2] == [1, 0] and ids[-1] == 2 and all(i in range(len(PHONES) + 3) for i in ids)
    assert ids[2::2][:-1] and all(x == 0 for x in ids[3:-1:2])  # PAD after every phoneme
    lex = PiperPhonemes(voice_json("espeak"), lexicon={"mi": "ɛmˈaɪ"})
    lex._espeak = None
    assert lex.phonemize("mi") == list("ɛmˈaɪ")


def test_piper_synthesises_through_worker(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.tts import TTSServicer
    path, sd, cfg = make_voice(tmp_path)
    s = TTSServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="en_US-test-medium.onnx", ModelPath=str(tmp_path),
                                    LibrarySearchPath=str(tmp_path / "espeak-ng-data")), None)
    assert r.success, r.message
    s.tok._espeak = None
    dst = str(tmp_path / "o.wav")
    r = s.TTS(pb.TTSRequest(text="Hello from the GPU.", model="en_US-test-medium.onnx", dst=dst), None)
    assert r.success, r.message
    import wave
    with wave.open(dst) as w:
        assert w.getframerate() == 22050 and w.getnframes() > 0
    # the same ids through the VITS engine directly with the source weights: identical audio
    ids = s.tok.encode("Hello from the GPU.")
    ref = T.VitsModel(s.model.cfg, sd, "cpu").synthesize(ids, seed=0)
    got = s.model.synthesize(ids, seed=0)
    np.testing.assert_array_equal(got, ref)


def test_piper_x_low_refused(tmp_path):
    from localai_tfp_amd.formats import onnx as O
    path, sd, cfg = make_voice(tmp_path)
    t, _ = O.initializers(path)
    t = {re.sub(r"\.convs1\.", ".convs.", k): v for k, v in t.items() if ".convs2." not in k}
    p2 = tmp_path / "x_low.onnx"
    p2.write_bytes(O.make_model(t))
    (tmp_path / "x_low.onnx.json").write_text(json.dumps(voice_json()), encoding="utf-8")
    with pytest.raises(ValueError, match="x_low"):
        load_piper(str(p2))


def test_piper_non_english_without_espeak_refused(monkeypatch):
    """No espeak-ng program and no reader of espeak-ng-data's compiled dictionaries: a non-English espeak voice
    is refused at load instead of being fed the built-in English phonemes (English voices still fall back)."""
    import localai_tfp_amd.models.piper as P
    monkeypatch.setattr(P.shutil, "which", lambda name: None)
    meta = voice_json("espeak")
    meta["espeak"] = {"voice": "de"}
    with pytest.raises(ValueError, match="espeak-ng"):
        PiperPhonemes(meta)
    meta["espeak"] = {"voice": "en-gb"}
    assert PiperPhonemes(meta).encode("hi")[:2] == [1, 0]
