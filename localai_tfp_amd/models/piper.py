"""Piper voices: `<voice>.onnx` + `<voice>.onnx.json` (the reference's default TTS backend,
backend/go/tts/piper.go:16-49 -> go-piper -> piper -> onnxruntime; core/backend/tts.go:24;
pkg/model/initializers.go:451-453) served by this framework's VITS engine (models/tts.py) instead of an
ONNX runtime.

* weights: the graph initializers of the exported piper VITS (formats/onnx.py reads them without onnx),
  in the original VITS module names of piper's training code (enc_p / dp / flow / dec / emb_g), are
  renamed to the HF VitsModel names models/tts.py consumes (`piper_to_hf`): kernel-1 attention convs
  become linears, the coupling layers lose the interleaved Flip modules' indices, LayerNorm gamma/beta
  become weight/bias. The posterior encoder (enc_q, training only) is dropped.
* architecture: piper's .onnx.json stores audio / inference / phoneme settings but no layer sizes, so
  they are read off the tensor shapes (`config_from`); the head count (2) and the HiFi-GAN upsample
  rates (kernel / 2) and dilations (1, 3, 5, ...) follow piper's fixed training configs.
* text -> ids (`PiperPhonemes`, piper-phonemize semantics): phonemes are Unicode code points looked up
  in `phoneme_id_map`, with BOS "^", EOS "$" and the pad "_" after BOS and after every phoneme.
  phoneme_type "text" uses the characters themselves; "espeak" runs the `espeak-ng` program when one is
  installed (`--ipa`, data directory = the backend's LibrarySearchPath / `espeak_data` option), else a
  built-in English letter-to-sound rule set (approximate; parity with espeak-ng is unpinned).
Only ResBlock1 vocoders (piper's medium / high voices) are supported; x_low voices (ResBlock2) refuse.
"""
from __future__ import annotations

import json
import logging
import os
import re
import shutil
import subprocess
import unicodedata

import numpy as np
import torch

from .tts import VitsConfig, VitsModel

log = logging.getLogger("localai_tfp_amd.piper")

_ATT = {"q": "q_proj", "k": "k_proj", "v": "v_proj", "o": "out_proj"}
_LN = {"gamma": "weight", "beta": "bias"}
_DDS = {"convs_sep": "convs_dilated", "convs_1x1": "convs_pointwise", "norms_1": "norms_1", "norms_2": "norms_2"}


def _rename(k: str) -> str | None:
    """One original-VITS (piper) parameter name -> the HF VitsModel name, None if not used at inference."""
    m = re.match(r"enc_p\.encoder\.attn_layers\.(\d+)\.conv_([qkvo])\.(weight|bias)$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[1]}.attention.{_ATT[m[2]]}.{m[3]}"
    m = re.match(r"enc_p\.encoder\.attn_layers\.(\d+)\.emb_rel_([kv])$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[1]}.attention.emb_rel_{m[2]}"
    m = re.match(r"enc_p\.encoder\.norm_layers_([12])\.(\d+)\.(gamma|beta)$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[2]}.{'layer_norm' if m[1] == '1' else 'final_layer_norm'}.{_LN[m[3]]}"
    m = re.match(r"enc_p\.encoder\.ffn_layers\.(\d+)\.conv_([12])\.(weight|bias)$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[1]}.feed_forward.conv_{m[2]}.{m[3]}"
    if k == "enc_p.emb.weight":
        return "text_encoder.embed_tokens.weight"
    m = re.match(r"enc_p\.proj\.(weight|bias)$", k)
    if m:
        return f"text_encoder.project.{m[1]}"
    # stochastic duration predictor
    m = re.match(r"dp\.(pre|proj|post_pre|post_proj|cond)\.(weight|bias)$", k)
    if m:
        nm = {"pre": "conv_pre", "proj": "conv_proj", "post_pre": "post_conv_pre", "post_proj": "post_conv_proj",
              "cond": "cond"}[m[1]]
        return f"duration_predictor.{nm}.{m[2]}"
    m = re.match(r"dp\.(convs|post_convs)\.(convs_sep|convs_1x1|norms_1|norms_2)\.(\d+)\.(weight|bias|gamma|beta)$", k)
    if m:
        blk = "conv_dds" if m[1] == "convs" else "post_conv_dds"
        return f"duration_predictor.{blk}.{_DDS[m[2]]}.{m[3]}.{_LN.get(m[4], m[4])}"
    m = re.match(r"dp\.(flows|post_flows)\.0\.(m|logs)$", k)
    if m:
        return f"duration_predictor.{m[1]}.0.{'translate' if m[2] == 'm' else 'log_scale'}"
    # ConvFlows sit at the odd indices of [ElementwiseAffine, (ConvFlow, Flip) x n]
    m = re.match(r"dp\.(flows|post_flows)\.(\d+)\.(pre|proj)\.(weight|bias)$", k)
    if m:
        return f"duration_predictor.{m[1]}.{(int(m[2]) + 1) // 2}.conv_{m[3]}.{m[4]}"
    m = re.match(r"dp\.(flows|post_flows)\.(\d+)\.convs\.(convs_sep|convs_1x1|norms_1|norms_2)\.(\d+)\.(weight|bias|gamma|beta)$", k)
    if m:
        return f"duration_predictor.{m[1]}.{(int(m[2]) + 1) // 2}.conv_dds.{_DDS[m[3]]}.{m[4]}.{_LN.get(m[5], m[5])}"
    # deterministic duration predictor (use_sdp = False voices)
    m = re.match(r"dp\.(conv_1|conv_2|proj)\.(weight|bias)$", k)
    if m:
        return f"duration_predictor.{m[1]}.{m[2]}"
    m = re.match(r"dp\.(norm_1|norm_2)\.(gamma|beta)$", k)
    if m:
        return f"duration_predictor.{m[1]}.{_LN[m[2]]}"
    # prior flow: coupling layers at the even indices of [(ResidualCouplingLayer, Flip) x n]
    m = re.match(r"flow\.flows\.(\d+)\.(pre|post)\.(weight|bias)$", k)
    if m:
        return f"flow.flows.{int(m[1]) // 2}.conv_{m[2]}.{m[3]}"
    m = re.match(r"flow\.flows\.(\d+)\.enc\.(in_layers|res_skip_layers)\.(\d+)\.(weight|bias)$", k)
    if m:
        return f"flow.flows.{int(m[1]) // 2}.wavenet.{m[2]}.{m[3]}.{m[4]}"
    m = re.match(r"flow\.flows\.(\d+)\.enc\.cond_layer\.(weight|bias)$", k)
    if m:
        return f"flow.flows.{int(m[1]) // 2}.wavenet.cond_layer.{m[2]}"
    # HiFi-GAN generator
    m = re.match(r"dec\.(conv_pre|conv_post|cond)\.(weight|bias)$", k)
    if m:
        return f"decoder.{m[1]}.{m[2]}"
    m = re.match(r"dec\.ups\.(\d+)\.(weight|bias)$", k)
    if m:
        return f"decoder.upsampler.{m[1]}.{m[2]}"
    m = re.match(r"dec\.resblocks\.(\d+)\.(convs1|convs2)\.(\d+)\.(weight|bias)$", k)
    if m:
        return f"decoder.resblocks.{m[1]}.{m[2]}.{m[3]}.{m[4]}"
    if k == "emb_g.weight":
        return "embed_speaker.weight"
    return None


def piper_to_hf(tensors: dict) -> dict[str, torch.Tensor]:
    """Original-VITS state (piper ONNX initializers; weight norm already removed at export) -> HF names."""
    if any(re.match(r"dec\.resblocks\.\d+\.convs\.", k) for k in tensors):
        raise ValueError("piper x_low voices (HiFi-GAN ResBlock2 vocoder) are not supported; use a medium/high voice")
    out = {}
    unused = []
    for k, v in tensors.items():
        nk = _rename(k)
        if nk is None:
            if not k.startswith("enc_q."):
                unused.append(k)
            continue
        t = torch.from_numpy(np.asarray(v, np.float32).copy())
        if ".attention." in nk and nk.endswith("proj.weight") and t.dim() == 3:
            t = t[..., 0]  # kernel-1 Conv1d -> Linear
        out[nk] = t
    if unused:
        log.info("piper: %d initializers not used at inference (e.g. %s)", len(unused), unused[:3])
    return out


def _count(sd, pat):
    idx = {int(m[1]) for k in sd for m in [re.match(pat, k)] if m}
    return max(idx) + 1 if idx else 0


def config_from(sd: dict, meta: dict) -> VitsConfig:
    """VitsConfig from the HF-named tensors + the voice's .onnx.json."""
    emb = sd["text_encoder.embed_tokens.weight"]
    hidden = int(emb.shape[1])
    n_layers = _count(sd, r"text_encoder\.encoder\.layers\.(\d+)\.")
    c1 = sd["text_encoder.encoder.layers.0.feed_forward.conv_1.weight"]
    rel = sd.get("text_encoder.encoder.layers.0.attention.emb_rel_k")
    sdp = "duration_predictor.conv_pre.weight" in sd
    n_ups = _count(sd, r"decoder\.upsampler\.(\d+)\.")
    kernels = tuple(int(sd[f"decoder.upsampler.{i}.weight"].shape[2]) for i in range(n_ups))
    nk = _count(sd, r"decoder\.resblocks\.(\d+)\.") // max(n_ups, 1)
    rk = tuple(int(sd[f"decoder.resblocks.{j}.convs1.0.weight"].shape[2]) for j in range(nk))
    ndil = _count(sd, r"decoder\.resblocks\.0\.convs1\.(\d+)\.")
    base_dil = (1, 3, 5, 7, 9, 11)[:ndil]
    kw = {}
    if sdp:
        kw.update(dp_filter=int(sd["duration_predictor.conv_pre.weight"].shape[0]),
                  dp_kernel=int(sd["duration_predictor.conv_dds.convs_dilated.0.weight"].shape[2]),
                  dds_layers=_count(sd, r"duration_predictor\.conv_dds\.convs_dilated\.(\d+)\."),
                  dp_flows=_count(sd, r"duration_predictor\.flows\.(\d+)\.") - 1,
                  flow_bins=(int(sd["duration_predictor.flows.1.conv_proj.weight"].shape[0]) + 1) // 3)
    else:
        kw.update(dp_filter=int(sd["duration_predictor.conv_1.weight"].shape[0]),
                  dp_kernel=int(sd["duration_predictor.conv_1.weight"].shape[2]))
    spk = sd.get("embed_speaker.weight")
    inf = meta.get("inference", {})
    ls = float(inf.get("length_scale", 1.0) or 1.0)
    return VitsConfig(
        vocab=int(emb.shape[0]), hidden=hidden, n_layers=n_layers, n_heads=2, ffn=int(c1.shape[0]),
        ffn_kernel=int(c1.shape[2]), window=(int(rel.shape[1]) - 1) // 2 if rel is not None else 0,
        flow_size=int(sd["text_encoder.project.weight"].shape[0]) // 2, sdp=sdp,
        prior_flows=_count(sd, r"flow\.flows\.(\d+)\."),
        prior_wn_layers=_count(sd, r"flow\.flows\.0\.wavenet\.in_layers\.(\d+)\."),
        wn_kernel=int(sd["flow.flows.0.wavenet.in_layers.0.weight"].shape[2]),
        upsample_initial=int(sd["decoder.conv_pre.weight"].shape[0]), upsample_rates=tuple(k // 2 for k in kernels),
        upsample_kernels=kernels, resblock_kernels=rk, resblock_dilations=tuple(base_dil for _ in rk),
        n_speakers=int(spk.shape[0]) if spk is not None else 1, spk_dim=int(spk.shape[1]) if spk is not None else 0,
        sample_rate=int(meta.get("audio", {}).get("sample_rate", 22050)),
        noise_scale=float(inf.get("noise_scale", 0.667)), noise_scale_duration=float(inf.get("noise_w", 0.8)),
        speaking_rate=1.0 / ls, name=os.path.basename(meta.get("dataset", "") or "piper") or "piper", **kw)


# ------------------------------------------------------------------------------------------------ text
BOS, EOS, PAD = "^", "$", "_"


class PiperPhonemes:
    """text -> phoneme ids with piper-phonemize's id layout (BOS, PAD, then each phoneme + PAD, EOS)."""

    def __init__(self, meta: dict, espeak_data: str = "", lexicon: dict | None = None):
        self.id_map = {k: list(v) for k, v in meta.get("phoneme_id_map", {}).items()}
        if not self.id_map:
            raise ValueError("piper voice config has no phoneme_id_map")
        self.phoneme_map = meta.get("phoneme_map", {}) or {}
        self.kind = meta.get("phoneme_type", "espeak")
        self.voice = meta.get("espeak", {}).get("voice", "en-us")
        self.espeak_data = espeak_data
        self.lexicon = lexicon or {}
        self._espeak = shutil.which("espeak-ng") if self.kind == "espeak" else None
        if self.kind == "espeak" and not self._espeak and not self.voice.lower().startswith("en"):
            # the built-in rules are English only; a non-English voice would be fed English phonemes. No reader
            # of espeak-ng-data's compiled dictionaries ships here: refuse instead of synthesising garbage
            raise ValueError(f"piper voice {self.voice!r} needs the espeak-ng program for its phonemes (not found "
                             "on PATH); only English voices fall back to the built-in letter-to-sound rules")

    def phonemize(self, text: str) -> list[str]:
        text = unicodedata.normalize("NFC", text)
        if self.kind == "text":
            ph = unicodedata.normalize("NFD", text)
        elif self._espeak:
            ph = self._run_espeak(text)
        else:
            ph = english_to_ipa(text, self.lexicon)
        out = []
        for ch in ph:
            mapped = self.phoneme_map.get(ch, [ch])
            out.extend(mapped if isinstance(mapped, list) else [mapped])
        return out

    def _run_espeak(self, text: str) -> str:
        cmd = [self._espeak, "-q", "--ipa", "-v", self.voice]
        if self.espeak_data:
            cmd += ["--path", os.path.dirname(os.path.abspath(self.espeak_data.rstrip("/")))]
        try:
            r = subprocess.run(cmd + [text], capture_output=True, text=True, timeout=30, check=True)
            return " ".join(line.strip() for line in r.stdout.splitlines() if line.strip())
        except (OSError, subprocess.SubprocessError) as ex:
            log.warning("espeak-ng failed (%s): built-in English rules", ex)
            return english_to_ipa(text, self.lexicon)

    def encode(self, text: str) -> list[int]:
        m = self.id_map
        ids = list(m.get(BOS, [])) + list(m.get(PAD, []))
        for p in self.phonemize(text):
            if p in m:
                ids += m[p]
                ids += m.get(PAD, [])
        return ids + list(m.get(EOS, []))


# A compact English letter-to-sound rule set producing espeak-style IPA (stress mark before the first
# vowel of every word). Multi-letter rules first; a user lexicon (word -> IPA) overrides.
_RULES = [
    ("tion", "ʃən"), ("sion", "ʒən"), ("ough", "ɔː"), ("igh", "aɪ"), ("tch", "tʃ"), ("dge", "dʒ"), ("sch", "sk"),
    ("ph", "f"), ("th", "θ"), ("sh", "ʃ"), ("ch", "tʃ"), ("ck", "k"), ("ng", "ŋ"), ("qu", "kw"), ("wh", "w"),
    ("kn", "n"), ("wr", "ɹ"), ("ee", "iː"), ("ea", "iː"), ("oo", "uː"), ("ai", "eɪ"), ("ay", "eɪ"), ("oa", "oʊ"),
    ("ow", "aʊ"), ("ou", "aʊ"), ("oi", "ɔɪ"), ("oy", "ɔɪ"), ("au", "ɔː"), ("aw", "ɔː"), ("ew", "juː"), ("ie", "iː"),
    ("ar", "ɑːɹ"), ("or", "ɔːɹ"), ("er", "ɚ"), ("ir", "ɜː"), ("ur", "ɜː"), ("ll", "l"), ("ss", "s"), ("ff", "f"),
    ("tt", "t"), ("pp", "p"), ("mm", "m"), ("nn", "n"), ("rr", "ɹ"), ("bb", "b"), ("dd", "d"), ("gg", "ɡ"),
]
_SHORT = {"a": "æ", "e": "ɛ", "i": "ɪ", "o": "ɑ", "u": "ʌ", "y": "ɪ"}
_LONG = {"a": "eɪ", "e": "iː", "i": "aɪ", "o": "oʊ", "u": "juː", "y": "aɪ"}
_CONS = {"b": "b", "c": "k", "d": "d", "f": "f", "g": "ɡ", "h": "h", "j": "dʒ", "k": "k", "l": "l", "m": "m", "n": "n",
         "p": "p", "q": "k", "r": "ɹ", "s": "s", "t": "t", "v": "v", "w": "w", "x": "ks", "z": "z"}
_WORDS = {"the": "ðə", "a": "ə", "of": "ʌv", "to": "tuː", "and": "ænd", "is": "ɪz", "you": "juː", "i": "aɪ",
          "are": "ɑːɹ", "was": "wʌz", "one": "wʌn", "two": "tuː", "hello": "həlˈoʊ", "world": "wˈɜːld",
          "have": "hæv", "what": "wʌt", "do": "duː", "said": "sɛd", "there": "ðɛɹ", "this": "ðɪs", "be": "biː"}
_VOW = set("aeiouy")
_NUM = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine"]


def _word_ipa(w: str) -> str:
    out, i, n = [], 0, len(w)
    while i < n:
        for pat, ipa in _RULES:
            if w.startswith(pat, i):
                out.append(ipa)
                i += len(pat)
                break
        else:
            ch = w[i]
            nxt = w[i + 1] if i + 1 < n else ""
            if ch in _VOW and not (ch == "y" and i == 0):
                # magic e: vowel + one consonant + final e -> long vowel, the e silent
                if i + 2 == n - 1 and w[-1] == "e" and nxt and nxt not in _VOW:
                    out.append(_LONG[ch])
                elif ch == "e" and i == n - 1 and n > 2:
                    pass  # silent final e
                else:
                    out.append(_SHORT[ch] if i < n - 1 else _LONG.get(ch, _SHORT[ch]) if ch != "e" else "iː")
            elif ch == "y":
                out.append("j")
            elif ch == "c":
                out.append("s" if nxt in ("e", "i", "y") else "k")
            elif ch == "g" and nxt in ("e", "i", "y") and i > 0:
                out.append("dʒ")
            elif ch in _CONS:
                out.append(_CONS[ch])
            i += 1
    s = "".join(out)
    m = re.search(r"[æɛɪɑʌəeiaoɔuɚɜ]", s)
    return s if m is None or "ˈ" in s else s[:m.start()] + "ˈ" + s[m.start():]


def english_to_ipa(text: str, lexicon: dict | None = None) -> str:
    """Approximate English G2P (espeak-ng IPA conventions); punctuation kept as its own phoneme."""
    lex = lexicon or {}
    out = []
    for tok in re.findall(r"[A-Za-z']+|\d|[.,;:!?]", text):
        low = tok.lower().replace("'", "")
        if tok.isdigit():
            low = _NUM[int(tok)]
        if tok in ".,;:!?":
            out.append(tok)
            continue
        ipa = lex.get(low) or _WORDS.get(low) or _word_ipa(low)
        out.append(ipa)
    s = ""
    for t in out:
        s += t if (t in ".,;:!?" or not s) else " " + t
    return s


def _read_lexicon(paths: list[str]) -> dict:
    lex = {}
    for p in paths:
        if p and os.path.isfile(p):
            with open(p, encoding="utf-8") as f:
                for line in f:
                    parts = line.rstrip("\n").split("\t")
                    if len(parts) >= 2 and parts[0] and not parts[0].startswith("#"):
                        lex[parts[0].lower()] = parts[1]
    return lex


def load_piper(onnx_path: str, device="cpu", espeak_data: str = ""):
    """-> (VitsModel, PiperPhonemes) for `<voice>.onnx` with its `<voice>.onnx.json` next to it."""
    from ..formats import onnx as O
    cfg_path = onnx_path + ".json"
    if not os.path.isfile(cfg_path):
        alt = os.path.splitext(onnx_path)[0] + ".json"
        cfg_path = alt if os.path.isfile(alt) else cfg_path
    if not os.path.isfile(cfg_path):
        raise ValueError(f"{onnx_path}: piper voice config {os.path.basename(onnx_path)}.json not found next to it")
    meta = json.load(open(cfg_path, encoding="utf-8"))
    tensors, _ = O.initializers(onnx_path)
    sd = piper_to_hf(tensors)
    cfg = config_from(sd, meta)
    d = os.path.dirname(os.path.abspath(onnx_path))
    lex = _read_lexicon([os.path.splitext(onnx_path)[0] + ".lexicon", os.path.join(d, "lexicon.txt"),
                         os.path.join(espeak_data, "lexicon.txt") if espeak_data else ""])
    if espeak_data and not os.path.isdir(espeak_data):
        log.warning("espeak-ng data directory %s does not exist", espeak_data)
    return VitsModel(cfg, sd, device), PiperPhonemes(meta, espeak_data, lex)
