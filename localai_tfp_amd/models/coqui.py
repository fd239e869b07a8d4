"""Coqui TTS VITS checkpoints (the reference's `coqui` backend: backend/python/coqui/backend.py:26-80 loads
`TTS(request.Model)`, its test loads "tts_models/en/vctk/vits" — test.py:55) served by this framework's
VITS engine (models/tts.py).

A Coqui model directory holds `config.json` (Coqpit dump: `model`, `model_args`, `audio`, `characters`,
phonemizer settings) and a `model_file.pth` / `model.pth` / `best_model.pth` whose `"model"` entry is the
state dict in Coqui's module names (text_encoder / duration_predictor / flow / waveform_decoder / emb_g;
posterior_encoder and the discriminator are training-only). Loaded with `torch.load(weights_only=True)`:
a checkpoint that pickles anything but tensors and plain containers is refused, never unpickled.

* weights: weight-norm pairs folded (`fold_weight_norm`), then renamed to the HF VitsModel names the
  engine consumes. Coqui's flows carry no Flip modules (it flips in forward), so flow / duration-flow
  indices map 1:1 — unlike piper's original-VITS names (models/piper.py).
* architecture: layer sizes from tensor shapes (`piper.config_from`), decoder rates / dilations and the
  inference noise / length scales from `model_args`.
* text -> ids (`CoquiTokenizer`, TTS/tts/utils/text semantics): cleaners (lower-case, whitespace), an
  optional phonemizer (`espeak-ng` when installed, else the built-in English rules of models/piper.py —
  parity with Coqui's phonemizer output is unpinned), the character vocabulary in Coqui's order
  (VitsCharacters: pad, punctuations, characters, blank; the other character classes: pad, eos, bos,
  blank, characters, punctuations), optional BOS/EOS and blank interspersing (`add_blank`).
* speakers: `voice` is a speaker name from `speakers.json` / `speaker_ids.json` / `speakers.pth` (or
  config `speaker_ids`), or an integer id.
XTTS (`"model": "xtts"`, a GPT-2 audio-code LM + HiFi-GAN decoder) directories load through models/xtts.py
(the TTS worker dispatches on config.json before calling load_coqui).
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
import re
import shutil
import subprocess

import torch

from .piper import config_from, english_to_ipa
from .tts import VitsModel, fold_weight_norm

log = logging.getLogger("localai_tfp_amd.coqui")

CKPT_NAMES = ("model_file.pth", "model.pth", "best_model.pth", "checkpoint.pth", "model_file.pth.tar")
_ATT = {"q": "q_proj", "k": "k_proj", "v": "v_proj", "o": "out_proj"}
_LN = {"gamma": "weight", "beta": "bias", "weight": "weight", "bias": "bias"}
_DDS = {"convs_sep": "convs_dilated", "convs_1x1": "convs_pointwise", "norms_1": "norms_1", "norms_2": "norms_2"}


def _rename(k: str) -> str | None:
    """One Coqui VITS parameter name -> the HF VitsModel name, None if not used at inference."""
    m = re.match(r"text_encoder\.encoder\.attn_layers\.(\d+)\.conv_([qkvo])\.(weight|bias)$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[1]}.attention.{_ATT[m[2]]}.{m[3]}"
    m = re.match(r"text_encoder\.encoder\.attn_layers\.(\d+)\.emb_rel_([kv])$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[1]}.attention.emb_rel_{m[2]}"
    m = re.match(r"text_encoder\.encoder\.norm_layers_([12])\.(\d+)\.(gamma|beta|weight|bias)$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[2]}.{'layer_norm' if m[1] == '1' else 'final_layer_norm'}.{_LN[m[3]]}"
    m = re.match(r"text_encoder\.encoder\.ffn_layers\.(\d+)\.conv_([12])\.(weight|bias)$", k)
    if m:
        return f"text_encoder.encoder.layers.{m[1]}.feed_forward.conv_{m[2]}.{m[3]}"
    if k == "text_encoder.emb.weight":
        return "text_encoder.embed_tokens.weight"
    m = re.match(r"text_encoder\.proj\.(weight|bias)$", k)
    if m:
        return f"text_encoder.project.{m[1]}"
    # stochastic duration predictor (no Flip modules: flow i -> HF flow i)
    dp = "duration_predictor."
    if k.startswith(dp):
        r = k[len(dp):]
        m = re.match(r"(pre|proj|post_pre|post_proj|cond)\.(weight|bias)$", r)
        if m:
            nm = {"pre": "conv_pre", "proj": "conv_proj", "post_pre": "post_conv_pre", "post_proj": "post_conv_proj",
                  "cond": "cond"}[m[1]]
            return f"{dp}{nm}.{m[2]}"
        m = re.match(r"(convs|post_convs)\.(convs_sep|convs_1x1|norms_1|norms_2)\.(\d+)\.(weight|bias|gamma|beta)$", r)
        if m:
            blk = "conv_dds" if m[1] == "convs" else "post_conv_dds"
            return f"{dp}{blk}.{_DDS[m[2]]}.{m[3]}.{_LN[m[4]]}"
        m = re.match(r"(flows|post_flows)\.0\.(translation|translate|m|log_scale|logs)$", r)
        if m:
            return f"{dp}{m[1]}.0.{'log_scale' if m[2] in ('log_scale', 'logs') else 'translate'}"
        m = re.match(r"(flows|post_flows)\.(\d+)\.(pre|proj)\.(weight|bias)$", r)
        if m:
            return f"{dp}{m[1]}.{m[2]}.conv_{m[3]}.{m[4]}"
        m = re.match(r"(flows|post_flows)\.(\d+)\.convs\.(convs_sep|convs_1x1|norms_1|norms_2)\.(\d+)\.(weight|bias|gamma|beta)$", r)
        if m:
            return f"{dp}{m[1]}.{m[2]}.conv_dds.{_DDS[m[3]]}.{m[4]}.{_LN[m[5]]}"
        # deterministic duration predictor (use_sdp = false)
        m = re.match(r"(conv_1|conv_2|proj|cond)\.(weight|bias)$", r)
        if m:
            return f"{dp}{m[1]}.{m[2]}"
        m = re.match(r"(norm_1|norm_2)\.(gamma|beta|weight|bias)$", r)
        if m:
            return f"{dp}{m[1]}.{_LN[m[2]]}"
        return None
    # prior flow: coupling layers only (Coqui flips in forward)
    m = re.match(r"flow\.flows\.(\d+)\.(pre|post)\.(weight|bias)$", k)
    if m:
        return f"flow.flows.{m[1]}.conv_{m[2]}.{m[3]}"
    m = re.match(r"flow\.flows\.(\d+)\.enc\.(in_layers|res_skip_layers)\.(\d+)\.(weight|bias)$", k)
    if m:
        return f"flow.flows.{m[1]}.wavenet.{m[2]}.{m[3]}.{m[4]}"
    m = re.match(r"flow\.flows\.(\d+)\.enc\.cond_layer\.(weight|bias)$", k)
    if m:
        return f"flow.flows.{m[1]}.wavenet.cond_layer.{m[2]}"
    # HiFi-GAN generator
    m = re.match(r"waveform_decoder\.(conv_pre|conv_post)\.(weight|bias)$", k)
    if m:
        return f"decoder.{m[1]}.{m[2]}"
    m = re.match(r"waveform_decoder\.(cond_layer|cond)\.(weight|bias)$", k)
    if m:
        return f"decoder.cond.{m[2]}"
    m = re.match(r"waveform_decoder\.ups\.(\d+)\.(weight|bias)$", k)
    if m:
        return f"decoder.upsampler.{m[1]}.{m[2]}"
    m = re.match(r"waveform_decoder\.resblocks\.(\d+)\.(convs1|convs2)\.(\d+)\.(weight|bias)$", k)
    if m:
        return f"decoder.resblocks.{m[1]}.{m[2]}.{m[3]}.{m[4]}"
    if k == "emb_g.weight":
        return "embed_speaker.weight"
    return None


def coqui_to_hf(sd: dict) -> dict[str, torch.Tensor]:
    """Coqui VITS state dict (weight-norm pairs allowed) -> HF VitsModel names."""
    if any(re.match(r"waveform_decoder\.resblocks\.\d+\.convs\.", k) for k in sd):
        raise ValueError("Coqui VITS with a ResBlock2 HiFi-GAN decoder (resblock_type_decoder '2') is not supported")
    sd = fold_weight_norm({k: v.float() for k, v in sd.items() if isinstance(v, torch.Tensor)})
    out, unused = {}, []
    for k, v in sd.items():
        nk = _rename(k)
        if nk is None:
            if not k.startswith(("posterior_encoder.", "disc.", "discriminator.", "emb_l.", "audio_transform")):
                unused.append(k)
            continue
        if ".attention." in nk and nk.endswith("proj.weight") and v.dim() == 3:
            v = v[..., 0]  # kernel-1 Conv1d -> Linear
        out[nk] = v.contiguous()
    if unused:
        log.info("coqui: %d tensors not used at inference (e.g. %s)", len(unused), unused[:3])
    return out


# ------------------------------------------------------------------------------------------------ text
_PUNCT = ";:,.!?¡¿—…\"«»“” "


class CoquiTokenizer:
    """Coqui TTSTokenizer semantics: clean -> (phonemize) -> ids in the characters config's vocabulary ->
    optional BOS/EOS -> optional blank interspersing."""

    def __init__(self, cfg: dict, espeak_data: str = ""):
        ch = cfg.get("characters") or {}
        self.use_phonemes = bool(cfg.get("use_phonemes", False))
        self.language = cfg.get("phoneme_language") or "en-us"
        self.add_blank = bool(cfg.get("add_blank", False))
        self.use_eos_bos = bool(cfg.get("enable_eos_bos_chars", False) or cfg.get("use_eos_bos", False))
        self.cleaner = cfg.get("text_cleaner") or ""
        cls_name = str(ch.get("characters_class", "") or "")
        pad, eos, bos, blank = (ch.get(k) for k in ("pad", "eos", "bos", "blank"))
        puncs = ch.get("punctuations", _PUNCT) if ch else _PUNCT
        syms = (ch.get("phonemes") if self.use_phonemes and ch.get("phonemes") else ch.get("characters")) or ""
        if ch.get("is_unique", True):
            syms = "".join(dict.fromkeys(syms))
        if ch.get("is_sorted", True) and "VitsCharacters" not in cls_name:
            syms = "".join(sorted(syms))
        if "VitsCharacters" in cls_name:
            vocab = ([pad] if pad else []) + list(puncs) + list(syms) + ([blank] if blank else [])
        else:
            vocab = [x for x in (pad, eos, bos, blank) if x] + list(syms) + list(puncs)
        self.vocab = vocab
        self.ids = {}
        for i, c in enumerate(vocab):
            self.ids.setdefault(c, i)
        self.pad_id = self.ids.get(pad, 0) if pad else 0
        self.blank_id = self.ids[blank] if blank and blank in self.ids else self.pad_id
        self.bos_id = self.ids.get(bos) if bos else None
        self.eos_id = self.ids.get(eos) if eos else None
        self.espeak_data = espeak_data
        self._espeak = (shutil.which("espeak-ng") or shutil.which("espeak")) if self.use_phonemes else None

    def clean(self, text: str) -> str:
        t = text
        if "english" in self.cleaner or "phoneme" in self.cleaner or "basic" in self.cleaner or "lowercase" in self.cleaner:
            t = t.lower()
        return re.sub(r"\s+", " ", t).strip()

    def phonemize(self, text: str) -> str:
        if self._espeak:
            cmd = [self._espeak, "-q", "--ipa", "-v", self.language]
            if self.espeak_data:
                cmd += ["--path", os.path.dirname(os.path.abspath(self.espeak_data.rstrip("/")))]
            try:
                r = subprocess.run(cmd + [text], capture_output=True, text=True, timeout=30, check=True)
                return " ".join(line.strip() for line in r.stdout.splitlines() if line.strip())
            except (OSError, subprocess.SubprocessError) as ex:
                log.warning("espeak-ng failed (%s): built-in English rules", ex)
        return english_to_ipa(text)

    def encode(self, text: str) -> list[int]:
        t = self.clean(text)
        if self.use_phonemes:
            t = self.phonemize(t)
        ids = [self.ids[c] for c in t if c in self.ids]
        if self.use_eos_bos:
            ids = ([self.bos_id] if self.bos_id is not None else []) + ids + ([self.eos_id] if self.eos_id is not None else [])
        if self.add_blank:
            out = [self.blank_id] * (2 * len(ids) + 1)
            out[1::2] = ids
            ids = out
        return ids


# ------------------------------------------------------------------------------------------------ load
def _find_ckpt(d: str) -> str:
    for n in CKPT_NAMES:
        p = os.path.join(d, n)
        if os.path.isfile(p):
            return p
    pths = sorted(f for f in os.listdir(d) if f.endswith((".pth", ".pt", ".pth.tar")) and "speaker" not in f)
    if pths:
        return os.path.join(d, pths[0])
    raise ValueError(f"{d}: no Coqui checkpoint ({' / '.join(CKPT_NAMES)})")


def resolve_model_dir(name: str, model_path: str = "") -> str | None:
    """A Coqui model name ("tts_models/en/vctk/vits") or path -> a local directory holding config.json.
    Coqui's own download cache layout (`tts_models--en--vctk--vits` under $TTS_HOME/tts or
    ~/.local/share/tts) is searched too; nothing is downloaded."""
    flat = name.replace("/", "--")
    homes = [os.environ.get("TTS_HOME", ""), os.environ.get("XDG_DATA_HOME", ""),
             os.path.join(os.path.expanduser("~"), ".local", "share")]
    cands = [name, os.path.join(model_path, name) if model_path else "", os.path.join(model_path, flat) if model_path else ""]
    cands += [os.path.join(h, "tts", flat) for h in homes if h]
    for c in cands:
        if c and os.path.isdir(c) and os.path.isfile(os.path.join(c, "config.json")):
            return c
        if c and os.path.isfile(c) and c.endswith((".pth", ".pt", ".pth.tar")) and \
                os.path.isfile(os.path.join(os.path.dirname(c), "config.json")):
            return os.path.dirname(c)
    return None


def is_coqui_dir(d: str) -> bool:
    try:
        cj = json.load(open(os.path.join(d, "config.json"), encoding="utf-8"))
    except (OSError, ValueError):
        return False
    return isinstance(cj, dict) and "model" in cj and ("model_args" in cj or "characters" in cj or "audio" in cj)


def _speakers(d: str, cfg: dict) -> dict:
    names = {}
    ma = cfg.get("model_args") or {}
    for key in ("speakers_file", "speaker_ids_file"):
        p = ma.get(key) or cfg.get(key)
        if p and not os.path.isabs(p):
            p = os.path.join(d, os.path.basename(p))
        if p and os.path.isfile(p):
            names.update(_read_speaker_file(p))
    for f in ("speakers.json", "speaker_ids.json", "speakers.pth"):
        p = os.path.join(d, f)
        if os.path.isfile(p):
            names.update(_read_speaker_file(p))
    if isinstance(cfg.get("speaker_ids"), dict):
        names.update(cfg["speaker_ids"])
    return {str(k): int(v) for k, v in names.items() if isinstance(v, (int, float))}


def _read_speaker_file(p: str) -> dict:
    try:
        if p.endswith(".json"):
            return json.load(open(p, encoding="utf-8"))
        v = torch.load(p, map_location="cpu", weights_only=True)
        return v if isinstance(v, dict) else {}
    except Exception as ex:  # a speaker file that only the unsafe loader could read: names unavailable
        log.warning("coqui speakers file %s not read (%s)", p, ex)
        return {}


def load_coqui(d: str, device="cpu", espeak_data: str = ""):
    """-> (VitsModel, CoquiTokenizer, speaker name -> id) for a Coqui VITS model directory."""
    cfg = json.load(open(os.path.join(d, "config.json"), encoding="utf-8"))
    kind = str(cfg.get("model", "")).lower()
    if kind == "xtts" or "xtts" in kind:
        raise ValueError("a Coqui XTTS directory: load it with models/xtts.load_xtts (load_coqui serves VITS)")
    if kind and kind != "vits":
        raise ValueError(f"Coqui model type {kind!r} is not implemented (Coqui VITS models are)")
    try:
        ck = torch.load(_find_ckpt(d), map_location="cpu", weights_only=True)
    except Exception as ex:
        raise ValueError(f"Coqui checkpoint not loadable with the weights-only loader: {ex}") from ex
    sd = ck.get("model", ck) if isinstance(ck, dict) else None
    if not isinstance(sd, dict):
        raise ValueError("Coqui checkpoint holds no state dict")
    hf = coqui_to_hf(sd)
    ma = cfg.get("model_args") or {}
    audio = cfg.get("audio") or {}
    meta = {"audio": {"sample_rate": int(audio.get("sample_rate", 22050))},
            "inference": {"noise_scale": ma.get("inference_noise_scale", 0.667),
                          "length_scale": ma.get("length_scale", 1.0),
                          "noise_w": ma.get("inference_noise_scale_dp", 1.0)},
            "dataset": os.path.basename(os.path.normpath(d))}
    vc = config_from(hf, meta)
    over = {}
    if ma.get("upsample_rates_decoder"):
        over["upsample_rates"] = tuple(int(x) for x in ma["upsample_rates_decoder"])
    if ma.get("resblock_dilation_sizes_decoder"):
        over["resblock_dilations"] = tuple(tuple(int(y) for y in x) for x in ma["resblock_dilation_sizes_decoder"])
    if ma.get("num_heads_text_encoder"):
        over["n_heads"] = int(ma["num_heads_text_encoder"])
    if ma.get("dilation_rate_flow"):
        over["wn_dilation"] = int(ma["dilation_rate_flow"])
    if str(ma.get("resblock_type_decoder", "1")) != "1":
        raise ValueError("Coqui VITS with a ResBlock2 HiFi-GAN decoder is not supported")
    vc = dataclasses.replace(vc, **over)
    tok = CoquiTokenizer(cfg, espeak_data)
    return VitsModel(vc, hf, device), tok, _speakers(d, cfg)
