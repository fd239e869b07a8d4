"""OuteTTS: a causal LM that writes audio-codec tokens word by word, decoded by WavTokenizer.

Reference: backend/python/transformers/backend.py:205-243 (LoadModel `type: OuteTTS`, options
`tokenizer:` / `version:` / `speaker:`, `AudioPath` speaker cloning) and :509-526 (generation at
temperature 0.1, repetition penalty 1.1, `max_length` = the request's max tokens, WAV written to `dst`).
The reference's handler synthesises a hard-coded sentence instead of the request text; this one speaks
`request.text`.

The LM (OuteTTS-0.2/0.3: Qwen-2.5-0.5B or Llama-3.2-1B weights in a Hugging Face directory) runs on this
framework's engine (paged KV, MFMA kernels, on-GPU sampler). Prompt (interface v0.2/v0.3):

  <|im_start|>\\n<|text_start|>w1<|text_sep|>w2...<|text_end|>\\n<|audio_start|>\\n
  [speaker words: word<|t_1.23|><|code_start|><|c_17|><|c_901|>...<|code_end|>\\n ...]

The speaker's transcript is prepended to the text and its words (with their durations and codes) are the
prefix of the audio section, so the model continues in that voice. v0.2 writes codes as `<|17|>` without
code_start/code_end. Speakers are outetts JSON profiles ({"text", "words": [{"word", "duration",
"codes"}]}); the outetts package's bundled default voices are not shipped here (no voice = the model's
own). AudioPath creates a profile (`create_speaker`): the clip's codes from the WavTokenizer SEANet encoder
(models/wavtokenizer.py `WavTokenizerEncoder`), its words from `speaker_text:` or Whisper segments, each
segment's codes shared over its words by length (outetts uses word timestamps; the boundaries here are an
approximation, the codes are exact).
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import dataclass

import numpy as np


def normalize_words(text: str) -> list[str]:
    """Lower-case words without punctuation (numbers kept as digits), as the outetts text processor
    feeds them to the model."""
    t = text.lower().replace("’", "'")
    t = re.sub(r"[^a-z0-9'\s]", " ", t)
    return [w for w in t.split() if w.strip("'")]


@dataclass
class Speaker:
    text: str
    words: list  # [{"word": str, "duration": float, "codes": [int]}]

    @classmethod
    def load(cls, path: str) -> "Speaker":
        with open(path, encoding="utf-8") as f:
            d = json.load(f)
        return cls(text=d.get("text", ""), words=list(d.get("words", [])))


def create_speaker(encoder, audio: np.ndarray, sample_rate: int, fps: float, transcript: str = "",
                   segments: list | None = None) -> Speaker:
    """Speaker profile from a reference clip (outetts `create_speaker`): the clip's WavTokenizer codes, cut into
    words. segments: [(start_s, end_s, text)] (e.g. Whisper's), else the whole clip with `transcript`. Within a
    segment the codes are shared out over its words in proportion to their length (outetts aligns words with
    Whisper word timestamps or a CTC aligner, neither of which ships here: the word boundaries are an
    approximation, the codes themselves are the clip's)."""
    import torch
    codes = encoder.encode(torch.from_numpy(np.asarray(audio, np.float32)))
    items = segments or [(0.0, len(audio) / sample_rate, transcript)]
    words, texts = [], []
    for s0, s1, text in items:
        ws = normalize_words(text or "")
        if not ws:
            continue
        texts.append(text.strip())
        c0, c1 = int(round(s0 * fps)), min(len(codes), int(round(s1 * fps)))
        if c1 <= c0:
            continue
        wt = np.cumsum([len(w) + 1 for w in ws], dtype=np.float64)
        bounds = [c0] + [c0 + int(round(x / wt[-1] * (c1 - c0))) for x in wt]
        for w, a, b in zip(ws, bounds, bounds[1:]):
            if b > a:
                wc = [int(v) for v in codes[a:b]]
                words.append({"word": w, "duration": round(len(wc) / fps, 2), "codes": wc})
    if not words:
        raise ValueError("speaker creation: no words (empty transcript, or the clip is shorter than a code frame)")
    return Speaker(text=" ".join(texts), words=words)


class PromptV2:
    """outetts interface v0.2 / v0.3 prompt format."""

    def __init__(self, version: str = "0.3"):
        self.version = version
        self.v3 = version.startswith("0.3")

    def code(self, c: int) -> str:
        return f"<|c_{c}|>" if self.v3 else f"<|{c}|>"

    def word_line(self, w: dict) -> str:
        codes = "".join(self.code(int(c)) for c in w["codes"])
        if self.v3:
            codes = f"<|code_start|>{codes}<|code_end|>"
        return f"{w['word']}<|t_{float(w['duration']):.2f}|>{codes}"

    def completion(self, text: str, speaker: Speaker | None = None) -> str:
        words = normalize_words(text)
        if speaker is not None:
            words = normalize_words(speaker.text) + words
        p = "<|im_start|>\n<|text_start|>" + "<|text_sep|>".join(words) + "<|text_end|>\n<|audio_start|>\n"
        if speaker is not None and speaker.words:
            p += "\n".join(self.word_line(w) for w in speaker.words) + "\n"
        return p

    def codes(self, generated: str) -> list[int]:
        pat = r"<\|c_(\d+)\|>" if self.v3 else r"<\|(\d+)\|>"
        return [int(m) for m in re.findall(pat, generated)]


def _single_id(tok, s: str):
    """Id of a token written as one added token (None if the tokenizer splits it)."""
    try:
        ids = tok.encode(s, add_special=False, parse_special=True)
    except Exception:
        return None
    return ids[0] if len(ids) == 1 else None


class OuteTTS:
    """LM engine + WavTokenizer. `generate_text(prompt, max_tokens)` is the LM call (the engine here;
    replaceable in tests)."""

    def __init__(self, engine, tok, codec, version: str = "0.3", speaker: Speaker | None = None):
        self.engine, self.tok, self.codec = engine, tok, codec
        self.prompt = PromptV2(version)
        self.speaker = speaker

    def generate_text(self, prompt: str, max_tokens: int, seed: int = 0) -> str:
        from ..engine.sequence import Request
        from ..ops.sampling import SamplingParams
        ids = self.tok.encode(prompt, add_special=False, parse_special=True)
        sp = SamplingParams(temperature=0.1, top_k=40, top_p=0.9, min_p=0.05, repeat_penalty=1.1,
                            repeat_last_n=64, seed=seed)
        stop = [i for i in (_single_id(self.tok, "<|audio_end|>"), getattr(self.tok, "eos_token_id", None))
                if i is not None]
        h = self.engine.submit(Request(ids, sp, max_tokens, stop_token_ids=stop))
        self.engine.run_until_done()
        out = []
        for o in h:
            out += o.token_ids
        return self.tok.decode(out, skip_special=False)  # the code tokens are added (special) tokens

    def synthesize(self, text: str, max_tokens: int = 4096, seed: int = 0) -> np.ndarray:
        import torch
        gen = self.generate_text(self.prompt.completion(text, self.speaker), max_tokens, seed)
        codes = self.prompt.codes(gen)
        if not codes:
            raise ValueError("the model produced no audio codes")
        dev = self.codec.codebook.device
        return self.codec.decode(torch.tensor(codes, device=dev)).cpu().numpy()

    @property
    def sample_rate(self) -> int:
        return self.codec.cfg.sample_rate


def load_outetts(model: str, device: str, options: dict, audio_path: str = "", model_path: str = "") -> OuteTTS:
    """model: a Hugging Face OuteTTS directory (or `synthetic:outetts-test`); options: version (0.2 / 0.3),
    tokenizer (directory), speaker (an outetts speaker JSON, relative to model_path), wavtokenizer
    (codec checkpoint; default <model>/wavtokenizer); audio_path (a reference clip: the speaker is created
    from it, with option speaker_text:<its transcript> or whisper:<model> to transcribe it)."""
    from ..engine.engine import EngineConfig, LLMEngine
    from .loader import load_llm
    from .wavtokenizer import WAVTOKENIZER_TEST, WavTokenizerDecoder, load_wavtokenizer
    version = options.get("version", "0.3")

    def full(p):
        return p if not p or os.path.isabs(p) or not model_path else os.path.join(model_path, p)
    wt = ""
    if model.startswith("synthetic:"):
        model_, tok, cfg, _ = load_llm("synthetic:tiny", device)
        codec = WavTokenizerDecoder(WAVTOKENIZER_TEST)
        from .diffusion.nn import init_synthetic
        init_synthetic(codec, 7)
        codec = codec.to(device).eval()
    else:
        model_, tok, cfg, _ = load_llm(model, device)
        if options.get("tokenizer"):
            from ..tokenizer import from_hf_dir
            tok = from_hf_dir(full(options["tokenizer"]))
        wt = full(options.get("wavtokenizer", "")) or os.path.join(model, "wavtokenizer")
        if not os.path.exists(wt):
            raise FileNotFoundError(f"OuteTTS: WavTokenizer checkpoint not found at {wt} (option wavtokenizer:<path>)")
        import torch
        codec = load_wavtokenizer(wt, device, torch.float32)
    eng = LLMEngine(model_, tok, EngineConfig(max_num_seqs=1, max_model_len=min(8192, cfg.ctx_train or 8192)))
    spk = Speaker.load(full(options["speaker"])) if options.get("speaker", "").endswith(".json") else None
    if audio_path and spk is None:
        opts = dict(options)
        if opts.get("whisper") and not opts["whisper"].startswith("synthetic:"):
            opts["whisper"] = full(opts["whisper"])
        spk = speaker_from_audio(full(audio_path), codec, wt, opts, device)
    return OuteTTS(eng, tok, codec, version, spk)


def speaker_from_audio(path: str, codec, wt_path: str, options: dict, device) -> Speaker:
    """AudioPath speaker cloning (reference transformers/backend.py:235-241 `interface.create_speaker`): the
    clip at the codec's rate through the WavTokenizer encoder; the transcript from `speaker_text:` or, with
    `whisper:<model>`, this framework's Whisper (segment timestamps)."""
    from ..utils.audio import load_audio
    from .wavtokenizer import WavTokenizerEncoder, load_wavtokenizer_encoder, synthetic_encoder_state
    sr = codec.cfg.sample_rate
    if wt_path:
        enc = load_wavtokenizer_encoder(wt_path, codec.codebook.detach(), device)
    else:  # synthetic codec: an encoder of the same geometry
        enc = WavTokenizerEncoder(synthetic_encoder_state(codec.cfg), codec.codebook.detach(), device)
    audio = load_audio(path, sr)
    segments = None
    text = options.get("speaker_text", "")
    if not text and options.get("whisper"):
        from .whisper import Transcriber, load_whisper
        wm, wtok = load_whisper(options["whisper"], device)
        _, segs, _ = Transcriber(wm, wtok).transcribe(load_audio(path, 16000))
        segments = [(sg.start, sg.end, sg.text) for sg in segs]
    if not text and not segments:
        raise ValueError("OuteTTS speaker from AudioPath needs its transcript: option speaker_text:<text>, or "
                         "whisper:<model> to transcribe it")
    return create_speaker(enc, audio, sr, sr / codec.cfg.hop, text, segments)
