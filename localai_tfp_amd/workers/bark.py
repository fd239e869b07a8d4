"""Bark TTS worker: the reference's ``bark`` (suno bark, backend/python/bark/backend.py:32-56) and
``bark-cpp`` (backend/go/bark/gobark.cpp:22-80) backends, served by models/bark.py on the GPU.

LoadModel: a Hugging Face Bark directory (config.json + safetensors + BERT tokenizer files, optional
``speaker_embeddings/``), or ``synthetic:bark-small`` / ``synthetic:bark-test`` (random-init weights).
ModelOptions.Options ("key:value"): text_temp (0.7), waveform_temp (0.7), min_eos_p (0.05),
max_semantic_tokens (768), seed.
TTS: ``voice`` is a speaker preset — a ``.npz`` path, ``<name>.npz`` in the model's ``speaker_embeddings/``
directory, or the Hugging Face split layout ``speaker_embeddings/<name>_{semantic,coarse,fine}_prompt.npy``
(all loaded with allow_pickle=False); empty = no history prompt. Output: 24 kHz 16-bit WAV in ``dst``.
"""
from __future__ import annotations

import logging
import os

import numpy as np

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.bark")


class BarkServicer(BackendServicer):
    locking = True

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.model = None
        self.opts: dict = {}
        self.root = ""

    def LoadModel(self, request, context):
        import torch
        from ..models import bark as BK
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            path = request.ModelFile or request.Model
            if path.startswith("synthetic:"):
                self.model = BK.synthetic_bark(path.split(":", 1)[1], self.device)
            else:
                if not os.path.isabs(path) and request.ModelPath:
                    path = os.path.join(request.ModelPath, path)
                if os.path.isfile(path):
                    path = os.path.dirname(path)
                self.model = BK.load_bark(path, self.device)
                self.root = path
            self.opts = {}
            for kv in request.Options:
                k, _, v = kv.partition(":")
                self.opts[k.strip()] = v.strip()
            return pb.Result(message="loaded bark", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def _voice(self, voice: str):
        from ..models.bark import load_voice
        if not voice:
            return None
        cands = [voice, os.path.join(self.root, "speaker_embeddings", voice + ".npz"),
                 os.path.join(self.root, voice + ".npz")]
        for c in cands:
            if c and os.path.isfile(c):
                return load_voice(c)
        d = os.path.join(self.root, "speaker_embeddings")
        parts = {k: os.path.join(d, f"{voice}_{k}.npy") for k in ("semantic_prompt", "coarse_prompt", "fine_prompt")}
        if all(os.path.isfile(p) for p in parts.values()):
            return {k: np.load(p, allow_pickle=False) for k, p in parts.items()}
        raise FileNotFoundError(f"Bark voice preset {voice!r} not found (tried {cands[1]} and the split .npy layout)")

    def TTS(self, request, context):
        from ..utils.audio import write_wav
        if self.model is None:
            return pb.Result(message="model not loaded", success=False)
        try:
            o = self.opts
            m = self.model
            wav = m.generate(m.tokenize(request.text), history=self._voice(request.voice),
                             text_temp=float(o.get("text_temp", 0.7)) or None,
                             waveform_temp=float(o.get("waveform_temp", 0.7)) or None,
                             seed=int(o["seed"]) if "seed" in o else None,
                             min_eos_p=float(o.get("min_eos_p", 0.05)),
                             max_semantic=int(o.get("max_semantic_tokens", 768)))
            write_wav(request.dst, wav, m.g.sample_rate)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("TTS failed")
            return pb.Result(message=f"tts failed: {ex}", success=False)


def main(argv=None):
    worker_main(BarkServicer, argv)
