"""MusicGen sound-generation worker: the reference's ``transformers-musicgen`` backend and the
``transformers`` backend with ``type: MusicgenForConditionalGeneration``
(backend/python/transformers/backend.py:452-507), behind the SoundGeneration RPC that serves
ElevenLabs-style ``/v1/sound-generation`` (core/http/endpoints/elevenlabs/soundgeneration.go).

LoadModel: a Hugging Face MusicGen directory (config.json + safetensors + tokenizer.json / spiece.model),
or ``synthetic:musicgen-small`` / ``synthetic:musicgen-test`` (random-init weights of that architecture,
byte-level stand-in tokenizer) for benchmarks without a network.
SoundGeneration semantics follow the reference: ``duration`` seconds -> int(duration * 51.2) tokens
(default 256 = 5 s), ``temperature`` is the classifier-free guidance scale (default 3.0), ``sample``
toggles sampling (default on, top-k 250), an empty text generates unconditionally, the WAV goes to ``dst``.
TTS on this worker is the same generation with the text as the prompt (the reference's musicgen TTS path).
"""
from __future__ import annotations

import logging
import os

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.musicgen")


class MusicgenServicer(BackendServicer):
    locking = True

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.model = None

    def LoadModel(self, request, context):
        import torch
        from ..models import musicgen as MG
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            path = request.ModelFile or request.Model
            if path.startswith("synthetic:"):
                self.model = MG.synthetic_musicgen(path.split(":", 1)[1], self.device)
            else:
                if not os.path.isabs(path) and request.ModelPath:
                    path = os.path.join(request.ModelPath, path)
                if os.path.isfile(path):
                    path = os.path.dirname(path)
                self.model = MG.load_musicgen(path, self.device)
            return pb.Result(message="loaded musicgen", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def _generate(self, text: str, duration: float | None, guidance: float, sample: bool, dst: str):
        import torch
        from ..utils.audio import write_wav
        m = self.model
        tokens = int(duration * 51.2) if duration else 256
        if text:
            ids = m.tokenize(text)
        else:
            ids = None
        codes = m.generate_codes(ids, None, tokens, guidance if ids is not None else 1.0, sample,
                                 top_k=int(m.generation.get("top_k", 250)) if hasattr(m, "generation") else 250)
        wav = m.decode_audio(codes)[0, 0].float().cpu().numpy()
        torch.cuda.synchronize() if m.device.type == "cuda" else None
        write_wav(dst, wav, m.sample_rate)
        return wav

    def SoundGeneration(self, request, context):
        if self.model is None:
            return pb.Result(message="model not loaded", success=False)
        try:
            duration = request.duration if request.HasField("duration") else None
            guidance = request.temperature if request.HasField("temperature") else 3.0
            sample = request.sample if request.HasField("sample") else True
            self._generate(request.text, duration, guidance, sample, request.dst)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("SoundGeneration failed")
            return pb.Result(message=f"sound generation failed: {ex}", success=False)

    def TTS(self, request, context):
        if self.model is None:
            return pb.Result(message="model not loaded", success=False)
        try:
            self._generate(request.text, None, 3.0, True, request.dst)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("TTS failed")
            return pb.Result(message=f"tts failed: {ex}", success=False)


def main(argv=None):
    worker_main(MusicgenServicer, argv)
