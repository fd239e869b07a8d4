"""OuteTTS behind the transformers backend's TTS RPC (backend/python/transformers/backend.py:205-243,
509-531): LoadModel with `type: OuteTTS` (options version:, tokenizer:, speaker:<profile.json>,
wavtokenizer:<checkpoint>), TTS -> 24 kHz 16-bit WAV in `dst`, at most the model's max tokens of codes."""
from __future__ import annotations

import logging

from ..grpc import pb
from ..grpc.server import BackendServicer

log = logging.getLogger("localai_tfp_amd.workers.outetts")


class OuteTTSServicer(BackendServicer):
    locking = True

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.tts = None
        self.max_tokens = 4096

    def LoadModel(self, request, context):
        import torch
        from ..models.outetts import load_outetts
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            opts = {}
            for kv in request.Options:
                k, _, v = kv.partition(":")
                opts[k.strip()] = v.strip()
            model = request.Model or request.ModelFile
            if model and not model.startswith("synthetic:") and not model.startswith("/") and request.ModelPath:
                import os
                model = os.path.join(request.ModelPath, model)
            self.tts = load_outetts(model, self.device, opts, request.AudioPath, request.ModelPath)
            return pb.Result(message="loaded OuteTTS", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def TTS(self, request, context):
        from ..utils.audio import write_wav
        if self.tts is None:
            return pb.Result(message="model not loaded", success=False)
        try:
            wav = self.tts.synthesize(request.text, self.max_tokens)
            write_wav(request.dst, wav, self.tts.sample_rate)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("TTS failed")
            return pb.Result(message=f"tts failed: {ex}", success=False)

    def SoundGeneration(self, request, context):
        return pb.Result(message="OuteTTS serves speech (TTS), not sound generation", success=False)
