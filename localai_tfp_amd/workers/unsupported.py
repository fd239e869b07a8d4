"""Backend names of the reference whose model families this framework does not implement (Bark is served
by workers/bark.py, MusicGen by workers/musicgen.py, Kokoro by workers/kokoro.py, Coqui VITS by
workers/tts.py, Coqui XTTS-v2 by workers/tts.py + models/xtts.py).

The worker starts and answers Health like any backend (so the process manager's lifecycle is the same),
but LoadModel fails with an explicit error naming the backend — a request for Bark never silently gets
a different speech model."""
from __future__ import annotations

import os

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

SUPPORTED_TTS = "piper / coqui (VITS) / transformers-tts (VITS, MMS-TTS checkpoints, OuteTTS) / kokoro / bark"


class UnsupportedServicer(BackendServicer):
    def __init__(self, device: str | None = None):
        super().__init__()
        self.backend = os.environ.get("MX_BACKEND_NAME", "this backend")

    def LoadModel(self, request, context):
        return pb.Result(success=False, message=(
            f"backend {self.backend!r} is not implemented by this MI355X build (model {request.Model!r}); "
            f"text-to-speech is served by {SUPPORTED_TTS}"))


def main(argv=None):
    worker_main(UnsupportedServicer, argv)
