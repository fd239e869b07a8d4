"""Voice-activity-detection worker: the reference's `silero-vad` backend
(backend/go/vad/silero/vad.go:17-57; gateway endpoint core/http/endpoints/localai/vad.go).

LoadModel: a silero v5 state dict (safetensors / weights-only torch file) or `synthetic:silero-vad`.
ModelOptions.Options ("key:value"): threshold, min_silence_ms, speech_pad_ms (the reference hard-codes
0.5 / 0 / 0). VAD: 16 kHz float samples -> segments with start/end in seconds.
"""
from __future__ import annotations

import logging
import os

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.vad")


class VADServicer(BackendServicer):
    locking = True  # base.SingleThread in the reference

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.model = None
        self.params = None

    def LoadModel(self, request, context):
        import torch
        from ..models import vad as V
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            path = request.ModelFile or request.Model
            if not path.startswith("synthetic:") and not os.path.isabs(path) and request.ModelPath:
                path = os.path.join(request.ModelPath, path)
            self.model = V.SileroVAD.load(path, self.device)
            p = V.VADParams()
            for kv in request.Options:
                k, _, v = kv.partition(":")
                k = k.strip()
                if k == "threshold":
                    p.threshold = float(v)
                elif k == "min_silence_ms":
                    p.min_silence_ms = int(v)
                elif k == "speech_pad_ms":
                    p.speech_pad_ms = int(v)
            self.params = p
            return pb.Result(message="loaded silero-vad", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def VAD(self, request, context):
        if self.model is None:
            raise RuntimeError("model not loaded")
        segs = self.model.detect(list(request.audio), self.params)
        return pb.VADResponse(segments=[pb.VADSegment(start=a, end=b) for a, b in segs])


def main(argv=None):
    worker_main(VADServicer, argv)


if __name__ == "__main__":
    main()
