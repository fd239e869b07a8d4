"""Kokoro TTS worker (the reference's `kokoro` backend, backend/python/kokoro/backend.py:47-99).

LoadModel: `ModelFile` = the Kokoro .pth checkpoint (weights-only load; `synthetic:kokoro-test` for tests),
option `voice:<name>` (required, as in the reference) or `voice:<a>+<b>` (the two packs averaged) naming
`<ModelPath>/<voice>.pt`; `speed:<x>` and `seed:<n>` options. TTS: phonemise (models/kokoro.py), pick the
voice-pack row for the phoneme count, synthesise, write a 24 kHz 16-bit WAV to `dst`.
"""
from __future__ import annotations

import logging
import os

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.kokoro")


class KokoroServicer(BackendServicer):
    locking = True

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.model = None
        self.voice = None
        self.opts: dict = {}

    def LoadModel(self, request, context):
        import torch
        from ..models import kokoro as KK
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            o = {}
            for kv in request.Options:
                k, _, v = kv.partition(":")
                o[k.strip()] = v.strip()
            self.opts = o
            if not o.get("voice"):
                return pb.Result(message="No voice specified in options (voice:<name>)", success=False)
            path = request.ModelFile or request.Model
            if path.startswith("synthetic:"):
                cfg = KK.KOKORO_TEST if path.endswith("test") else KK.KOKORO_V019
                params = KK.synthetic_params(cfg, 0)
            else:
                if not os.path.isabs(path) and request.ModelPath:
                    path = os.path.join(request.ModelPath, path)
                params = KK.load_checkpoint(path)
                cfg = KK.config_for(params)
            self.model = KK.Kokoro(cfg, params, self.device)
            self.voice = KK.load_voice(request.ModelPath or os.path.dirname(path), o["voice"], self.device)
            return pb.Result(message=f"Model loaded successfully (voice {o['voice']})", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def TTS(self, request, context):
        from ..models import kokoro as KK
        from ..utils.audio import write_wav
        if self.model is None:
            return pb.Result(message="model not loaded", success=False)
        try:
            lang = "b" if self.opts.get("voice", "").startswith("b") else "a"
            toks = KK.tokenize(KK.phonemize(request.text, lang))
            if not toks:
                raise ValueError("no speakable characters in the input text")
            toks = toks[:510]
            ref = self.voice[len(toks)]
            wav = self.model.synthesize(toks, ref, float(self.opts.get("speed", 1.0)), int(self.opts.get("seed", 0)))
            write_wav(request.dst, wav, KK.SAMPLE_RATE)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("TTS failed")
            return pb.Result(message=f"tts failed: {ex}", success=False)


def main(argv=None):
    worker_main(KokoroServicer, argv)


if __name__ == "__main__":
    main()
