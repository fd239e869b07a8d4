"""Speech-to-text worker: the reference's `whisper` (whisper.cpp) and `faster-whisper` backends
(backend/go/transcribe/whisper/whisper.go:28-105, backend/python/faster-whisper/backend.py:26-62).

LoadModel accepts a whisper.cpp ggml file, a Hugging Face whisper directory/safetensors, or
`synthetic:whisper-<size>`. Model `options` (ModelOptions.Options, "key:value"):
  beam_size:N         beam search width (faster-whisper uses 5; default greedy like whisper.cpp)
  temperatures:a,b,.. fallback schedule (default 0,0.2,...,1.0)
  condition_on_previous_text:true|false
  initial_prompt:<text>
AudioTranscription: audio decoded natively (WAV) or through ffmpeg, resampled to 16 kHz; returns
segments with start/end in nanoseconds (the Go binding's time.Duration, whisper.go:83-101) and
the concatenated text.
"""
from __future__ import annotations

import logging
import os

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.whisper")


class WhisperServicer(BackendServicer):
    locking = True  # one transcription at a time per GPU context (base.SingleThread in the reference)

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.tr = None
        self.opts = None

    def LoadModel(self, request, context):
        import torch
        from ..models import whisper as W
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            path = request.ModelFile or request.Model
            if not path.startswith("synthetic:") and not os.path.isabs(path) and request.ModelPath:
                path = os.path.join(request.ModelPath, path)
            model, tok = W.load_whisper(path, self.device)
            self.tr = W.Transcriber(model, tok)
            o = W.DecodeOptions()
            for kv in request.Options:
                k, _, v = kv.partition(":")
                k = k.strip()
                if k == "beam_size":
                    o.beam_size = int(v)
                elif k == "temperatures":
                    o.temperatures = tuple(float(x) for x in v.split(",") if x.strip())
                elif k == "condition_on_previous_text":
                    o.condition_on_previous_text = v.strip().lower() in ("1", "true", "yes")
                elif k == "initial_prompt":
                    o.initial_prompt = v
                elif k == "no_timestamps":
                    o.timestamps = v.strip().lower() not in ("1", "true", "yes")
            self.opts = o
            return pb.Result(message=f"loaded {model.cfg.name}", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def AudioTranscription(self, request, context):
        from dataclasses import replace

        from ..utils.audio import load_audio
        if self.tr is None:
            raise RuntimeError("model not loaded")
        audio = load_audio(request.dst)
        opt = replace(self.opts, language=request.language or None,
                      task="translate" if request.translate else "transcribe")
        text, segs, _lang = self.tr.transcribe(audio, opt)
        out = [pb.TranscriptSegment(id=s.id, start=int(round(s.start * 1e9)), end=int(round(s.end * 1e9)),
                                    text=s.text, tokens=s.tokens) for s in segs]
        return pb.TranscriptResult(segments=out, text=text)


def main(argv=None):
    worker_main(WhisperServicer, argv)


if __name__ == "__main__":
    main()
