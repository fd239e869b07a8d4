"""Text-to-speech worker: the reference's `piper` (backend/go/tts/piper.go:20-49) and the transformers
backend's VITS / MMS-TTS path behind the TTS RPC, served by the VITS engine (models/tts.py) on the GPU.
The reference's `coqui` backend (backend/python/coqui/backend.py:26-80) is routed here too: Coqui VITS
model directories (config.json + model_file.pth, models/coqui.py), found by path or by Coqui model name
("tts_models/en/vctk/vits") in the models directory or Coqui's local cache. Coqui XTTS-v2 directories load
models/xtts.py: voice cloning from the LoadModel AudioPath clip (speaker_wav) or a named speaker (`voice`,
speakers_xtts.pth); `language` is required, as the reference requires it for multi-lingual models.
Bark, Kokoro and MusicGen have workers of their own.

LoadModel: a piper voice (`<voice>.onnx` + `<voice>.onnx.json`, models/piper.py; espeak-ng data from
LibrarySearchPath or the `espeak_data` option), a Coqui VITS directory, a Hugging Face VITS directory
(MMS-TTS layout) or `synthetic:vits-test | vits-base`.
ModelOptions.Options ("key:value"): noise_scale, noise_scale_duration (alias noise_w), speaking_rate
(alias length_scale = 1 / rate), seed.
TTS: text -> 16-bit PCM WAV at the model's sample rate in `dst`. `voice` selects the speaker of a
multi-speaker model (an integer id, or a Coqui speaker name such as "p225"; piper's per-voice .onnx file selection has no equivalent because
voices are separate checkpoints here — configure one model per voice). `language` is accepted and
ignored like piper does.
SoundGeneration (ElevenLabs /v1/sound-generation) is a MusicGen feature in the reference
(backend/python/transformers/backend.py:452-507); a speech model does not generate sound effects, so
this worker reports it unsupported.
"""
from __future__ import annotations

import logging
import os

import numpy as np

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.tts")


class TTSServicer(BackendServicer):
    locking = True  # base.SingleThread in the reference backends

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.model = None
        self.tok = None
        self.opts: dict = {}
        self.speakers: dict = {}
        self.xtts = None  # models/xtts.Xtts when the model directory holds a Coqui XTTS checkpoint
        self.xtts_voice = None  # (GPT conditioning latents, speaker embedding) of LoadModel's AudioPath clip

    def LoadModel(self, request, context):
        import torch
        from ..models import tts as T
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            path = request.ModelFile or request.Model
            if not path.startswith("synthetic:") and not os.path.isabs(path) and request.ModelPath:
                path = os.path.join(request.ModelPath, path)
            o = {}
            for kv in request.Options:
                k, _, v = kv.partition(":")
                o[k.strip()] = v.strip()
            self.opts = o
            if not path.startswith("synthetic:") and os.path.isfile(path) and path.endswith(".onnx"):
                # piper voice: <voice>.onnx + <voice>.onnx.json (models/piper.py)
                from ..models.piper import load_piper
                self.model, self.tok = load_piper(path, self.device,
                                                  o.get("espeak_data", "") or request.LibrarySearchPath)
                return pb.Result(message=f"loaded piper voice {os.path.basename(path)}", success=True)
            from ..models import coqui as CQ
            cdir = None if path.startswith("synthetic:") else CQ.resolve_model_dir(request.Model or path, request.ModelPath)
            if cdir is None and not path.startswith("synthetic:") and CQ.is_coqui_dir(
                    path if os.path.isdir(path) else os.path.dirname(path)):
                cdir = path if os.path.isdir(path) else os.path.dirname(path)
            if cdir is not None and CQ.is_coqui_dir(cdir):
                from ..models import xtts as XT
                if XT.is_xtts_dir(cdir):
                    # Coqui XTTS-v2: voice cloning from AudioPath (speaker_wav) or a named speaker; the reference
                    # clip is conditioned once here (backend/python/coqui/backend.py:40-47, 77-80)
                    self.xtts = XT.load_xtts(cdir, self.device)
                    self.model = self.xtts
                    if request.AudioPath:
                        ap = request.AudioPath if os.path.isabs(request.AudioPath) else os.path.join(
                            request.ModelPath, request.AudioPath)
                        self.xtts_voice = self.xtts.voice(audio_path=ap)
                    return pb.Result(message=f"loaded Coqui XTTS {os.path.basename(os.path.normpath(cdir))}",
                                     success=True)
                self.model, self.tok, self.speakers = CQ.load_coqui(
                    cdir, self.device, o.get("espeak_data", "") or request.LibrarySearchPath)
                return pb.Result(message=f"loaded Coqui VITS {os.path.basename(os.path.normpath(cdir))}", success=True)
            if os.environ.get("MX_BACKEND_NAME") == "coqui" and not path.startswith("synthetic:") and not os.path.exists(path):
                return pb.Result(success=False, message=(
                    f"Coqui model {request.Model!r} not found locally (looked in the models directory and the Coqui "
                    "cache $TTS_HOME/tts, ~/.local/share/tts); this build does not download models"))
            if not path.startswith("synthetic:") and os.path.isfile(path):
                path = os.path.dirname(path)
            self.model, self.tok = T.load_vits(path, self.device)
            return pb.Result(message=f"loaded {self.model.cfg.name}", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def _synth(self, text: str, voice: str = "") -> np.ndarray:
        o = self.opts
        rate = float(o["speaking_rate"]) if "speaking_rate" in o else (
            1.0 / float(o["length_scale"]) if "length_scale" in o else None)
        nsd = o.get("noise_scale_duration", o.get("noise_w"))
        spk = int(voice) if voice and voice.strip().lstrip("-").isdigit() else None
        if spk is None and voice and self.speakers:
            if voice not in self.speakers:
                raise ValueError(f"unknown speaker {voice!r} (known: {', '.join(sorted(self.speakers)[:8])} ...)")
            spk = self.speakers[voice]
        ids = self.tok.encode(text)
        if len(ids) <= 1:
            raise ValueError("no speakable characters in the input text")
        return self.model.synthesize(ids, speaker=spk, speaking_rate=rate,
                                     noise_scale=float(o["noise_scale"]) if "noise_scale" in o else None,
                                     noise_scale_duration=float(nsd) if nsd is not None else None,
                                     seed=int(o.get("seed", 0)))

    def _synth_xtts(self, request) -> np.ndarray:
        """XTTS: the reference's rules — a multi-lingual model needs `language` (or COQUI_LANGUAGE); a named
        `voice` wins over the AudioPath clip (backend/python/coqui/backend.py:66-80)."""
        lang = request.language or os.environ.get("COQUI_LANGUAGE", "")
        if not lang:
            raise ValueError("Model is multi-lingual, but no language was provided")
        if request.voice:
            voice = self.xtts.voice(speaker=request.voice)
        elif self.xtts_voice is not None:
            voice = self.xtts_voice
        else:
            raise ValueError("Model is multi-speaker, but no speaker was provided (voice, or AudioPath at load)")
        mx = self.opts.get("max_new")
        return self.xtts.synthesize(request.text, lang, voice=voice, seed=int(self.opts.get("seed", 0)),
                                    max_new=int(mx) if mx else None)

    def TTS(self, request, context):
        from ..utils.audio import write_wav
        if self.model is None:
            return pb.Result(message="model not loaded", success=False)
        try:
            if self.xtts is not None:
                write_wav(request.dst, self._synth_xtts(request), self.xtts.sample_rate)
                return pb.Result(message="ok", success=True)
            wav = self._synth(request.text, request.voice)
            write_wav(request.dst, wav, self.model.cfg.sample_rate)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("TTS failed")
            return pb.Result(message=f"tts failed: {ex}", success=False)

    def SoundGeneration(self, request, context):
        return pb.Result(message="sound generation needs a MusicGen model; this TTS backend serves speech "
                                 "(VITS) only", success=False)


def main(argv=None):
    worker_main(TTSServicer, argv)


if __name__ == "__main__":
    main()
