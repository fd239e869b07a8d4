"""Speech synthesis realtime factors on MI355X (synthetic weights of the real architectures):

* Kokoro-82M (StyleTTS 2 + iSTFTNet, `models/kokoro.py`): ALBERT on the repo GEMM + flash attention, BiLSTMs on the
  cooperative LSTM kernel, convolutions on conv.hip (f16 operands), iSTFT;
* VITS base (piper-medium / MMS-TTS sized, `models/tts.py`): HiFi-GAN on conv.hip, text encoder / flows / duration
  predictor convs as fp32 im2col GEMMs.

RTF here = seconds of audio produced per wall second (higher is better), after one warm-up utterance.

    python tools/bench_tts.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TEXT = ("The quick brown fox jumps over the lazy dog while the morning sun rises slowly over the quiet hills, "
        "and somewhere far away a train whistles as it crosses the old iron bridge.")


def _time(fn, n=3):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(n):
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    return best, out


def main():
    from localai_tfp_amd.models import kokoro as KK
    from localai_tfp_amd.models import tts as T
    c = KK.KOKORO_V019
    m = KK.Kokoro(c, KK.synthetic_params(c, 0), "cuda")
    toks = KK.tokenize(KK.phonemize(TEXT))
    ref = torch.randn(1, 2 * c.style, generator=torch.Generator().manual_seed(1))
    dt, wav = _time(lambda: m.synthesize(toks, ref, seed=1))
    secs = len(wav) / KK.SAMPLE_RATE
    print(json.dumps({"model": "kokoro-82m (synthetic)", "tokens": len(toks), "audio_s": round(secs, 2),
                      "wall_s": round(dt, 3), "realtime_factor": round(secs / dt, 1)}), flush=True)
    for name in ("vits-base",):
        vm, tok = T.load_vits(f"synthetic:{name}", "cuda")
        ids = tok.encode(TEXT) if hasattr(tok, "encode") else tok(TEXT)
        dt, wav = _time(lambda: vm.synthesize(ids, noise_scale=0.667, noise_scale_duration=0.8))
        secs = len(wav) / vm.cfg.sample_rate
        print(json.dumps({"model": f"{name} (synthetic, piper-medium sized)", "tokens": len(ids),
                          "audio_s": round(secs, 2), "wall_s": round(dt, 3), "realtime_factor": round(secs / dt, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
