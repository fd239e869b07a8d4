"""Audio generation timings on MI355X: MusicGen-small (synthetic weights) seconds of audio per second and
per-step decode latency (hipGraph vs eager), Bark-small (synthetic) end-to-end.

    python tools/bench_audio.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from localai_tfp_amd.models import bark as BK
    from localai_tfp_amd.models import musicgen as MG
    m = MG.synthetic_musicgen("musicgen-small", "cuda")
    ids = m.tokenize("lofi hip hop beat with warm piano")
    for graph in (True, False):
        m.generate_codes(ids, None, 16, 3.0, True, seed=0, use_graph=graph)
        torch.cuda.synchronize()
        t = time.perf_counter()
        codes = m.generate_codes(ids, None, 256, 3.0, True, seed=0, use_graph=graph)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        t2 = time.perf_counter()
        wav = m.decode_audio(codes)
        torch.cuda.synchronize()
        dec = time.perf_counter() - t2
        secs = wav.shape[-1] / m.sample_rate
        print(json.dumps({"model": "musicgen-small (synthetic)", "hipgraph": graph, "tokens": 256,
                          "gen_s": round(dt, 3), "ms_per_step": round(dt / 256 * 1e3, 2),
                          "encodec_decode_s": round(dec, 3), "audio_s": round(secs, 2),
                          "realtime_factor": round(secs / (dt + dec), 2)}), flush=True)
    b = BK.synthetic_bark("bark-small", "cuda")
    b.generate(b.tokenize("warm up"), seed=0, max_semantic=8)
    torch.cuda.synchronize()
    t = time.perf_counter()
    wav = b.generate(b.tokenize("Hello, this is a test of the bark model."), seed=0, max_semantic=200)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"model": "bark-small (synthetic)", "semantic_tokens": 200, "total_s": round(dt, 3),
                      "audio_s": round(wav.size / 24000, 2), "realtime_factor": round(wav.size / 24000 / dt, 2)}))


if __name__ == "__main__":
    main()
