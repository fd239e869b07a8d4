"""Whisper transcription benchmark (BASELINE config #4: whisper-base /v1/audio/transcriptions, 1 GPU).

Random-init whisper-base weights (no checkpoint download), synthetic audio. Reports the front end,
encoder and hipGraph decoder-step latencies and the end-to-end real-time factor of `transcribe`
(decoding forced to a fixed token budget per 30 s window so random weights give a stable workload).

    python tools/bench_whisper.py --model whisper-base --seconds 120 --tokens 128
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="whisper-base")
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--tokens", type=int, default=128, help="decoded tokens per 30 s window")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--beam", type=int, default=0)
    a = ap.parse_args()
    from localai_tfp_amd.models import whisper as W
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    model, tok = W.load_whisper("synthetic:" + a.model, dev)
    tr = W.Transcriber(model, tok)
    rng = np.random.default_rng(0)
    audio = (0.1 * rng.standard_normal(int(a.seconds * W.SAMPLE_RATE))).astype(np.float32)

    def sync():
        if dev != "cpu":
            torch.cuda.synchronize()

    def timeit(fn, n):
        fn()
        sync()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        sync()
        return (time.perf_counter() - t) / n * 1e3

    res = {"model": a.model, "device": torch.cuda.get_device_name(0) if dev != "cpu" else "cpu"}
    res["logmel_ms_per_30s"] = timeit(lambda: model.log_mel(audio[:W.N_SAMPLES]), a.iters)
    mel = model.log_mel(audio[:W.N_SAMPLES])[:, :W.N_FRAMES][None]
    res["encoder_ms"] = timeit(lambda: model.encode(mel), a.iters)
    mel4 = mel.repeat(4, 1, 1)
    res["encoder_ms_batch4"] = timeit(lambda: model.encode(mel4), max(1, a.iters // 2))
    xa = model.encode(mel)
    st = model.new_state(1)
    st.set_audio(xa)
    model.decode_prefix(st, [tok.sot_sequence("en")])
    t1 = torch.tensor([tok.timestamp_begin], device=dev)

    def step():
        if st.pos >= st.cap - 1:
            st.pos = 3
        model.decode_step(st, t1)
    res["decoder_step_ms"] = timeit(step, 200)

    # end-to-end: fixed token budget per window (no eot), greedy with timestamp rules
    eot = tok.eot
    orig = tr._apply_rules

    def rules(logits, sampled, opt, first):
        lg = orig(logits, sampled, opt, first)
        if len(sampled) < a.tokens - 1:
            lg[eot] = -np.inf
        if not np.isfinite(lg).any():
            lg[tok.timestamp_begin] = 0.0
        return lg
    tr._apply_rules = rules
    opt = W.DecodeOptions(language="en", temperatures=(0.0,), sample_len=a.tokens, beam_size=a.beam)
    tr.transcribe(audio[:W.N_SAMPLES], opt)  # warm
    sync()
    t = time.perf_counter()
    text, segs, _ = tr.transcribe(audio, opt)
    sync()
    dt = time.perf_counter() - t
    res.update({"audio_s": a.seconds, "wall_s": round(dt, 3), "rtf": round(dt / a.seconds, 5),
                "x_realtime": round(a.seconds / dt, 1), "segments": len(segs), "tokens_per_window": a.tokens,
                "beam": a.beam})
    for k, v in list(res.items()):
        if isinstance(v, float):
            res[k] = round(v, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
