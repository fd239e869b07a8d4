#!/usr/bin/env python3
"""Tile / split-K sweep of qgemm32.hip vs qgemm16.hip vs the dense f16 hipBLASLt path on the
Llama-3-8B decode projections (one JSON line per (shape, M) with the best config of each path)."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from localai_tfp_amd import _build
    _build.build_all()
    from localai_tfp_amd.formats.gguf import QType
    from localai_tfp_amd.ops import linear as L
    from localai_tfp_amd.ops.quant import random_quantized
    dev = torch.device("cuda")
    shapes = [("qkv", 6144, 4096, QType.Q4_K, L.EPI_F32), ("wo", 4096, 4096, QType.Q4_K, L.EPI_ADD_F32),
              ("gate_up", 28672, 4096, QType.Q4_K, L.EPI_SWIGLU), ("down", 4096, 14336, QType.Q4_K, L.EPI_ADD_F32),
              ("down_q6", 4096, 14336, QType.Q6_K, L.EPI_ADD_F32), ("lm_head", 128256, 4096, QType.Q6_K, L.EPI_F32)]
    Ms = [int(m) for m in os.environ.get("MS", "64,128,256").split(",")]

    def bench(fn, it=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / it * 1e3

    for name, N, K, qt, epi in shapes:
        raw = random_quantized(np.random.default_rng(1), int(qt), N, K)
        W = L.QWeight.from_ggml(raw, int(qt), N, K, dev)
        cache = W.build_bf16_cache(torch.float16)
        for M in Ms:
            x = torch.randn(M, K, device=dev).half()
            if epi == L.EPI_SWIGLU:
                out = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
            else:
                out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            res = {"shape": name, "M": M}
            W.bf16_cache = None
            L.BF16_CACHE_MIN_M = 10**9
            L.Q32_MIN_M = 10**9
            res["q16_us"] = round(bench(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True)), 2)
            L.Q32_MIN_M = 1
            best = None
            for wm in (2, 4):
                for wn in (1, 2):
                    for sp in ((1, 2, 4, 8) if epi in (L.EPI_F32, L.EPI_ADD_F32) else (1,)):
                        L.Q32_FORCE = (wm, wn, sp)
                        us = bench(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True))
                        if best is None or us < best[0]:
                            best = (us, wm, sp, wn)
            L.Q32_FORCE = None
            res["q32_auto_us"] = round(bench(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True)), 2)
            res["q32_best_us"], res["q32_wm"], res["q32_splits"], res["q32_wn"] = round(best[0], 2), best[1], best[2], best[3]
            W.bf16_cache = cache
            L.BF16_CACHE_MIN_M = 1
            res["dense_us"] = round(bench(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True)), 2)
            L.BF16_CACHE_MIN_M = None
            wbytes = W.data.numel() + (W.dplane.numel() * 2 if W.dplane is not None else 0)
            res["q32_wTBps"] = round(wbytes / best[0] / 1e6, 2)
            res["q32_tflops"] = round(2 * M * N * K / best[0] / 1e6, 1)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
