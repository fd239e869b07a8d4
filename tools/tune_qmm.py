#!/usr/bin/env python3
"""Tile / split-K sweep of qmm.hip against the previous quantised path (qgemm32) and the dense f16
hipBLASLt path on the Llama-3-8B projections; one JSON line per (shape, M). Also checks every qmm
configuration against the dense fp32 result (rel error) so a fast-but-wrong tile cannot win.

    MS=64,128,256,512,2048 python tools/tune_qmm.py > gpurun_out/tune_qmm.jsonl
"""
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
    only = os.environ.get("SHAPES")
    if only:
        shapes = [s for s in shapes if s[0] in only.split(",")]
    Ms = [int(m) for m in os.environ.get("MS", "64,128,256,512,2048").split(",")]
    full = os.environ.get("FULL", "1") == "1"

    def bench(fn, it=20):
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
        W = L.QWeight.from_ggml(raw, int(qt), N, K, dev)   # ggml rows: qgemm32 + dense-cache paths
        Wt = L.QWeight.from_ggml(raw, int(qt), N, K, dev)  # t32 tiles: qmm
        assert Wt.to_t32()
        cache = W.build_bf16_cache(torch.float16)
        can_split = epi in (L.EPI_F32, L.EPI_ADD_F32)
        for M in Ms:
            x = (torch.randn(M, K, device=dev) * 0.5).half()
            if epi == L.EPI_SWIGLU:
                out = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
            else:
                out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            # dense reference (f16 weights, fp32 accumulate)
            ref = (x.float() @ cache.float().t())
            res = {"shape": name, "M": M}
            W.bf16_cache = None
            L.Q32_MIN_M = 1
            res["q32_us"] = round(bench(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True)), 2)
            res["qmm_auto_us"] = round(bench(lambda: L.qmatmul(Wt, x, epi, out, out_zeroed=True)), 2)
            res["qmm_auto_cfg"] = list(L._qmm_shape(M, N, K, can_split))
            best = None
            errs = []
            cfgs = [(*c, sp) for c in L.QMM_CONFIGS for sp in ((1, 2, 4, 8) if can_split else (1,))] if full else []
            for cfg in cfgs:
                L.QMM_FORCE = cfg
                if epi != L.EPI_SWIGLU:
                    out.zero_()
                    L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                    errs.append(float((out - ref).norm() / ref.norm()))
                us = bench(lambda: L.qmatmul(Wt, x, epi, out, out_zeroed=True))
                if best is None or us < best[0]:
                    best = (us, cfg)
            L.QMM_FORCE = None
            if best:
                res["qmm_best_us"], res["qmm_best_cfg"] = round(best[0], 2), list(best[1])
            if errs:
                res["qmm_max_rel_err"] = round(max(errs), 5)
            W.bf16_cache = cache
            L.BF16_CACHE_MIN_M = 1
            res["dense_us"] = round(bench(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True)), 2)
            L.BF16_CACHE_MIN_M = None
            t = min(res["qmm_auto_us"], res.get("qmm_best_us", 1e9))
            res["qmm_tflops"] = round(2 * M * N * K / t / 1e6, 1)
            wbytes = Wt.data.numel()
            res["qmm_wTBps"] = round(wbytes / t / 1e6, 2)
            print(json.dumps(res), flush=True)
        W.bf16_cache = None
        del cache


if __name__ == "__main__":
    main()
