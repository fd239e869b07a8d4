#!/usr/bin/env python3
"""Micro-benchmark of the decode-shape projections of Llama-3-8B: quantised MFMA kernel vs the bf16
weight-cache hipBLASLt path, per (shape, M). Prints one JSON line per case (µs, effective TB/s of
weight bytes, TFLOP/s)."""
from __future__ import annotations

import json
import os
import sys

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
              ("gate_up", 28672, 4096, QType.Q4_K, L.EPI_SWIGLU), ("down", 4096, 14336, QType.Q6_K, L.EPI_ADD_F32)]
    Ms = [int(m) for m in os.environ.get("MS", "16,32,64,128,256").split(",")]
    for name, N, K, qt, epi in shapes:
        import numpy as np
        raw = random_quantized(np.random.default_rng(1), int(qt), N, K)
        W = L.QWeight.from_ggml(raw, int(qt), N, K, dev)
        caches = {}
        for dt in (torch.bfloat16, torch.float16):
            W.bf16_cache = None
            caches[dt] = W.build_bf16_cache(dt)
        for M in Ms:
            res = {"shape": name, "M": M, "N": N, "K": K}
            for path in ("mfma", "dense", "mfma16", "dense16"):
                dt = torch.float16 if path.endswith("16") else torch.bfloat16
                W.bf16_cache = caches[dt]
                x = torch.randn(M, K, device=dev).to(dt)
                if epi == L.EPI_SWIGLU:
                    out = torch.empty(M, N // 2, device=dev, dtype=dt)
                else:
                    out = torch.zeros(M, N, device=dev, dtype=torch.float32)
                L.BF16_CACHE_MIN_M = 10**9 if path.startswith("mfma") else 1
                for _ in range(3):
                    L.qmatmul(W, x, epi, out, out_zeroed=True)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                it = 50
                e0.record()
                for _ in range(it):
                    L.qmatmul(W, x, epi, out, out_zeroed=True)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / it * 1e3
                wbytes = W.data.numel() * W.data.element_size() + (W.dplane.numel() * 2 if W.dplane is not None else 0)
                res[path + "_us"] = round(us, 2)
                res[path + "_tflops"] = round(2 * M * N * K / us / 1e6, 1)
                if path.startswith("mfma"):
                    res[path + "_wTBps"] = round(wbytes / us / 1e6, 2)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
