#!/usr/bin/env python3
"""Time of the default K-quant GEMM dispatch (ops/linear.py qmatmul) against M on the Llama-3-8B projections,
for several row-chunk settings (ROW_CHUNKS, 0 = one launch) — the curve the scheduler's step composition and the
row-chunk policy are chosen from. Every setting is checked against the fp32 product. One JSON line per (shape, M).

    MS=128,256,384 ROW_CHUNKS=0,256 python tools/gemm_curve.py > gpurun_out/gemm_curve.jsonl
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
              ("down_q6", 4096, 14336, QType.Q6_K, L.EPI_ADD_F32)]
    only = os.environ.get("SHAPES")
    if only:
        shapes = [s for s in shapes if s[0] in only.split(",")]
    Ms = [int(m) for m in os.environ.get("MS", "128,192,256,320,384,512").split(",")]
    chunks = [int(c) for c in os.environ.get("ROW_CHUNKS", "0,256").split(",")]
    it = int(os.environ.get("ITERS", "30"))

    def bench(fn):
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
        Wt = L.QWeight.from_ggml(raw, int(qt), N, K, dev)
        assert Wt.to_t32()
        dense = Wt.dequant_gpu(torch.float16).float()
        for M in Ms:
            x = (torch.randn(M, K, device=dev) * 0.5).half()
            if epi == L.EPI_SWIGLU:
                out = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
            else:
                out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            yref = x.float() @ dense.t()
            if epi == L.EPI_SWIGLU:
                v = yref.reshape(M, N // 32, 2, 16)
                ref = (torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1]).reshape(M, N // 2)
            else:
                ref = yref
            rec = {"shape": name, "M": M, "N": N, "K": K, "gflop": round(2 * M * N * K / 1e9, 2)}
            for c in chunks:
                L.ROW_CHUNK = c
                out.zero_()
                L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                torch.cuda.synchronize()
                err = float((out.float() - ref).norm() / ref.norm())
                us = bench(lambda: L.qmatmul(Wt, x, epi, out, out_zeroed=True))
                rec[f"chunk{c}_us"] = round(us, 2)
                rec[f"chunk{c}_err"] = round(err, 6)
                rec[f"chunk{c}_tflops"] = round(2 * M * N * K / us / 1e6, 1)
            print(json.dumps(rec), flush=True)
        del Wt, dense


if __name__ == "__main__":
    main()
