#!/usr/bin/env python3
"""Best-plan time of the Llama-3-8B Q4_K_M projections per M under the load-time tuner (ops/autotune.tune_weight),
for the kernel library in use (MX_KERNEL_LIB selects an alternative build): one JSON line per (shape, M) plus a
total, and every tuned plan checked against the fp32 product. Same-box A/B of kernel variants:

    for v in a b; do MX_KERNEL_LIB=jobs/libmxk_$v.so TAG=$v python tools/gemm_ab.py; done
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from localai_tfp_amd.formats.gguf import QType
    from localai_tfp_amd.ops import autotune as AT
    from localai_tfp_amd.ops import linear as L
    from localai_tfp_amd.ops.quant import random_quantized
    dev = torch.device("cuda")
    tag = os.environ.get("TAG", "default")
    ms = tuple(int(v) for v in os.environ.get("MS", "128,256,384,416").split(","))
    shapes = [("qkv", 6144, 4096, QType.Q4_K, L.EPI_F32, True), ("wo", 4096, 4096, QType.Q4_K, L.EPI_ADD_F32, True),
              ("gate_up", 28672, 4096, QType.Q4_K, L.EPI_SWIGLU, False),
              ("down", 4096, 14336, QType.Q4_K, L.EPI_ADD_F32, True),
              ("down_q6", 4096, 14336, QType.Q6_K, L.EPI_ADD_F32, True)]
    total = 0.0
    for name, N, K, qt, epi, split in shapes:
        raw = random_quantized(np.random.default_rng(7), int(qt), N, K)
        W = L.QWeight.from_ggml(raw, int(qt), N, K, dev)
        assert W.to_t32()
        AT.TIMES.clear()
        AT.tune_weight(W, epi, split, ms, iters=int(os.environ.get("ITERS", "20")))
        key = AT._key(N, K, int(qt), epi, split)
        dense = W.dequant_gpu(torch.float16).float()
        for b, plan, us in AT.TIMES.get(key, []):
            x = (torch.randn(b, K, device=dev) * 0.5).half()
            y = x.float() @ dense.t()
            ref = y if epi != L.EPI_SWIGLU else (lambda v: torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1])(
                y.reshape(b, N // 32, 2, 16)).reshape(b, N // 2)
            out = (torch.zeros(b, N // 2, device=dev, dtype=torch.float16) if epi == L.EPI_SWIGLU
                   else torch.zeros(b, N, device=dev, dtype=torch.float32))
            L.qmatmul(W, x, epi, out, out_zeroed=True)
            torch.cuda.synchronize()
            rel = float((out.float() - ref).norm() / ref.norm())
            total += us
            print(json.dumps({"tag": tag, "shape": name, "M": b, "plan": list(plan), "us": us,
                              "tflops": round(2 * b * N * K / us / 1e6, 1), "rel_err": round(rel, 6)}), flush=True)
            assert rel < 3e-3, (name, b, plan, rel)
        AT.TUNED.clear()
    print(json.dumps({"tag": tag, "total_us": round(total, 1)}), flush=True)


if __name__ == "__main__":
    main()
