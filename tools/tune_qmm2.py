#!/usr/bin/env python3
"""Every compiled qmm.hip configuration x split-K on the Llama-3-8B projections, each checked against an
fp32 reference of the same quantised weights (SwiGLU epilogue included), against the dense f16 hipBLASLt
path. One JSON line per (shape, M, config) with "kind": "cfg", and one summary line per (shape, M).

    MS=128,256,384,2048 SHAPES=gate_up,down python tools/tune_qmm2.py > gpurun_out/tune_qmm2.jsonl
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
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
    Ms = [int(m) for m in os.environ.get("MS", "128,256,384,2048").split(",")]
    cfg_filter = os.environ.get("CFGS")  # e.g. "2.2.2.33,4.2.2.33"
    cfgs_all = list(L.QMM_CONFIGS)
    if cfg_filter:
        cfgs_all = [tuple(int(v) for v in c.split(".")) for c in cfg_filter.split(",")]

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
        Wt = L.QWeight.from_ggml(raw, int(qt), N, K, dev)
        wf = Wt.dequant_gpu(torch.float32)  # ggml-layout dequant (the oracle) before tiling
        assert Wt.to_t32()
        can_split = epi in (L.EPI_F32, L.EPI_ADD_F32)
        for M in Ms:
            x = (torch.randn(M, K, device=dev) * 0.5).half()
            y = x.float() @ wf.t()
            if epi == L.EPI_SWIGLU:
                v = y.reshape(M, N // 32, 2, 16)
                ref = (F.silu(v[:, :, 0]) * v[:, :, 1]).reshape(M, N // 2)
                out = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
            else:
                ref = y
                out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            res = {"kind": "shape", "shape": name, "M": M}
            res["auto_cfg"] = list(L._qmm_shape(M, N, K, can_split))
            res["auto_us"] = round(bench(lambda: L.qmatmul(Wt, x, epi, out, out_zeroed=True)), 2)
            best = None
            for c in cfgs_all:
                for sp in ((1, 2, 4) if can_split else (1,)):
                    L.QMM_FORCE = (*c, sp)
                    try:
                        out.zero_()
                        L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                        torch.cuda.synchronize()
                    except Exception as ex:  # configuration not compiled / does not fit this format
                        L.QMM_FORCE = None
                        print(json.dumps({"kind": "cfg", "shape": name, "M": M, "cfg": [*c, sp], "error": str(ex)[:80]}))
                        continue
                    err = float((out.float() - ref).norm() / ref.norm())
                    us = bench(lambda: L.qmatmul(Wt, x, epi, out, out_zeroed=True))
                    L.QMM_FORCE = None
                    print(json.dumps({"kind": "cfg", "shape": name, "M": M, "cfg": [*c, sp], "us": round(us, 2),
                                      "tflops": round(2 * M * N * K / us / 1e6, 1), "rel_err": round(err, 5)}), flush=True)
                    if err < 2e-2 and (best is None or us < best[0]):
                        best = (us, [*c, sp])
            if best:
                res["best_us"], res["best_cfg"] = round(best[0], 2), best[1]
                res["best_tflops"] = round(2 * M * N * K / best[0] / 1e6, 1)
            cache = Wt.dequant_gpu(torch.float16) if False else None
            wd = wf.half()
            if epi == L.EPI_SWIGLU:
                fn = lambda: torch.matmul(x, wd.t())
            else:
                fn = lambda: torch.addmm(out, x, wd.t(), out_dtype=torch.float32, out=out) if epi == L.EPI_ADD_F32 \
                    else torch.mm(x, wd.t(), out_dtype=torch.float32, out=out)
            try:
                res["dense_us"] = round(bench(fn), 2)
            except Exception:
                res["dense_us"] = round(bench(lambda: torch.matmul(x, wd.t())), 2)
            del wd
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
