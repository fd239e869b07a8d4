#!/usr/bin/env python3
"""int8-MFMA qmm8.hip configurations x split-K on the Llama-3-8B projections (Q8_K activations), each checked
against the fp32 product of the dequantised operands, next to the f16 qmm.hip default and the dense f16
hipBLASLt path. One JSON line per (shape, M, config) ("kind": "cfg") and one summary per (shape, M).

    MS=128,256,384,2048 python tools/tune_qmm8.py > gpurun_out/tune_qmm8.jsonl
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
    from localai_tfp_amd.ops import core as K
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
    sweep = os.environ.get("SWEEP", "1") == "1"

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

    for name, N, Kd, qt, epi in shapes:
        raw = random_quantized(np.random.default_rng(1), int(qt), N, Kd)
        Wt = L.QWeight.from_ggml(raw, int(qt), N, Kd, dev)
        wf = Wt.dequant_gpu(torch.float32)
        assert Wt.to_t32()
        can_split = epi in (L.EPI_F32, L.EPI_ADD_F32)
        for M in Ms:
            x = torch.randn(M, Kd, device=dev) * 0.5
            a = K.Q8KAct.empty(M, Kd, dev)
            K.quant_q8k(x, a)
            y = a.dequant() @ wf.t()
            xh = x.half()
            if epi == L.EPI_SWIGLU:
                v = y.reshape(M, N // 32, 2, 16)
                ref = (F.silu(v[:, :, 0]) * v[:, :, 1]).reshape(M, N // 2)
                out = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
            else:
                ref = y
                out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            res = {"kind": "shape", "shape": name, "M": M}
            res["q8_auto_cfg"] = list(L._qmm8_shape(M, N, Kd, can_split))
            res["q8_auto_us"] = round(bench(lambda: L.qmatmul8(Wt, a, epi, out, out_zeroed=True)), 2)
            res["quant_us"] = round(bench(lambda: K.quant_q8k(x, a)), 2)
            res["f16_qmm_us"] = round(bench(lambda: L.qmatmul(Wt, xh, epi, out, out_zeroed=True)), 2)
            best = None
            for c in (L.QMM8_CONFIGS if sweep else ()):
                for sp in ((1, 2, 4) if can_split else (1,)):
                    L.QMM8_FORCE = (*c, sp)
                    try:
                        out.zero_()
                        L.qmatmul8(Wt, a, epi, out, out_zeroed=True)
                        torch.cuda.synchronize()
                    except Exception as ex:
                        L.QMM8_FORCE = None
                        print(json.dumps({"kind": "cfg", "shape": name, "M": M, "cfg": [*c, sp], "error": str(ex)[:80]}))
                        continue
                    err = float((out.float() - ref).norm() / ref.norm())
                    us = bench(lambda: L.qmatmul8(Wt, a, epi, out, out_zeroed=True))
                    L.QMM8_FORCE = None
                    print(json.dumps({"kind": "cfg", "shape": name, "M": M, "cfg": [*c, sp], "us": round(us, 2),
                                      "tops": round(2 * M * N * Kd / us / 1e6, 1), "rel_err": round(err, 6)}), flush=True)
                    if err < 1e-3 and (best is None or us < best[0]):
                        best = (us, [*c, sp])
            if best:
                res["q8_best_us"], res["q8_best_cfg"] = round(best[0], 2), best[1]
                res["q8_best_tops"] = round(2 * M * N * Kd / best[0] / 1e6, 1)
            wd = wf.half()
            res["dense_us"] = round(bench(lambda: torch.matmul(xh, wd.t())), 2)
            del wd
            print(json.dumps(res), flush=True)
        del wf


if __name__ == "__main__":
    main()
