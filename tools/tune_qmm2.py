#!/usr/bin/env python3
"""qmm2.hip sweep on the Llama-3-8B projections: every compiled (wm, ks) x split choice against the
round-3 qmm.hip default and hipBLASLt on a dense f16 copy of the same weights, all in ONE process,
interleaved, on the same random data. Every qmm2 configuration is checked against the fp32 product of the
dequantised weights (rel. Frobenius error) so a fast-but-wrong tile cannot win. One JSON line per (shape, M).

    MS=128,256 SHAPES=gate_up,down python tools/tune_qmm2.py > gpurun_out/tune_qmm2.jsonl
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
    rounds = int(os.environ.get("ROUNDS", "3"))

    def bench(fn, it=20):
        for _ in range(2):
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
        dense = Wt.dequant_gpu(torch.float16)
        can_split = epi in (L.EPI_F32, L.EPI_ADD_F32)
        for M in Ms:
            x = (torch.randn(M, K, device=dev) * 0.5).half()
            if epi == L.EPI_SWIGLU:
                out = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
            else:
                out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            yref = x.float() @ dense.float().t()
            if epi == L.EPI_SWIGLU:
                v = yref.reshape(M, N // 32, 2, 16)
                ref = (torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1]).reshape(M, N // 2)
            else:
                ref = yref

            def err():
                if epi == L.EPI_ADD_F32:
                    out.zero_()
                elif epi == L.EPI_F32:
                    out.zero_()
                L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                torch.cuda.synchronize()
                return float((out.float() - ref).norm() / ref.norm())

            cands = {}

            def run_old():
                L.QMM2, L.GEMM_POLICY = False, "r3"
                L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                L.QMM2, L.GEMM_POLICY = True, "auto"

            def run_policy():
                L.QMM2 = False
                L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                L.QMM2 = True

            cands["qmm_r3"] = run_old
            cands["policy"] = run_policy
            L.QMM2 = False
            errs["policy"] = round(err(), 6)
            pol = L._gemm_pick(M, N, K, int(qt), can_split)
            L.QMM2 = True
            if epi == L.EPI_SWIGLU:
                cands["dense_f16"] = lambda: L._dense_cached(_DW(dense), x, epi, out, M)
            elif epi == L.EPI_ADD_F32:
                cands["dense_f16"] = lambda: torch.addmm(out, x, dense.t(), out_dtype=torch.float32, out=out)
            else:
                cands["dense_f16"] = lambda: torch.mm(x, dense.t(), out_dtype=torch.float32, out=out)
            L.QMM2_FORCE = None
            auto = L._qmm2_shape(M, N, K, can_split)
            if full:
                cfgs = [(*c, sp) for c in L.QMM2_CONFIGS for sp in ((1, 2, 4, 8) if can_split else (1,))]
            else:  # every tile shape whose row tile is not more than twice M, at the auto split count
                cfgs = [(*c, auto[3]) for c in L.QMM2_CONFIGS if 32 * c[0] * c[2] <= 2 * M and (*c, auto[3]) != auto]
            errs = {}
            for cfg in [auto] + cfgs:
                L.QMM2_FORCE = cfg
                e = err()
                errs[str(list(cfg))] = round(e, 6)

                def mk(c):
                    def f():
                        L.QMM2_FORCE = c
                        L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                    return f
                cands["qmm2" + str(list(cfg))] = mk(cfg)
            # qmm3 (warp-specialised) row tiles, each at the split count qmm3's heuristic gives that tile
            for wm3 in (1, 2, 4):
                if wm3 > 1 and 64 * wm3 > 2 * M:
                    continue
                tiles3 = -(-M // (64 * wm3)) * -(-N // 128)
                sp3 = 1
                while can_split and tiles3 * sp3 < 3 * L.CU_COUNT // 4 and (K // 256) // (sp3 * 2) >= 2:
                    sp3 *= 2
                L.QMM3, L.QMM3_FORCE = True, (wm3, sp3)
                errs[f"q3[{wm3},{sp3}]"] = round(err(), 6)
                L.QMM3 = False

                def mk3(c):
                    def f():
                        L.QMM3, L.QMM3_FORCE = True, c
                        L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                        L.QMM3 = False
                    return f
                cands[f"qmm3[{wm3}, {sp3}]"] = mk3((wm3, sp3))
            from localai_tfp_amd import _native as Nn
            xp = torch.empty(M, K + 64, device=dev, dtype=torch.float16)[:, :K]
            xp.copy_(x)

            def run_rot():
                L.QMM2_FORCE = auto
                Nn.kcall("mxk_qmm2_set_rot", 7)
                L.qmatmul(Wt, x, epi, out, out_zeroed=True)
                Nn.kcall("mxk_qmm2_set_rot", 0)

            def run_pad():
                L.QMM2_FORCE = auto
                L.qmatmul(Wt, xp, epi, out, out_zeroed=True)

            cands["qmm2_rot"] = run_rot
            cands["qmm2_pad"] = run_pad
            # correctness of the rotated order
            Nn.kcall("mxk_qmm2_set_rot", 7)
            L.QMM2_FORCE = auto
            errs["rot"] = round(err(), 6)
            Nn.kcall("mxk_qmm2_set_rot", 0)
            L.QMM2_FORCE = None
            times = {k: [] for k in cands}
            for _ in range(rounds):
                for k, f in cands.items():
                    times[k].append(bench(f))
            res = {"shape": name, "M": M, "auto": list(auto)}
            med = {k: float(np.median(v)) for k, v in times.items()}
            res["qmm_r3_us"] = round(med.pop("qmm_r3"), 2)
            res["policy"] = [str(pol), round(med.pop("policy"), 2)]
            res["dense_f16_us"] = round(med.pop("dense_f16"), 2)
            res["qmm2_auto_us"] = round(med["qmm2" + str(list(auto))], 2)
            res["qmm2_rot_us"] = round(med.pop("qmm2_rot"), 2)
            res["qmm2_padlda_us"] = round(med.pop("qmm2_pad"), 2)
            q3 = {k: v for k, v in med.items() if k.startswith("qmm3")}
            if q3:
                b3 = min(q3, key=q3.get)
                res["qmm3_best"] = [b3[4:], round(q3[b3], 2)]
                for k in q3:
                    med.pop(k)
                res["qmm3_all"] = {k[4:]: round(v, 2) for k, v in q3.items()}
            best = min(med, key=med.get)
            res["qmm2_best"] = [best[4:], round(med[best], 2)]
            flops = 2.0 * M * N * K
            res["qmm2_auto_tflops"] = round(flops / (res["qmm2_auto_us"] * 1e-6) / 1e12, 1)
            res["max_rel_err"] = max(errs.values())
            res["auto_rel_err"] = errs[str(list(auto))]
            if os.environ.get("VERBOSE"):
                res["all"] = {k[4:]: round(v, 2) for k, v in med.items()}
            print(json.dumps(res), flush=True)


class _DW:
    def __init__(self, dense):
        self.bf16_cache = dense
        self.N = dense.shape[0]


if __name__ == "__main__":
    main()
