#!/usr/bin/env python3
"""Sweep the warp-specialised qmm (qmm_ws.hip) against the monolithic qmm at the Llama-3-8B serving shapes.

    python tools/tune_qmm_ws.py --shapes gate_up,qkv --M 128,256 > gpurun_out/ws.jsonl

One JSON line per (shape, M): the monolithic kernel's auto config time, every qmm_ws config / split-K time,
max relative error of each against the monolithic output (same f16 operands, fp32 accumulation).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHAPES = {"qkv": (6144, 4096, 12, 0), "wo": (4096, 4096, 12, 2), "gate_up": (28672, 4096, 12, 3),
          "down": (4096, 14336, 12, 2), "down_q6": (4096, 14336, 14, 2), "lm_head": (128256, 4096, 14, 0)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="qkv,wo,gate_up,down")
    ap.add_argument("--M", default="128,256,384")
    ap.add_argument("--cfgs", default="")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dbg", default="", help="isolation flag sets, e.g. 1,2,3,4,8 (1 no MFMA, 2 no dequant, 4 no A loads, 8 no W loads)")
    a = ap.parse_args()
    from localai_tfp_amd.ops import linear as L
    from localai_tfp_amd.ops.quant import random_quantized
    cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else list(L.QMM_WS_CONFIGS)
    for sh in a.shapes.split(","):
        N, K, qt, epi = SHAPES[sh]
        W = L.QWeight.from_ggml(random_quantized(np.random.default_rng(1), qt, N, K), qt, N, K, "cuda", t32=True)
        assert W.to_t32()
        for M in (int(m) for m in a.M.split(",")):
            x = (torch.randn(M, K, device="cuda") * 0.5).half()
            mk = (lambda: torch.empty(M, N // 2, device="cuda", dtype=torch.float16)) if epi == 3 else \
                (lambda: torch.zeros(M, N, device="cuda"))
            L.QMM_WS_FORCE = None
            ref = mk()
            L.qmatmul(W, x, epi, ref, out_zeroed=True)
            torch.cuda.synchronize()
            out = mk()
            base_us = timeit(lambda: L.qmatmul(W, x, epi, out, out_zeroed=True), a.iters)
            rec = {"shape": sh, "M": M, "qmm_us": round(base_us, 2), "qmm_cfg": L._qmm_shape(M, N, K, epi == 2),
                   "ws": []}
            refn = ref.float().abs().max().item() + 1e-9
            for cfg in cfgs:
                bm, bn = L.qmm_ws_geom(cfg)
                tiles = -(-M // bm) * -(-N // bn)
                for splits in ((1, 2, 4, 8) if epi == 2 else (1,)):
                    if splits > 1 and tiles * splits > 4 * L.CU_COUNT:
                        continue
                    L.QMM_WS_FORCE = (cfg, splits)
                    o = mk()
                    try:
                        L.qmatmul(W, x, epi, o, out_zeroed=True)
                        torch.cuda.synchronize()
                    except Exception as e:  # config not valid for this format
                        rec["ws"].append({"cfg": cfg, "splits": splits, "err": str(e)[:80]})
                        continue
                    err = ((o.float() - ref.float()).abs().max().item()) / refn
                    o2 = mk()
                    us = timeit(lambda: L.qmatmul(W, x, epi, o2, out_zeroed=True), a.iters)
                    rec["ws"].append({"cfg": cfg, "splits": splits, "us": round(us, 2), "rel_err": float(f"{err:.2e}"),
                                      "tflops": round(2 * M * N * K / us / 1e6, 1)})
                    if a.dbg and splits == 1:
                        from localai_tfp_amd import _native as NN
                        for fl in (int(f) for f in a.dbg.split(",")):
                            NN.kcall("mxk_qmm_ws_dbg", fl)
                            rec["ws"][-1][f"dbg{fl}_us"] = round(timeit(lambda: L.qmatmul(W, x, epi, o2, out_zeroed=True), a.iters), 2)
                        NN.kcall("mxk_qmm_ws_dbg", 0)
            L.QMM_WS_FORCE = None
            ok = [w for w in rec["ws"] if "us" in w]
            if ok:
                best = min(ok, key=lambda w: w["us"])
                rec["best"] = best
                rec["speedup"] = round(base_us / best["us"], 3)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
