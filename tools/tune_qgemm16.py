#!/usr/bin/env python3
"""Sweep qgemm16 tile shapes / split-K for the Llama-3-8B decode projections (MI355X)."""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from localai_tfp_amd import _build, _native as N
    _build.build_all()
    from localai_tfp_amd.formats.gguf import QType
    from localai_tfp_amd.ops import linear as L
    from localai_tfp_amd.ops.quant import random_quantized
    dev = torch.device("cuda")
    shapes = [("qkv", 6144, 4096, QType.Q4_K, 2), ("wo", 4096, 4096, QType.Q4_K, 2),
              ("gate_up", 28672, 4096, QType.Q4_K, 3), ("down", 4096, 14336, QType.Q6_K, 2),
              ("lm_head", 128256, 4096, QType.Q6_K, 0)]
    for name, n, k, qt, epi in shapes:
        W = L.QWeight.from_ggml(random_quantized(np.random.default_rng(1), int(qt), n, k), int(qt), n, k, dev)
        for M in [int(m) for m in os.environ.get("MS", "64,128,256").split(",")]:
            x = torch.randn(M, k, device=dev).half()
            out = (torch.empty(M, n // 2, device=dev, dtype=torch.float16) if epi == 3
                   else torch.zeros(M, n, device=dev))
            res = []
            for wm, wn, sp in itertools.product([2, 4, 8], [1, 2, 4], [1, 2, 4, 8]):
                if epi in (0, 3) and sp > 1:
                    continue
                if epi == 3 and wn == 1:
                    continue
                if (wm, wn) not in [(1, 2), (2, 2), (4, 2), (8, 2), (4, 4), (2, 4), (4, 1), (8, 1)]:
                    continue
                args = (int(W.qtype), epi, wm, wn, x.data_ptr(), x.stride(0), W.data.data_ptr(), N.ptr(W.dplane),
                        M, n, k, sp, out.data_ptr(), out.stride(0), N.stream_ptr())
                try:
                    for _ in range(3):
                        N.kcall("mxk_qgemm16", *args)
                except Exception:
                    continue
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(30):
                    N.kcall("mxk_qgemm16", *args)
                e1.record()
                torch.cuda.synchronize()
                res.append((round(e0.elapsed_time(e1) / 30 * 1e3, 2), wm, wn, sp))
            res.sort()
            print(json.dumps({"shape": name, "M": M, "best": res[:4], "worst": res[-1]}), flush=True)


if __name__ == "__main__":
    main()
