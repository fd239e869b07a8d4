#!/usr/bin/env python3
"""Time the GPU sampler (reference settings: temp 0.9 / top-k 40 / top-p 0.95) at a batch size, row kernel vs
split-vocabulary kernel, and check both draw the same tokens.   python tools/time_sampler.py --B 128"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--trace", action="store_true", help="print tk_slice_kernel phase stamps (workgroup 0)")
    a = ap.parse_args()
    from localai_tfp_amd.ops.sampling import SamplerBatch, SamplingParams
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B, V = a.B, 128256
    logits = torch.randn(B, V, device=dev) * 2.0
    ps = [SamplingParams(temperature=0.9, top_k=40, top_p=0.95, seed=10 + r) for r in range(B)]
    hist = [[] for _ in range(B)]
    row, split = SamplerBatch(dev), SamplerBatch(dev)
    row.SPLIT_MAX_B, split.SPLIT_MAX_B = 0, 1 << 20
    res = {}
    for name, smp in (("row", row), ("split", split)):
        toks = []
        for it in range(3):
            toks.append(smp.sample(logits.clone(), ps, hist, [it] * B)[0].cpu())
        lg = [logits.clone() for _ in range(a.iters)]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for it in range(a.iters):
            smp.sample(lg[it], ps, hist, [it] * B)
        e1.record()
        torch.cuda.synchronize()
        res[name] = (e0.elapsed_time(e1) / a.iters * 1e3, toks)
    same = all(torch.equal(x, y) for x, y in zip(res["row"][1], res["split"][1]))
    print(f"B={B} row {res['row'][0]:.1f} us/call  split {res['split'][0]:.1f} us/call  same_tokens={same}")
    if a.trace:
        import ctypes
        import numpy as np
        from localai_tfp_amd import _native as Nn
        Nn.kcall("mxk_sample_trace", 1, 0)
        split.sample(logits.clone(), ps, hist, [0] * B)
        torch.cuda.synchronize()
        ts = np.zeros(16, np.uint64)
        Nn.kcall("mxk_sample_trace", 0, ts.ctypes.data)
        Nn.kcall("mxk_sample_trace", 0, 0)
        d = np.diff(ts[:5].astype(np.int64)) * 10  # 100 MHz ticks -> ns
        print("tk_slice phases (ns): load+max", d[0], "pass1+scan", d[1], "pass2+scan", d[2], "compact", d[3])


if __name__ == "__main__":
    main()
