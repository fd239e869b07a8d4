#!/usr/bin/env python3
"""Run one qmm configuration in a loop (for rocprofv3 --pmc passes / kernel traces).

    python tools/prof_qmm.py --shape gate_up --M 2048 --cfg 4,2,8,1 --iters 20
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHAPES = {"qkv": (6144, 4096, 12, 0), "wo": (4096, 4096, 12, 2), "gate_up": (28672, 4096, 12, 3), "gate_up_f32": (28672, 4096, 12, 2),
          "down": (4096, 14336, 12, 2), "down_q6": (4096, 14336, 14, 2), "lm_head": (128256, 4096, 14, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="gate_up")
    ap.add_argument("--M", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--gemv", action="store_true", help="M <= 4 decode GEMV with the fused RMSNorm / q8 prologue")
    ap.add_argument("--q2", default="", help="qmm2 wm,ks,wn,splits")
    ap.add_argument("--qmv1", type=int, default=1, help="0: disable the batch-1 fast-prologue GEMV (qmv1_kernel)")
    ap.add_argument("--q3dbg", default="", help="qmm3 isolation build dbg,wm (Q4_K SwiGLU only)")
    ap.add_argument("--q2dbg", default="", help="qmm2 isolation build dbg,wm,ks,wn (Q4_K SwiGLU only)")
    ap.add_argument("--qt", type=int, default=0, help="ggml type override (e.g. 3 = Q4_1 -> MX4F t32)")
    a = ap.parse_args()
    from localai_tfp_amd.ops import linear as L
    from localai_tfp_amd.ops.quant import random_quantized
    N, K, qt, epi = SHAPES[a.shape]
    qt = a.qt or qt
    W = L.QWeight.from_ggml(random_quantized(np.random.default_rng(1), qt, N, K), qt, N, K, "cuda", t32=True)
    assert W.to_t32()
    if a.q2:
        L.QMM2, L.QMM2_FORCE = True, tuple(int(v) for v in a.q2.split(","))
    from localai_tfp_amd import _native as Nq
    Nq.kcall("mxk_qmv1_enable", a.qmv1)
    x = (torch.randn(a.M, K, device="cuda") * 0.5).half()
    out = (torch.empty(a.M, N // 2, device="cuda", dtype=torch.float16) if epi == 3
           else torch.zeros(a.M, N, device="cuda"))
    if a.gemv:  # h fp32 residual rows -> rmsnorm -> q8 -> qmv, one launch
        h = torch.randn(a.M, K, device="cuda")
        nw = torch.ones(K, device="cuda")
        call = (lambda: L.qmv_fused(W, h, epi, out, norm=nw, eps=1e-5, out_zeroed=True)) if K == 4096 else \
            (lambda: L.qmv_fused(W, x, epi, out, out_zeroed=True))
        assert call()
    elif a.q3dbg:
        from localai_tfp_amd import _native as Nn
        dbg, wm = (int(v) for v in a.q3dbg.split(","))
        Nn.ensure_act(torch.float16)

        def call():
            Nn.kcall("mxk_qmm3_dbg", dbg, wm, x.data_ptr(), x.stride(0), W.data.data_ptr(), a.M, N, K, out.data_ptr(),
                     out.stride(0), Nn.stream_ptr())
    elif a.q2dbg:
        from localai_tfp_amd import _native as Nn
        dbg, wm, ks, wn = (int(v) for v in a.q2dbg.split(","))
        Nn.ensure_act(torch.float16)

        def call():
            Nn.kcall("mxk_qmm2_dbg", dbg, wm, ks, wn, x.data_ptr(), x.stride(0), W.data.data_ptr(), a.M, N, K, out.data_ptr(),
                     out.stride(0), Nn.stream_ptr())
    else:
        def call():
            L.qmatmul(W, x, epi, out, out_zeroed=True)
    for _ in range(a.iters):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    cfg = ("qmv_fused" if a.gemv else f"q2dbg {a.q2dbg}" if a.q2dbg else f"q3dbg {a.q3dbg}" if a.q3dbg else
           f"qmm2 {L._qmm2_shape(a.M, N, K, epi in (0, 2))}" if a.q2 else L._gemm_pick(a.M, N, K, qt, epi in (0, 2)))
    print(f"{a.shape} qt={int(W.qtype)} M={a.M} cfg={cfg} {us:.1f} us {2*a.M*N*K/us/1e6:.0f} TF {W.data.numel() / us / 1e6:.2f} TB/s weights")


if __name__ == "__main__":
    main()
