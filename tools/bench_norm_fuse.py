"""Time the qmm2 fused-epilogue instances against the plain ones on Llama-3-8B projection shapes (one MI355X).

    python tools/bench_norm_fuse.py [--m 128]

For each GEMM (o_proj / down as residual-add producers, qkv / gate|up as consumers, qkv with the RoPE epilogue) the
tuned or rule plan is timed plain and fused, same plan; prints one JSON line per case (us per call)."""
import argparse
import json

import numpy as np
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import linear as L
from localai_tfp_amd.ops import quant as Q
from localai_tfp_amd.ops.linear import EPI_ADD_F32, EPI_F32, EPI_SWIGLU, NormFuse, QWeight, qmatmul


def weight(qt, n, k, seed):
    rng = np.random.default_rng(seed)
    raw = Q.QUANTIZERS[QType(qt)](rng.standard_normal((n, k), dtype=np.float32) * 0.05)
    W = QWeight.from_ggml(raw.reshape(n, -1), qt, n, k, "cuda", t32=True)
    assert W.to_t32()
    return W


def timeit(fn, it=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[128, 416])
    args = ap.parse_args()
    H, F, QKV = 4096, 14336, 6144
    Wo, Wd = weight(QType.Q4_K, H, H, 1), weight(QType.Q6_K, H, F, 2)
    Wqkv, Wgu = weight(QType.Q4_K, QKV, H, 3), weight(QType.Q4_K, 2 * F, H, 4)
    for M in args.m:
        xa = torch.randn(M, H, device="cuda").half()
        xf = torch.randn(M, F, device="cuda").half()
        h = torch.randn(M, H, device="cuda")
        xn = torch.empty(M, H, dtype=torch.float16, device="cuda")
        ss = torch.zeros(2, M, 32, device="cuda")
        tick = torch.zeros(-(-M // 32) * (QKV // 32), dtype=torch.int32, device="cuda")
        qkv = torch.zeros(M, QKV, device="cuda")
        act = torch.empty(M, F, dtype=torch.float16, device="cuda")
        q = torch.empty(M, 32 * 128, dtype=torch.bfloat16, device="cuda")
        kc = torch.zeros(64, 8, 16, 128, dtype=torch.bfloat16, device="cuda")
        vc = torch.zeros_like(kc)
        slots = torch.arange(M, dtype=torch.int32, device="cuda") % (64 * 16)
        rot = torch.randn(M, 64, 2, device="cuda")
        prod = lambda W, x: NormFuse(1, ss_out=ss[0], ss_zero=ss[1], gamma=torch.ones(H, device="cuda"), xn=xn,
                                     tick=tick)
        cases = [
            ("o_proj producer", lambda f: qmatmul(Wo, xa, EPI_ADD_F32, h, fuse=prod(Wo, xa) if f else None)),
            ("down producer", lambda f: qmatmul(Wd, xf, EPI_ADD_F32, h, fuse=prod(Wd, xf) if f else None)),
            ("gate_up consumer", lambda f: qmatmul(Wgu, xa, EPI_SWIGLU, act,
                                                   fuse=NormFuse(2, ss_in=ss[0], eps=1e-5) if f else None)),
            ("qkv consumer", lambda f: qmatmul(Wqkv, xa, EPI_F32, qkv, out_zeroed=True,
                                               fuse=NormFuse(2, ss_in=ss[0], eps=1e-5) if f else None)),
            ("qkv rope", lambda f: qmatmul(Wqkv, xa, EPI_F32, qkv, out_zeroed=True, fuse=NormFuse(
                4, tick=tick, rope=(slots, rot, None, q, kc, vc, 0, 128, 32, 8, 16)) if f else None)),
        ]
        for name, fn in cases:
            plain = timeit(lambda: fn(False))
            qkv.zero_()
            fused = timeit(lambda: fn(True))
            qkv.zero_()
            print(json.dumps({"M": M, "case": name, "plain_us": round(plain, 2), "fused_us": round(fused, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
