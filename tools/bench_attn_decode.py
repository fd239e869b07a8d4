"""Decode attention microbenchmark: the split-K VALU decode kernel (attention.hip attn_decode) vs the
MFMA flash kernel (attn_prefill) driven with one query row per sequence, on Llama-3-8B shapes
(Hq 32, Hkv 8, D 128, paged bf16 cache, block 16). Prints us per call and GB/s of KV streamed.

    python tools/bench_attn_decode.py [--batch 128] [--ctx 256,512,2048]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_tfp_amd.ops import core as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--ctx", default="256,512,2048")
    ap.add_argument("--part", type=int, default=256, help="decode split-K partition size")
    a = ap.parse_args()
    dev = "cuda"
    Hq, Hkv, D, bs = 32, 8, 128, 16
    for ctx in [int(x) for x in a.ctx.split(",")]:
        B = a.batch
        nb = B * (ctx // bs + 1) + 1
        kc = (torch.randn(nb, Hkv, bs, D, device=dev) * 0.5).to(torch.bfloat16)
        vc = torch.randn(nb, Hkv, bs, D, device=dev).to(torch.bfloat16)
        mb = ctx // bs + 1
        bt = torch.arange(1, 1 + B * mb, dtype=torch.int32, device=dev).view(B, mb)
        lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        q = torch.randn(B, Hq, D, device=dev).to(torch.bfloat16)
        o1 = torch.empty(B, Hq * D, dtype=torch.float16, device=dev)
        o2 = torch.empty_like(o1)
        cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
        scale = D ** -0.5
        npart = -(-ctx // a.part)
        ml = torch.empty(B * Hq * npart, 2, device=dev)
        po = torch.empty(B * Hq * npart, D, device=dev)

        def dec():
            K.attn_decode(q, kc, vc, bt, lens, scale, o1.view(B, Hq, D), part_size=a.part, max_seq_len=ctx,
                          workspace=(ml, po))

        def pf():
            K.attn_prefill(q, kc, vc, bt, cu, lens, scale, o2.view(B, Hq, D), [1] * B, [ctx] * B)
        res = {}
        for name, fn in (("decode", dec), ("prefill1", pf)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            n = 50
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / n * 1e6
            gbs = B * ctx * Hkv * D * 2 * 2 / (us * 1e-6) / 1e9
            res[name] = us
            print(f"ctx={ctx} B={B} {name}: {us:.1f} us  {gbs:.0f} GB/s")
        err = float((o1.float() - o2.float()).abs().max())
        print(f"ctx={ctx} max|decode - prefill1| = {err:.2e}  speedup {res['decode'] / res['prefill1']:.2f}x")


if __name__ == "__main__":
    main()
