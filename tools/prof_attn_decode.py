"""Where the batch-1 decode attention spends its time: the 16-wave single-pass kernel's debug instantiation stamps
wall-clock phases of workgroup 0 / wave 0 (attention.hip mxk_attn_decode_ts). Llama-3-8B shapes (Hq 32, Hkv 8,
D 128, paged bf16 cache, block 16), one sequence of --ctx keys.

    python tools/prof_attn_decode.py --ctx 300 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_tfp_amd import _native as N  # noqa: E402

PHASES = ["entry", "seq-len check", "block table in LDS", "first K tile landed", "tiles done", "merge barrier 1",
          "merge barrier 2", "output stored"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=300)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    Hq, Hkv, D, bs, B = 32, 8, 128, 16, 1
    nblk = a.ctx // bs + 2
    kc = (torch.randn(nblk + 1, Hkv, bs, D, device=dev) * 0.5).to(torch.bfloat16)
    vc = torch.randn(nblk + 1, Hkv, bs, D, device=dev).to(torch.bfloat16)
    bt = torch.zeros(B, 256, dtype=torch.int32, device=dev)
    bt[0, :nblk] = torch.randperm(nblk, device=dev).to(torch.int32) + 1
    lens = torch.full((B,), a.ctx, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq * D, device=dev).to(torch.bfloat16)
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    ts = torch.zeros(8, dtype=torch.int64, device=dev)
    N.ensure_act(torch.bfloat16)
    rows = []
    for i in range(a.iters):
        ts.zero_()
        N.kcall("mxk_attn_decode_ts", q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(), bt.data_ptr(),
                bt.stride(0), lens.data_ptr(), B, Hq, Hkv, bs, D ** -0.5, 512, out.data_ptr(), out.stride(0),
                ts.data_ptr(), N.stream_ptr())
        torch.cuda.synchronize()
        t = ts.cpu().tolist()
        rows.append([(t[k] - t[0]) * 0.01 for k in range(8)])  # 100 MHz ticks -> us
    rows = rows[2:]
    for k, name in enumerate(PHASES):
        v = sorted(r[k] for r in rows)
        print(f"{name:22s} median {v[len(v) // 2]:7.2f} us   min {v[0]:7.2f}")


if __name__ == "__main__":
    main()
