"""attn_decode microbenchmark at the headline serving shape (B=128, Llama-3-8B heads, contexts
256..512, graph-style max_seq_len 4096) over partition sizes."""
import json
import sys

import torch

from localai_tfp_amd.ops import core as K

dev = torch.device("cuda:0")
B, Hq, Hkv, D, bs = 128, 32, 8, 128, 16
maxlen = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = torch.Generator().manual_seed(0)
lens = torch.randint(256, 513, (B,), generator=g, dtype=torch.int32)
maxb = maxlen // bs
nblocks = B * maxb + 1
kc = torch.randn(nblocks, Hkv, bs, D, dtype=torch.bfloat16, device=dev)
vc = torch.randn(nblocks, Hkv, bs, D, dtype=torch.bfloat16, device=dev)
perm = torch.randperm(B * maxb, generator=g).int() + 1
bt = perm.view(B, maxb).to(dev)
q = torch.randn(B, Hq, D, dtype=torch.bfloat16, device=dev)
sl = lens.to(dev)
out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=dev)
bytes_ = int(lens.sum()) * Hkv * D * 2 * 2
res = {"B": B, "max_len": maxlen, "mean_ctx": float(lens.float().mean()), "kv_mb": bytes_ / 1e6}
ref = None
for impl, part in (("valu", 256), ("mfma", 256), ("mfma", 512), ("mfma", 1024), ("mfma", 2048)):
    n_parts = -(-maxlen // part)
    ws = (torch.empty(B * Hq * n_parts, 2, device=dev), torch.empty(B * Hq * n_parts, D, device=dev))
    for _ in range(3):
        K.attn_decode(q, kc, vc, bt, sl, D ** -0.5, out, part_size=part, workspace=ws, max_seq_len=maxlen, impl=impl)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        K.attn_decode(q, kc, vc, bt, sl, D ** -0.5, out, part_size=part, workspace=ws, max_seq_len=maxlen, impl=impl)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    if ref is None:
        ref = out.float().clone()
    err = float((out.float() - ref).abs().max())
    res[f"{impl}{part}"] = {"us": round(us, 1), "TBps": round(bytes_ / us / 1e6, 2), "max_diff_vs_256": err}
print(json.dumps(res))
