"""qmm on MX4F weights with structured data (debug): per config, rel error vs fp32 and the pattern of errors."""
import numpy as np
import torch
from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import linear as L
from localai_tfp_amd.ops import quant as Q
from localai_tfp_amd.ops.linear import EPI_F32, QWeight, qmatmul

def rel(a, b):
    return float((a.float().cpu() - b).norm() / b.norm())

n, k = 64, 512
rng = np.random.default_rng(0)
for qt in (QType.Q4_0, QType.Q4_1, QType.Q5_1):
    raw = Q.random_quantized(rng, int(qt), n, k)
    dense = torch.from_numpy(Q.dequantize(raw, qt, (k, n)).copy())
    W = QWeight.from_ggml(raw, int(qt), n, k, "cuda", t32=True)
    W.to_t32()
    for cfg in ((1, 1, 4, 1, 1), (2, 1, 4, 1, 1), (2, 2, 4, 1, 1)):
        L.QMM_FORCE = cfg
        for M in (32, 64):
            x = torch.zeros(M, k)
            x[:, :] = 0
            for i in range(M):
                x[i, (i * 7) % k] = 1.0  # selects one weight column element per row
            ref = x @ dense.t()
            out = torch.zeros(M, n, device="cuda")
            qmatmul(W, x.half().cuda(), EPI_F32, out)
            o = out.cpu()
            err = rel(out, ref)
            print(qt.name, cfg, M, "rel", round(err, 4))
            if err > 1e-2:
                bad = (o - ref).abs() > 1e-3 * ref.abs().max()
                r, c = bad.nonzero()[0].tolist()
                kk = (r * 7) % k
                print("  first bad row", r, "col", c, "k", kk, "got", float(o[r, c]), "want", float(ref[r, c]),
                      "cands:", [round(float(dense[c, j]), 5) for j in range(max(0, kk - 2), kk + 3)],
                      "matching k:", [j for j in range(k) if abs(float(dense[c, j]) - float(o[r, c])) < 1e-4][:6])
