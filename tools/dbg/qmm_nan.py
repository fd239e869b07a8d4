import sys, os, torch, numpy as np
sys.path.insert(0, os.getcwd())
from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import linear as L, quant as Q
from localai_tfp_amd.ops.linear import QWeight, qmatmul, EPI_F32
L.QMM_MIN_M = 1
for qt in (QType.Q8_0, QType.Q6_K):
  for cfg in [(4,2,2),(4,1,1),(2,2,1)]:
    L.QMM_FORCE = cfg
    n,k,M = 416,2304,77
    rng = np.random.default_rng(105)
    x0 = rng.standard_normal((n, k), dtype=np.float32) * 0.05
    raw = Q.QUANTIZERS[qt](x0); dense = torch.from_numpy(Q.dequantize(raw, qt, (k, n)))
    W = QWeight.from_ggml(raw.reshape(n,-1), qt, n, k, "cuda")
    x = torch.randn(M, k, device="cuda").half()
    ref = x.float().cpu() @ dense.t()
    out = torch.full((M, n), 7.0, device="cuda")
    qmatmul(W, x, EPI_F32, out)
    o = out.cpu()
    bad = ~torch.isfinite(o)
    err = (o-ref).abs()
    err[bad] = 0
    print(qt.name, cfg, "nan", int(bad.sum()), "rows", sorted(set(bad.nonzero()[:,0].tolist()))[:10], "cols", sorted(set(bad.nonzero()[:,1].tolist()))[:10], "unwritten", int((o==7.0).sum()), "maxerr", float(err.max()))
