"""RWKV-6 precapture corruption: hipBLASLt (dense F32->f16 weights through torch.matmul) or not?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.models import rwkv as RW  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

mode = sys.argv[1]
if mode == "rocblas":
    torch.backends.cuda.preferred_blas_library("cublas")
qt = "Q8_0" if mode == "q8" else "F32"
cfg = RW.tiny_rwkv_config()
src = RW.synthetic_rwkv_source(cfg, seed=6, qtype=qt)
model = RW.RwkvModel.load(cfg, src, "cuda:0")
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
res = {}
for pre in (False, True):
    eng = _engine(model, use_graphs=True)
    if pre:
        eng.precapture_graphs()
    calls = []
    orig = model.forward

    def fwd(fb, st, ws, _o=orig):
        out = _o(fb, st, ws)
        if len(calls) < 1:
            calls.append(out.float().clone())
        return out
    model.forward = fwd
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in prompts]
    eng.run_until_done()
    model.forward = orig
    res[pre] = calls[0]
    print(mode, "precapture" if pre else "lazy", [_tokens(h) for h in hs], flush=True)
print(mode, "first-forward max diff", float((res[True] - res[False]).abs().max()), flush=True)
