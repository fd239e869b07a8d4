"""RWKV-6 precapture_graphs corruption: what does capture change?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _model, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

model, src = _model("cuda:0", seed=6)
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]


def wsum(m):
    s = 0.0
    for L in m.layers:
        for k, v in vars(L).items():
            t = getattr(v, "data", v)
            if isinstance(t, torch.Tensor):
                s += float(t.float().abs().sum())
    return s


def run(eng, ps):
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in ps]
    eng.run_until_done()
    return [_tokens(h) for h in hs]


w0 = wsum(model)
for buckets in ((4,), (1,), (2,), (1, 2, 4)):
    eng = _engine(model, use_graphs=True)
    eng.cfg.graph_buckets = buckets
    st0 = [float(t.float().abs().sum()) for t in eng.kv.__dict__.values() if isinstance(t, torch.Tensor)]
    n = eng.precapture_graphs()
    torch.cuda.synchronize()
    st1 = [float(t.float().abs().sum()) for t in eng.kv.__dict__.values() if isinstance(t, torch.Tensor)]
    print("buckets", buckets, "captured", n, "weights changed", wsum(model) != w0, "state", st0, st1, flush=True)
    print("  ", run(eng, prompts), flush=True)
print("kv type", type(eng.kv), [k for k in eng.kv.__dict__], flush=True)
