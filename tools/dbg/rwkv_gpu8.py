"""RWKV-6 read-before-write hunt: NaN-fill one engine buffer at a time (workspace / state), run eager."""
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


def run(fill=None, graphs=False):
    eng = _engine(model, use_graphs=graphs)
    if fill:
        obj, name = fill
        t = getattr(eng.ws if obj == "ws" else eng.kv, name)
        if t.is_floating_point():
            t.fill_(float("nan"))
        else:
            t.fill_(-7)
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in prompts]
    eng.run_until_done()
    return [_tokens(h) for h in hs]


ref = run()
print("ref", ref, flush=True)
eng0 = _engine(model)
names = [("ws", k) for k, v in vars(eng0.ws).items() if isinstance(v, torch.Tensor)]
names += [("kv", k) for k, v in vars(eng0.kv).items() if isinstance(v, torch.Tensor)]
del eng0
for nm in names:
    got = run(nm)
    print(nm, "OK" if got == ref else f"WRONG {got}", flush=True)
