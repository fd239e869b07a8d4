"""RWKV-6 precapture in a FRESH process (nothing ran before): which lazy init breaks it?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _model, _ref_logits, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

mode = sys.argv[1]
if mode == "rocblas":
    torch.backends.cuda.preferred_blas_library("cublas")
model, src = _model("cuda:0", seed=6)
if mode == "prime_mm":
    a = torch.randn(8, 256, device="cuda:0", dtype=torch.float16)
    (a @ a.t()).sum().item()
    torch.bmm(a.view(1, 8, 256), a.view(1, 256, 8)).sum().item()
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
refs = [int(_ref_logits(model.cfg, src, p)[-1].argmax()) for p in prompts]
eng = _engine(model, use_graphs=True)
eng.precapture_graphs()
hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in prompts]
eng.run_until_done()
got = [_tokens(h) for h in hs]
print(mode, "ref", refs, "got", got, "OK" if [g[0] for g in got] == refs else "WRONG", flush=True)
