"""RWKV-6: eager engine, lazy-graph engine, then a precapture engine in one process (reproduces the wrong
tokens). Variants: gc.collect() between engines / empty_cache / keep the old engines alive."""
import gc
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _model, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

mode = sys.argv[1]
model, src = _model("cuda:0", seed=6)
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
keep = []
for step in ("eager", "graphs", "precapture"):
    eng = _engine(model, use_graphs=step != "eager")
    if step == "precapture":
        eng.precapture_graphs()
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in prompts]
    eng.run_until_done()
    print(mode, step, [_tokens(h) for h in hs], flush=True)
    if mode == "keep":
        keep.append(eng)
    del eng, hs
    if mode in ("gc", "gc_empty"):
        gc.collect()
        torch.cuda.synchronize()
    if mode == "gc_empty":
        torch.cuda.empty_cache()
