"""Which engine mode gives the wrong RWKV-6 greedy tokens on the GPU (test_rwkv6_engine_gpu_graphs)?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _model, _ref_logits, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

model, src = _model("cuda:0", seed=6)
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
refs = [int(_ref_logits(model.cfg, src, p)[-1].argmax()) for p in prompts]
print("ref first tokens", refs, flush=True)
for mode in ("eager", "graphs", "graphs+precapture", "eager-single"):
    eng = _engine(model, use_graphs=mode.startswith("graphs"))
    if mode.endswith("precapture"):
        eng.precapture_graphs()
    ps = prompts[:1] if mode == "eager-single" else prompts
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in ps]
    eng.run_until_done()
    print(mode, [_tokens(h) for h in hs], eng.stats.get("graph_steps"), flush=True)
