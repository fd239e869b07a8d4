"""RWKV-6: the rwkv_gpu.py sequence (engine 3 built while engine 2 is still referenced), engine 3 traced."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _model, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

fix = sys.argv[1] if len(sys.argv) > 1 else ""
if fix == "rocblas":
    torch.backends.cuda.preferred_blas_library("cublas")
if fix == "q8":
    from localai_tfp_amd.models import rwkv as RW
    _c = RW.tiny_rwkv_config()
    src = RW.synthetic_rwkv_source(_c, seed=6, qtype="Q8_0")
    model = RW.RwkvModel.load(_c, src, "cuda:0")
else:
    model, src = _model("cuda:0", seed=6)
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
orig_fwd = model.forward
stash = []
for mode in ("eager", "graphs", "graphs+precapture"):
    eng = _engine(model, use_graphs=mode.startswith("graphs"))
    trace = []
    if mode.endswith("precapture"):
        if fix == "sync":
            torch.cuda.synchronize()
        eng.precapture_graphs()
        if fix == "sync":
            torch.cuda.synchronize()

        def fwd(fb, st, ws):
            inp = (fb.tokens[:12].tolist(), fb.slots[:12].tolist(), fb.positions[:12].tolist())
            out = orig_fwd(fb, st, ws)
            if len(trace) < 2:
                torch.cuda.synchronize()
                trace.append(("fwd", int(fb.n_decode), inp, out.float().argmax(-1).tolist(),
                              float(out.float().abs().sum()), [float(t.abs().sum()) for t in (st.att_shift, st.wkv)]))
            return out
        model.forward = fwd
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in prompts]
    eng.run_until_done()
    model.forward = orig_fwd
    if fix == "keepgraphs":
        stash.append((eng.graphs, eng._graph_pool))
    print(fix, mode, [_tokens(h) for h in hs], flush=True)
    for t in trace:
        print("   ", t, flush=True)
