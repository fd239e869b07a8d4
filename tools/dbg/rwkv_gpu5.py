"""RWKV-6 precapture: forward-level vs readback-level trace of the first steps (fresh process)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from test_rwkv import _engine, _model, _ref_logits, _tokens  # noqa: E402

from localai_tfp_amd.engine.sequence import Request  # noqa: E402
from localai_tfp_amd.ops.sampling import SamplingParams  # noqa: E402

buckets = tuple(int(b) for b in sys.argv[1].split(",")) if len(sys.argv) > 1 else None
model, src = _model("cuda:0", seed=6)
rng = np.random.default_rng(3)
prompts = [rng.integers(0, model.cfg.vocab, n).tolist() for n in (9, 26, 4)]
eng = _engine(model, use_graphs=True)
if buckets:
    eng.cfg.graph_buckets = buckets
eng.precapture_graphs()
trace = []
orig_fwd = model.forward


def fwd(fb, st, ws):
    out = orig_fwd(fb, st, ws)
    if len(trace) < 3:
        torch.cuda.synchronize()
        trace.append(("fwd", int(fb.n_decode), int(fb.tokens.numel()), fb.tokens[:12].tolist(), fb.slots[:12].tolist(),
                      fb.positions[:12].tolist(), out.float().argmax(-1).tolist()))
    return out


model.forward = fwd
orig_pi = eng._process_inflight


def pi(inf):
    orig_pi(inf)
    if len(trace) < 8:
        ev, k, items, _ = inf
        trace.append(("read", k, eng._pin_tok[k][:len(items)].tolist()))


eng._process_inflight = pi
hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 3)) for p in prompts]
eng.run_until_done()
refs = [int(_ref_logits(model.cfg, src, p)[-1].argmax()) for p in prompts]
got = [_tokens(h) for h in hs]
print(buckets, "ref", refs, "got", got, "OK" if [g[0] for g in got] == refs else "WRONG", flush=True)
for t in trace:
    print("  ", t, flush=True)
