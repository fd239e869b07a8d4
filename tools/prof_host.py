"""Host-side cost of the engine loop at high concurrency on CPU (tiny model, so the forward is cheap):
cProfile of run_until_done with N concurrent requests; prints the top functions by own time."""
import cProfile
import pstats
import sys
import time

from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
from localai_tfp_amd.engine.sequence import Request
from localai_tfp_amd.models.config import tiny_config
from localai_tfp_amd.models.llama import LlamaModel
from localai_tfp_amd.models.synthetic import synthetic_source
from localai_tfp_amd.ops.sampling import SamplingParams
from localai_tfp_amd.tokenizer import ByteTokenizer

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
GEN = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = tiny_config(n_layers=1)
m = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=1), "cpu")
tok = ByteTokenizer(cfg.vocab)
e = LLMEngine(m, tok, EngineConfig(num_blocks=8192, max_num_seqs=N, max_batched_tokens=4096, max_model_len=1024))
for i in range(N):
    e.submit(Request(rid=i, prompt_ids=tok.encode(f"request {i} " * 8), max_tokens=GEN,
                     params=SamplingParams(temperature=0.9, top_k=40, top_p=0.95, seed=i)))
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
e.run_until_done()
pr.disable()
dt = time.perf_counter() - t0
st = e.stats
print(f"{st['steps']} steps, {dt / st['steps'] * 1e3:.2f} ms/step wall (CPU forward included)")
for k in ("sched_s", "plan_s", "fwd_s", "process_s", "wait_s"):
    print(k, f"{st.get(k, 0) / st['steps'] * 1e3:.3f} ms/step")
pstats.Stats(pr).sort_stats("cumtime").print_stats("engine|scheduler|sequence|kv_cache|tokenizer|sampling.py", 40)
