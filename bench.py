#!/usr/bin/env python3
"""Headline benchmark: output tokens/s + p50 TTFT of chat-completion serving, Llama-3-8B-Instruct
Q4_K_M, one engine replica per GPU (BASELINE.json config #2; N GPUs = data-parallel replicas).

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 it is launched with
torch.distributed.run, one rank per GPU (RCCL). Each rank builds a random-init Llama-3-8B with the
exact Q4_K_M tensor types of a real checkpoint (models/synthetic.py; no network for weights) and
serves a closed-loop load of `--concurrency` chat requests (prompt `--prompt-len` tokens rendered
through the Llama-3 chat template, `--gen-len` output tokens, ignore_eos). A "step" is one engine
iteration (continuous batching: decode rows + chunked prefill). W untimed steps (graph capture,
warm caches), then exactly K timed steps bracketed by barrier + device sync. Output tokens counted
are those produced inside the timed window; TTFT is measured per request from submission to its
first token (requests whose first token lands in the window). Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "output tokens/sec + p50 TTFT, /v1/chat/completions Llama-3-8B Q4_K at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "llama3-70b", "llama32-1b"])
    ap.add_argument("--concurrency", type=int, default=128)
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=2048)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)

    from localai_tfp_amd import _build
    _build.build_all()
    from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
    from localai_tfp_amd.engine.sequence import Request
    from localai_tfp_amd.models import config as C
    from localai_tfp_amd.models.llama import LlamaModel
    from localai_tfp_amd.models.synthetic import synthetic_source
    from localai_tfp_amd.ops.sampling import SamplingParams
    from localai_tfp_amd.templates.chat import render_chat
    from localai_tfp_amd.tokenizer import ByteTokenizer

    cfg = {"llama3-8b": C.LLAMA3_8B, "llama3-70b": C.LLAMA3_70B, "llama32-1b": C.LLAMA32_1B}[args.model]
    if dev.type == "cpu":  # plumbing only
        cfg = C.tiny_config()
    t0 = time.time()
    model = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=1), dev)
    t_load = time.time() - t0
    tok = ByteTokenizer(cfg.vocab)
    ecfg = EngineConfig(max_num_seqs=args.concurrency, max_batched_tokens=args.max_batched_tokens,
                        max_model_len=max(4096, args.prompt_len + args.gen_len + 64), use_graphs=not args.no_graphs)
    eng = LLMEngine(model, tok, ecfg)

    rng = np.random.default_rng(1234 + rank)
    words = ["the", "model", "serves", "tokens", "fast", "on", "MI355X", "with", "paged", "attention", "and",
             "hipGraph", "decode", "kernels", "for", "every", "request", "in", "the", "batch"]

    def make_prompt():
        # chat request -> Llama-3 template -> byte tokens, trimmed/padded to prompt_len
        body = " ".join(rng.choice(words, size=args.prompt_len))
        ids = tok.encode(render_chat([{"role": "user", "content": body}], tok))
        ids = ids[: args.prompt_len]
        return ids

    sp = SamplingParams(temperature=0.0, top_k=1, ignore_eos=True)
    inflight = {}
    ttfts_all = []
    stats = {"tokens": 0}
    timed = {"on": False}
    handles = {}

    def submit():
        req = Request(make_prompt(), sp, max_tokens=args.gen_len)
        h = eng.submit(req)
        handles[req.rid] = (h, time.perf_counter())

    for _ in range(args.concurrency):
        submit()

    def drain():
        done = []
        for rid, (h, t_sub) in list(handles.items()):
            while not h.q.empty():
                o = h.q.get_nowait()
                if timed["on"]:
                    stats["tokens"] += len(o.token_ids)
                if o.token_ids and not getattr(h, "_first", False):
                    h._first = True
                    if timed["on"]:
                        ttfts_all.append((time.perf_counter() - t_sub) * 1e3)
                if o.finished:
                    done.append(rid)
        for rid in done:
            handles.pop(rid)
            submit()

    def step():
        eng._drain_inbox()
        eng.step()
        drain()

    for _ in range(args.warmup):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    timed["on"] = True
    t_start = time.perf_counter()
    prof = None
    if args.profile_steps:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA])
        prof.start()
    for i in range(args.steps):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t_el = time.perf_counter() - t_start
    if prof:
        prof.stop()
        if rank == 0:
            print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=30), file=sys.stderr)
    tokens = stats["tokens"]
    p50 = float(np.percentile(ttfts_all, 50)) if ttfts_all else float("nan")
    p99 = float(np.percentile(ttfts_all, 99)) if ttfts_all else float("nan")
    t_max = t_el
    tok_sum = tokens
    p50_all = p50
    if dist:
        tt = torch.tensor([t_el, float(tokens), p50], device=dev, dtype=torch.float64)
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        t_max = float(mx[0])
        tok_sum = float(sm[1])
        p50_all = float(sm[2] / world)
    value = tok_sum / t_max
    if rank == 0:
        st = eng.stats
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "output tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random-init Llama-3-8B weights in real Q4_K_M block formats; synthetic chat prompts)",
            "p50_ttft_ms": round(p50_all, 2),
            "p99_ttft_ms": round(p99, 2),
            "config": {
                "model": cfg.name + " Q4_K_M", "global_batch": args.concurrency * world,
                "seq_len": args.prompt_len + args.gen_len, "prompt_len": args.prompt_len, "gen_len": args.gen_len,
                "concurrency_per_gpu": args.concurrency, "parallelism": f"dp{world}",
                "path": "engine (scheduler+kernels, in-process; gateway/gRPC excluded)",
                "load_s": round(t_load, 1), "graph_steps": st["graph_steps"], "total_steps": st["steps"],
                "weights_gb": round(model.weight_bytes() / 1e9, 2), "kv_blocks": eng.kv.num_blocks,
            },
        }
        print(json.dumps(out), flush=True)
    eng.shutdown()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
