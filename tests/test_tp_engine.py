"""Tensor-parallel serving on CPU: 2 ranks over gloo (same code path as RCCL on GPU). The leader
schedules/samples and ships step plans; the follower replays them (engine.follow). Greedy output must
match the single-process engine."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


PROMPTS = [list(b"tensor parallel test prompt one"), list(b"another, somewhat longer prompt for the second seq")]


def _build(rank, world, link):
    from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
    from localai_tfp_amd.models.config import tiny_config
    from localai_tfp_amd.models.llama import LlamaModel
    from localai_tfp_amd.models.synthetic import synthetic_source
    from localai_tfp_amd.tokenizer import ByteTokenizer
    # row-parallel shards must be whole 256-element Q4_K/Q6_K super-blocks: hidden 512 / tp 2
    cfg = tiny_config(n_layers=2, hidden=512, ffn=1024, n_heads=8, n_kv_heads=2, head_dim=64, rope_dim=64)
    model = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=7), "cpu", rank, world, None)
    ec = EngineConfig(num_blocks=128, max_num_seqs=4, max_batched_tokens=32, max_model_len=256)
    return LLMEngine(model, ByteTokenizer(cfg.vocab), ec, tp=link)


def _worker(rank, world, port, q):
    import datetime
    import torch.distributed as dist
    from localai_tfp_amd.parallel.tp_engine import TPLink
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=120))
    link = TPLink(rank, world, cpu)
    eng = _build(rank, world, link)
    if rank == 0:
        from localai_tfp_amd.engine.sequence import Request
        from localai_tfp_amd.ops.sampling import SamplingParams
        hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 10)) for p in PROMPTS]
        eng.run_until_done()
        outs = []
        for h in hs:
            ids = []
            for o in h:
                ids += o.token_ids
            outs.append(ids)
        eng.shutdown()
        q.put(outs)
    else:
        eng.follow()
    dist.destroy_process_group()


def test_tp2_matches_single_process():
    eng = _build(0, 1, None)
    from localai_tfp_amd.engine.sequence import Request
    from localai_tfp_amd.ops.sampling import SamplingParams
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 10)) for p in PROMPTS]
    eng.run_until_done()
    ref = []
    for h in hs:
        ids = []
        for o in h:
            ids += o.token_ids
        ref.append(ids)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    import queue as _q
    import time
    outs = None
    t0 = time.time()
    try:
        while outs is None and time.time() - t0 < 240:
            try:
                outs = q.get(timeout=2)
            except _q.Empty:
                if any(p.exitcode not in (None, 0) for p in ps):
                    raise AssertionError(f"rank exited: {[p.exitcode for p in ps]}")
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert [len(o) for o in outs] == [10, 10]
    assert outs == ref
