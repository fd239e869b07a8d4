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


def _cfg(kind):
    from localai_tfp_amd.models.config import tiny_config
    if kind == "wide":  # TP 4 / 8 with whole 256-wide super-blocks per shard: hidden 2048, ffn 2048, 8 kv heads
        return tiny_config(n_layers=2, hidden=2048, ffn=2048, n_heads=16, n_kv_heads=8, head_dim=128, rope_dim=128,
                           vocab=1024)
    # row-parallel shards must be whole 256-element Q4_K/Q6_K super-blocks: hidden 512 / tp 2
    if kind == "moe":  # expert parallel: 8 experts, 4 per rank, top-2 routing + renorm
        return tiny_config(arch="qwen3moe", n_layers=2, hidden=512, ffn=1024, n_heads=8, n_kv_heads=2, head_dim=64,
                           rope_dim=64, n_expert=8, n_expert_used=2, expert_ffn=256, qk_norm=True)
    return tiny_config(n_layers=2, hidden=512, ffn=1024, n_heads=8, n_kv_heads=2, head_dim=64, rope_dim=64)


def _build(rank, world, link, kind="dense"):
    from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
    from localai_tfp_amd.models.llama import LlamaModel
    from localai_tfp_amd.models.synthetic import synthetic_source
    from localai_tfp_amd.tokenizer import ByteTokenizer
    cfg = _cfg(kind)
    model = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=7), "cpu", rank, world, None)
    ec = EngineConfig(num_blocks=128, max_num_seqs=4, max_batched_tokens=32, max_model_len=256)
    return LLMEngine(model, ByteTokenizer(cfg.vocab), ec, tp=link)


def _link(rank, world, port, timeout_s=120, heartbeat_s=None):
    import datetime
    import torch.distributed as dist
    from localai_tfp_amd.parallel.tp_engine import TPLink
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
    sync = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
    return TPLink(rank, world, cpu, sync_group=sync, heartbeat_s=heartbeat_s)


def _worker(rank, world, port, q, kind="dense"):
    import torch.distributed as dist
    link = _link(rank, world, port, heartbeat_s=0.5)  # heartbeats interleave with real plans
    eng = _build(rank, world, link, kind)
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
        import os
        if int(os.environ.get("MX_TP_CHUNKS", "1")) > 1:
            assert getattr(eng.model, "tp_chunked_calls", 0) > 0, "chunked row-parallel path never ran"
        q.put(outs)
    else:
        eng.follow()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,chunks", [("dense", 2, 1), ("moe", 2, 1), ("wide", 4, 1), ("wide", 8, 1),
                                               ("dense", 2, 3), ("wide", 8, 2)])
def test_tp_matches_single_process(kind, world, chunks, monkeypatch):
    """Greedy output of a TP group (leader + followers replaying plans over the /dev/shm ring, sampled
    tokens broadcast each overlap-mode step) equals the single-process engine. chunks > 1: the row-parallel
    projections run as row chunks whose all-reduce + residual add is pipelined behind the next chunk's GEMM
    (models/llama.py _chunked_proj_allreduce; in order on gloo), from 4 rows up so prefill and batched
    decode steps both take it."""
    monkeypatch.setenv("MX_TP_CHUNKS", str(chunks))
    monkeypatch.setenv("MX_TP_CHUNK_MIN_ROWS", "4" if chunks > 1 else "64")
    eng = _build(0, 1, None, kind)
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
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, kind)) for r in range(world)]
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


def test_plan_codec_roundtrip():
    import numpy as np
    from localai_tfp_amd.parallel.tp_engine import decode_plan, encode_plan
    rng = np.random.default_rng(0)
    plan = {"nd": 3, "tokens": rng.integers(0, 999, 9).astype(np.int32), "positions": np.arange(9, dtype=np.int32),
            "slots": np.arange(9, dtype=np.int32) + 16, "lidx": np.array([0, 1, 2, 8], np.int32),
            "dec_bt": rng.integers(0, 50, (3, 5)).astype(np.int32), "dec_lens": np.array([4, 5, 6], np.int32),
            "pf_bt": rng.integers(0, 50, (1, 2)).astype(np.int32), "pf_cu": np.array([0, 6], np.int32),
            "pf_ctx": np.array([6], np.int32), "pf_tseq": np.array([0], np.int32), "pf_tq0": np.array([0], np.int32),
            "keep_hidden": True, "graph": False, "gather": True,
            "fix": (np.array([0, 2], np.int64), np.array([1, 0], np.int64))}
    buf = encode_plan(plan)
    assert buf.dtype == np.int32
    out = decode_plan(buf)
    assert out["nd"] == 3 and out["keep_hidden"] and not out["graph"] and out["gather"]
    for k in ("tokens", "positions", "slots", "lidx", "dec_bt", "dec_lens", "pf_bt", "pf_cu", "pf_ctx", "pf_tseq", "pf_tq0"):
        assert np.array_equal(out[k], plan[k]) and out[k].shape == plan[k].shape, k
    assert all(np.array_equal(a, b) for a, b in zip(out["fix"], plan["fix"]))
    dec_only = decode_plan(encode_plan({"nd": 1, "tokens": np.array([5], np.int32), "positions": np.array([3], np.int32),
                                        "slots": np.array([19], np.int32), "lidx": np.array([0], np.int32),
                                        "graph": (8, 0, 0, 512)}))
    assert dec_only["graph"] == (8, 0, 0, 512) and "pf_cu" not in dec_only and "fix" not in dec_only
    assert out["argmax_on"] and dec_only["argmax_on"]  # default: the graph's greedy head runs
    assert not decode_plan(encode_plan({**plan, "argmax_on": False}))["argmax_on"]


def _die_worker(rank, world, port, who):
    link = _link(rank, world, port, timeout_s=6, heartbeat_s=0.5)
    import time
    if rank == who:
        time.sleep(1.0)
        os._exit(0)  # crash without tearing down the group
    if rank == 0:  # leader: keep sending until the dead follower is noticed
        for _ in range(200):
            link.send_control("noop")
            time.sleep(0.1)
    else:
        while True:
            link.recv_control()


@pytest.mark.parametrize("who", [0, 1])
def test_dead_rank_exits_nonzero(who):
    """A crashed leader (follower side) or follower (leader side) ends the survivor with
    EXIT_TP_FAILURE within the group timeout instead of hanging it."""
    from localai_tfp_amd.parallel.tp_engine import EXIT_TP_FAILURE
    ctx = mp.get_context("spawn")
    port = _port()
    ps = [ctx.Process(target=_die_worker, args=(r, 2, port, who)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=90)
    alive = [p.is_alive() for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert not any(alive), alive
    assert ps[1 - who].exitcode == EXIT_TP_FAILURE, [p.exitcode for p in ps]


def _vocab_argmax_worker(rank, world, port, q):
    import torch.distributed as dist
    from localai_tfp_amd.models.llama import LlamaModel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from localai_tfp_amd.models.config import tiny_config
    V = 1000  # not a multiple of world: the last shard carries padding columns
    cfg = tiny_config(vocab=V)
    m = LlamaModel.__new__(LlamaModel)
    m.cfg, m.tp_rank, m.tp_size, m.tp_group = cfg, rank, world, None
    g = torch.Generator().manual_seed(11)
    full = torch.randn(5, V, generator=g)
    full[1, 7] = full[1, 900] = 50.0  # tie across shards -> the lower index
    full[2] = -1.0  # all equal -> index 0
    vl = -(-V // world)
    loc = torch.full((5, vl), 1e9)  # padding columns must never win
    lo, hi = rank * vl, min(V, (rank + 1) * vl)
    loc[:, :hi - lo] = full[:, lo:hi]
    out = torch.zeros(5, dtype=torch.int32)
    m.vocab_argmax(loc, None, out)
    if rank == 0:
        q.put((out.tolist(), full.argmax(1).tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_vocab_parallel_argmax(world):
    """TP greedy head: per-shard (max, index) merged across ranks == argmax over the gathered logits."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_vocab_argmax_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got, want = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
    assert got == want and got[1] == 7 and got[2] == 0


def _big_plan_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist
    link = _link(rank, world, port, heartbeat_s=0)
    assert link.shm is not None
    n = link.shm.max_body() // 4 * 2 + 12345  # > 2 ring slots of int32: three raw pieces
    plan = {"nd": 3, "graph": False, "tokens": np.arange(n, dtype=np.int32), "positions": np.arange(7, dtype=np.int32)}
    if rank == 0:
        link.send_plan(plan)
        link.send_plan({"nd": 1, "graph": False, "tokens": np.array([5], np.int32)})
        link.send_plan(None)
        q.put("sent")
    else:
        got = link.recv_plan()
        small = link.recv_plan()
        stop = link.recv_plan()
        ok = (got["nd"] == 3 and np.array_equal(got["tokens"], plan["tokens"])
              and np.array_equal(got["positions"], plan["positions"]) and small["tokens"].tolist() == [5]
              and stop is None)
        q.put(("recv", ok))
    link.close()
    dist.destroy_process_group()


def test_oversized_plan_raw_pieces():
    """A plan larger than one shared-memory ring slot travels as raw int32 pieces (no pickle fallback)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_big_plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    assert "sent" in res and ("recv", True) in res, res
