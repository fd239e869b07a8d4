"""Remote layer split (reference LLAMACPP_GRPC_SERVERS + `local-ai worker llama-cpp-rpc`): a leader
holding the first layer range + embedding/head and two TCP pipeline stages produce the same tokens
as the unsplit model, across chunked prefill and batched decode; wire format round trip; worker
LoadModel path."""
import numpy as np
import pytest

from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
from localai_tfp_amd.engine.sequence import Request
from localai_tfp_amd.models.loader import load_llm
from localai_tfp_amd.ops.sampling import SamplingParams
from localai_tfp_amd.parallel import pp_rpc


@pytest.fixture()
def stages():
    ss = [pp_rpc.StageServer("127.0.0.1", 0, "cpu").start() for _ in range(2)]
    yield [f"127.0.0.1:{s.address[1]}" for s in ss]
    for s in ss:
        s.shutdown()


def _run(model, tok, prompts, mbt=32):
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_batched_tokens=mbt, max_model_len=256, num_blocks=64))
    hs = [eng.submit(Request(p, SamplingParams(temperature=0.0), 6)) for p in prompts]
    eng.run_until_done()
    out = []
    for h in hs:
        toks = []
        for o in h:
            toks += o.token_ids
        out.append(toks)
    return out


def test_split_layers():
    assert pp_rpc.split_layers(4, 3) == [(0, 1), (1, 3), (3, 4)]
    r = pp_rpc.split_layers(32, 3, [2, 1, 1])
    assert r[0] == (0, 16) and r[-1][1] == 32 and all(b > a for a, b in r)
    assert pp_rpc.split_layers(3, 3) == [(0, 1), (1, 2), (2, 3)]


def test_wire_roundtrip():
    import socket
    a, b = socket.socketpair()
    arr = {"x": np.arange(12, dtype=np.float32).reshape(3, 4), "i": np.array([1, -1], np.int32)}
    pp_rpc.send_msg(a, {"op": "t", "n": 3}, arr)
    h, got = pp_rpc.recv_msg(b)
    assert h == {"op": "t", "n": 3}
    assert np.array_equal(got["x"], arr["x"]) and np.array_equal(got["i"], arr["i"])


def test_layer_split_matches_unsplit(stages):
    full, tok, cfg, _ = load_llm("synthetic:tiny-4l", "cpu")
    split, tok2, _, _ = pp_rpc.load_split("synthetic:tiny-4l", stages, "cpu")
    assert len(split.layers) == 1 and split.remote.ranges == [(1, 3), (3, 4)]  # even split of 4 layers
    rng = np.random.default_rng(0)
    prompts = [rng.integers(0, cfg.vocab, n).tolist() for n in (50, 9, 21)]
    assert _run(split, tok2, prompts) == _run(full, tok, prompts)
    split.remote.close()


def test_worker_loads_split(stages, monkeypatch):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.llm import LLMServicer
    monkeypatch.setenv("LLAMACPP_GRPC_SERVERS", ",".join(stages))
    sv = LLMServicer(device="cpu")
    r = sv.LoadModel(pb.ModelOptions(Model="synthetic:tiny-4l", ContextSize=256, TensorSplit="2,1,1"), None)
    assert r.success, r.message
    assert sv.engine.model.remote is not None and sv.engine.model.remote.ranges == [(2, 3), (3, 4)]
    out = sv.engine.generate([1, 2, 3, 4, 5], SamplingParams(temperature=0.0), max_tokens=4)
    assert len(out.token_ids) == 4
    sv.engine.shutdown()


@pytest.mark.gpu
def test_layer_split_gpu_matches_unsplit():
    """Leader and stage on cuda:0 (stage served from its own thread) vs the unsplit model."""
    s = pp_rpc.StageServer("127.0.0.1", 0, "cuda:0").start()
    try:
        full, tok, cfg, _ = load_llm("synthetic:tiny-4l", "cuda:0")
        split, tok2, _, _ = pp_rpc.load_split("synthetic:tiny-4l", [f"127.0.0.1:{s.address[1]}"], "cuda:0")
        rng = np.random.default_rng(1)
        prompts = [rng.integers(0, cfg.vocab, n).tolist() for n in (40, 7)]
        assert _run(split, tok2, prompts) == _run(full, tok, prompts)
        split.remote.close()
    finally:
        s.shutdown()


def test_layer_split_applies_lora_on_every_stage(stages, tmp_path):
    """the split path used to serve the base model silently when LoraAdapter was set."""
    from localai_tfp_amd.formats.gguf import GGUFWriter
    full0, tok, cfg, _ = load_llm("synthetic:tiny-4l", "cpu")
    rng = np.random.default_rng(5)
    wr = GGUFWriter(str(tmp_path / "ad.gguf"))
    wr.add("general.type", "adapter")
    wr.add("adapter.type", "lora")
    wr.add("adapter.lora.alpha", 4.0)
    for i in range(cfg.n_layers):  # every layer, so remote stages must merge too
        wr.add_tensor(f"blk.{i}.ffn_down.weight.lora_a", rng.standard_normal((4, cfg.ffn)).astype(np.float32))
        wr.add_tensor(f"blk.{i}.ffn_down.weight.lora_b", rng.standard_normal((cfg.hidden, 4)).astype(np.float32))
    wr.write()
    ov = {"lora": [(str(tmp_path / "ad.gguf"), 1.0)]}
    full, _, _, _ = load_llm("synthetic:tiny-4l", "cpu", overrides=ov)
    split, tok2, _, _ = pp_rpc.load_split("synthetic:tiny-4l", stages, "cpu", overrides=ov)
    prompts = [rng.integers(0, cfg.vocab, n).tolist() for n in (30, 7)]
    want = _run(full, tok, prompts)
    assert want != _run(full0, tok, prompts)
    assert _run(split, tok2, prompts) == want
    split.remote.close()
