"""LLM worker over real gRPC (loopback), CPU fp32 path with a synthetic tiny Llama: the RPC surface
of backend/cpp/llama/grpc-server.cpp (LoadModel, Predict, PredictStream, Embedding, TokenizeString,
GetMetrics, Status) plus grammar-constrained decoding."""
import math

import pytest

from localai_tfp_amd.grpc import pb
from localai_tfp_amd.grpc.client import BackendClient
from localai_tfp_amd.grpc.server import AioServer
from localai_tfp_amd.workers.llm import LLMServicer


@pytest.fixture(scope="module")
def client():
    svc = LLMServicer(device="cpu")
    server = AioServer(svc, "127.0.0.1:0", max_workers=8)
    c = BackendClient(f"127.0.0.1:{server.port}")
    assert c.health()
    r = c.load_model(pb.ModelOptions(Model="synthetic:tiny", ContextSize=512, Embeddings=True))
    assert r.success, r.message
    yield c
    c.close()
    svc.engine.shutdown()
    server.stop()


def opts(**kw):
    base = dict(Prompt="Hello world", Tokens=8, Temperature=0.0, TopK=40, TopP=0.95, IgnoreEOS=True)
    base.update(kw)
    return pb.PredictOptions(**base)


def test_predict_and_stream_agree(client):
    r = client.predict(opts())
    assert r.tokens == 8 and r.prompt_tokens == len("Hello world") + 1
    assert r.timing_token_generation > 0
    chunks = list(client.predict_stream(opts()))
    assert chunks[-1].tokens == 8
    assert b"".join(c.message for c in chunks) == r.message


def test_sampling_seed_reproducible(client):
    a = client.predict(opts(Temperature=1.0, Seed=123, Tokens=12))
    b = client.predict(opts(Temperature=1.0, Seed=123, Tokens=12))
    assert a.message == b.message


def test_stop_words_and_chat_template(client):
    r = client.predict(opts(Messages=[pb.Message(role="user", content="hi")], UseTokenizerTemplate=True))
    # llama-3 template: <|begin_of_text|> + header tokens + "hi" + ... -> many more prompt tokens than "hi"
    assert r.prompt_tokens > 10
    full = client.predict(opts(Tokens=16)).message.decode(errors="replace")
    if len(full) > 4:
        stop = full[2:4]
        cut = client.predict(opts(Tokens=16, StopPrompts=[stop])).message.decode(errors="replace")
        assert stop not in cut and full.startswith(cut)


def test_grammar_constrained(client):
    r = client.predict(opts(Tokens=32, Temperature=0.7, Seed=5, Grammar='root ::= ("yes" | "no") "!"'))
    assert r.message in (b"yes!", b"no!")
    g = 'root ::= "{" "\\"a\\"" ":" [0-9]{1,3} "}"'
    r = client.predict(opts(Tokens=32, Temperature=1.0, Seed=9, Grammar=g))
    s = r.message.decode()
    assert s.startswith('{"a":') and s.endswith("}") and s[5:-1].isdigit()


def test_embedding_tokenize_metrics_status(client):
    e = client.Embedding(pb.PredictOptions(Embeddings="some text to embed"))
    v = list(e.embeddings)
    assert len(v) == 256 and math.isclose(sum(x * x for x in v), 1.0, rel_tol=1e-4)
    e2 = client.Embedding(pb.PredictOptions(Embeddings="some text to embed"))
    assert list(e2.embeddings) == pytest.approx(v, abs=1e-5)
    t = client.TokenizeString(pb.PredictOptions(Prompt="abc"))
    assert list(t.tokens) == [97, 98, 99] and t.length == 3
    m = client.GetMetrics(pb.MetricsRequest())
    assert m.tokens_generated > 0
    st = client.Status(pb.HealthMessage())
    assert st.state in (pb.STATE_READY, pb.STATE_BUSY) and st.memory.breakdown["gen_tokens_total"] > 0


def test_unimplemented_rpc(client):
    import grpc
    with pytest.raises(grpc.RpcError) as ei:
        client.TTS(pb.TTSRequest(text="x"))
    assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
