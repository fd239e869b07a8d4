"""BERT embeddings / reranker backend: model numerics vs a plain fp32 PyTorch encoder, worker
micro-batching, and the HTTP surface (/v1/embeddings, /v1/rerank) — reference coverage:
core/http/app_test.go embeddings + rerank cases, backend/python/rerankers/test.py."""
import math

import pytest
import torch
import yaml
from fastapi.testclient import TestClient

from localai_tfp_amd.config.app_config import ApplicationConfig
from localai_tfp_amd.gateway.app import create_app
from localai_tfp_amd.models import bert as BM


def _reference_encode(cfg, get, ids):
    """Straightforward fp32 BERT (post-LN) of one sequence."""
    t = lambda n: torch.from_numpy(get(n))  # noqa: E731
    S = len(ids)
    x = t("token_embd.weight")[ids] + t("position_embd.weight")[:S] + t("token_types.weight")[0]
    x = torch.nn.functional.layer_norm(x, (cfg.hidden,), t("token_embd_norm.weight"), t("token_embd_norm.bias"), cfg.eps)
    hd = cfg.hidden // cfg.n_heads
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        q, k, v = (x @ t(p + f"attn_{n}.weight").T + t(p + f"attn_{n}.bias") for n in "qkv")
        q, k, v = (z.view(S, cfg.n_heads, hd).transpose(0, 1) for z in (q, k, v))
        a = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(hd), -1) @ v
        a = a.transpose(0, 1).reshape(S, cfg.hidden)
        o = a @ t(p + "attn_output.weight").T + t(p + "attn_output.bias")
        x = torch.nn.functional.layer_norm(x + o, (cfg.hidden,), t(p + "attn_output_norm.weight"),
                                           t(p + "attn_output_norm.bias"), cfg.eps)
        u = torch.nn.functional.gelu(x @ t(p + "ffn_up.weight").T + t(p + "ffn_up.bias"))
        d = u @ t(p + "ffn_down.weight").T + t(p + "ffn_down.bias")
        x = torch.nn.functional.layer_norm(x + d, (cfg.hidden,), t(p + "layer_output_norm.weight"),
                                           t(p + "layer_output_norm.bias"), cfg.eps)
    return x


def test_bert_matches_reference_and_padding_invariant():
    cfg = BM.BERT_TINY
    get = BM.synthetic_bert(cfg, 3)
    m = BM.BertModel.load(cfg, get, "cpu")
    seqs = [[2, 17, 40, 9, 3], [2, 50, 3]]
    hid, lens = m.encode(seqs)
    for b, s in enumerate(seqs):
        ref = _reference_encode(cfg, get, s)
        assert torch.allclose(hid[b, :len(s)], ref, atol=2e-4), (hid[b, :len(s)] - ref).abs().max()
    e = m.embed(seqs)
    e1 = m.embed([seqs[1]])
    assert torch.allclose(e[1], e1[0], atol=1e-5)
    assert torch.allclose(e.norm(dim=-1), torch.ones(2), atol=1e-5)


def test_worker_batches_and_reranks():
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.bert import BertServicer
    s = BertServicer(device="cpu")
    assert s.LoadModel(pb.ModelOptions(Model="synthetic:bert-tiny-rerank"), None).success
    import concurrent.futures as cf
    texts = [f"doc number {i}" for i in range(12)]
    with cf.ThreadPoolExecutor(8) as ex:
        embs = list(ex.map(lambda t: s.Embedding(pb.PredictOptions(Embeddings=t), None).embeddings, texts))
    solo = s.Embedding(pb.PredictOptions(Embeddings=texts[5]), None).embeddings
    assert max(abs(a - b) for a, b in zip(embs[5], solo)) < 1e-5
    r = s.Rerank(pb.RerankRequest(query="q", documents=["aa", "bbb", "c"], top_n=2), None)
    assert len(r.results) == 2 and r.results[0].relevance_score >= r.results[1].relevance_score
    assert r.usage.total_tokens > 0


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    d = tmp_path_factory.mktemp("bert")
    models = d / "models"
    models.mkdir()
    (models / "emb.yaml").write_text(yaml.safe_dump({
        "name": "emb", "embeddings": True, "parameters": {"model": "synthetic:bert-tiny"}}))
    (models / "rr.yaml").write_text(yaml.safe_dump({
        "name": "rr", "backend": "rerankers", "parameters": {"model": "synthetic:bert-tiny-rerank"}}))
    cfg = ApplicationConfig(models_path=str(models), generated_content_dir=str(d / "gen"),
                            upload_dir=str(d / "up"), config_dir=str(d / "cfg"), api_keys=[])
    app = create_app(cfg, inproc=True)
    with TestClient(app) as c:
        yield c
    app.state.localai.shutdown()


def test_http_embeddings_and_rerank(client):
    r = client.post("/v1/embeddings", json={"model": "emb", "input": ["hello world", "goodbye"]})
    assert r.status_code == 200, r.text
    d = r.json()["data"]
    assert len(d) == 2 and len(d[0]["embedding"]) == BM.BERT_TINY.hidden
    assert abs(sum(x * x for x in d[0]["embedding"]) - 1) < 1e-4
    r = client.post("/v1/rerank", json={"model": "rr", "query": "what", "documents": ["x y", "z", "w w w"],
                                        "top_n": 3})
    assert r.status_code == 200, r.text
    j = r.json()
    assert sorted(x["index"] for x in j["results"]) == [0, 1, 2]
    sc = [x["relevance_score"] for x in j["results"]]
    assert sc == sorted(sc, reverse=True) and j["usage"]["total_tokens"] > 0


@pytest.mark.gpu
def test_bert_gpu_matches_fp32():
    """GPU path (hipBLASLt GEMMs + attention_dense.hip + norm.hip LayerNorm) vs the fp32 encoder."""
    cfg = BM.BertConfig(vocab=400, hidden=256, n_layers=2, n_heads=4, ffn=1024, max_pos=128, name="t")
    get = BM.synthetic_bert(cfg, 5)
    g = BM.BertModel.load(cfg, get, "cuda:0")
    seqs = [[2] + list(range(10, 10 + n)) + [3] for n in (70, 5, 33)]
    hid, _ = g.encode(seqs)
    for b, s in enumerate(seqs):
        ref = _reference_encode(cfg, get, s)
        err = (hid[b, :len(s)].cpu() - ref).abs().max().item()
        assert err < 5e-2, err
    e = g.embed(seqs).cpu()
    c = BM.BertModel.load(cfg, get, "cpu").embed(seqs)
    assert (e - c).abs().max() < 1e-2
