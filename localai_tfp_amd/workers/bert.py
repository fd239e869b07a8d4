"""Embedding / rerank worker (BERT-family encoders) — the reference's `bert-embeddings`
(llama.cpp bert arch), `sentencetransformers` and `rerankers` backends behind one servicer.

RPCs: LoadModel, Embedding (pooled + L2-normalised, as send_embedding), Rerank (cross-encoder head
when the checkpoint has one, else cosine similarity of bi-encoder embeddings; usage counts tokens
like backend/python/rerankers/backend.py:72-91 counts words), TokenizeString.
Concurrent Embedding calls are micro-batched (padding-aware attention) — one encoder pass per batch.
"""
from __future__ import annotations

import logging
import os
import queue
import threading
import time

import grpc

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.bert")

SYNTH = {"bert-tiny": "BERT_TINY", "bert-base": "BERT_BASE"}


def synthetic_wordpiece(n: int):
    from ..tokenizer.wordpiece import WordPieceTokenizer
    base = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    chars = [chr(c) for c in range(33, 127)]
    toks = base + chars + ["##" + c for c in chars]
    toks += [f"[unused{i}]" for i in range(max(0, n - len(toks)))]
    return WordPieceTokenizer(toks[:max(n, len(toks))])


class BertServicer(BackendServicer):
    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.model = None
        self.tok = None
        self.max_len = 512
        self._q: queue.Queue = queue.Queue()
        self._batcher: threading.Thread | None = None
        self.max_batch = int(os.environ.get("MX_EMBED_MAX_BATCH", "64"))

    def LoadModel(self, request, context):
        import torch
        from ..models import bert as BM
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            path = request.ModelFile or request.Model
            if path.startswith("synthetic:"):
                key = path.split(":", 1)[1]
                rerank = key.endswith("-rerank")
                cfg = getattr(BM, SYNTH[key.removesuffix("-rerank")])
                self.model = BM.BertModel.load(cfg, BM.synthetic_bert(cfg, 1, rerank), self.device)
                self.tok = synthetic_wordpiece(cfg.vocab)
            else:
                from ..formats.gguf import GGUFReader
                from ..tokenizer.wordpiece import WordPieceTokenizer
                if not os.path.isabs(path) and request.ModelPath:
                    path = os.path.join(request.ModelPath, path)
                r = GGUFReader(path)
                cfg = BM.BertConfig.from_gguf_metadata(r.metadata)
                self.model = BM.BertModel.load(cfg, BM.gguf_tensor_source(r), self.device)
                self.tok = WordPieceTokenizer.from_gguf(r.metadata)
            self.max_len = self.model.cfg.max_pos
            if self._batcher is None:
                self._batcher = threading.Thread(target=self._batch_loop, daemon=True, name="embed-batcher")
                self._batcher.start()
            return pb.Result(message=f"loaded {self.model.cfg.name}", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    # ------------------------------------------------------------------ micro-batching
    def _batch_loop(self):
        while True:
            first = self._q.get()
            batch = [first]
            deadline = time.perf_counter() + 0.002
            while len(batch) < self.max_batch:
                try:
                    batch.append(self._q.get(timeout=max(0.0, deadline - time.perf_counter())))
                except queue.Empty:
                    break
            try:
                embs = self.model.embed([ids for ids, _ in batch]).cpu()
                for (ids, fut), e in zip(batch, embs):
                    fut.put(e.tolist())
            except Exception as ex:  # fail every waiter
                for _, fut in batch:
                    fut.put(ex)

    def _embed_ids(self, ids):
        fut: queue.Queue = queue.Queue(1)
        self._q.put((ids[: self.max_len], fut))
        r = fut.get()
        if isinstance(r, Exception):
            raise r
        return r

    def _need(self, context):
        if self.model is None:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "model not loaded")

    def Embedding(self, request, context):
        self._need(context)
        ids = list(request.EmbeddingTokens) or self.tok.encode(request.Embeddings or request.Prompt)
        return pb.EmbeddingResult(embeddings=self._embed_ids(ids))

    def TokenizeString(self, request, context):
        self._need(context)
        ids = self.tok.encode(request.Prompt, add_special=False)
        return pb.TokenizationResponse(length=len(ids), tokens=ids)

    def Rerank(self, request, context):
        import torch
        self._need(context)
        docs = list(request.documents)
        if not docs:
            return pb.RerankResult(usage=pb.Usage())
        n_tok = 0
        if self.model.has_cls_head:
            pairs, types = [], []
            for d in docs:
                ids, ty = self.tok.encode_pair(request.query, d, self.max_len)
                pairs.append(ids)
                types.append(ty)
                n_tok += len(ids)
            with self._lock:
                scores = self.model.rerank_scores(pairs, types).cpu().tolist()
        else:
            qv = torch.tensor(self._embed_ids(self.tok.encode(request.query)))
            dv = [torch.tensor(self._embed_ids(self.tok.encode(d))) for d in docs]
            scores = [float(qv @ v) for v in dv]
            n_tok = sum(len(self.tok.encode(d)) for d in docs) + len(self.tok.encode(request.query))
        order = sorted(range(len(docs)), key=lambda i: -scores[i])
        top = request.top_n if request.top_n > 0 else len(docs)
        res = [pb.DocumentResult(index=i, text=docs[i], relevance_score=float(scores[i])) for i in order[:top]]
        return pb.RerankResult(usage=pb.Usage(total_tokens=n_tok, prompt_tokens=n_tok), results=res)


def main(argv=None):
    worker_main(BertServicer, argv)


if __name__ == "__main__":
    main()
