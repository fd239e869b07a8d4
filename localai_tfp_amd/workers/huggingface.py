"""`huggingface` / `langchain-huggingface` worker: text generation through the remote Hugging Face
Inference API (no local compute).

Behavioural parity: backend/go/llm/langchain/langchain.go:1-64 + pkg/langchain/huggingface.go —
LoadModel fails without HUGGINGFACEHUB_API_TOKEN; Predict sends the prompt with the request's
model, max tokens, temperature and stop words and returns the completion; PredictStream delivers
the whole completion as one chunk (the reference's stream is a single send as well).

`HUGGINGFACEHUB_API_BASE` overrides the endpoint (tests point it at a local server; the GPU box
has no egress). Stop words are also applied client-side, so a server that ignores
`stop_sequences` still honours them."""
from __future__ import annotations

import json
import os
import urllib.error
import urllib.request

import grpc

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

DEFAULT_BASE = "https://api-inference.huggingface.co/models"


class HuggingFaceServicer(BackendServicer):
    def __init__(self, device=None):
        super().__init__()
        self.model = ""
        self.token = ""
        self.timeout = float(os.environ.get("HUGGINGFACEHUB_TIMEOUT", "120"))

    def LoadModel(self, request, context):
        tok = os.environ.get("HUGGINGFACEHUB_API_TOKEN", "")
        if not tok:
            return pb.Result(message="no huggingface token provided", success=False)
        self.token = tok
        self.model = request.Model
        return pb.Result(message=f"remote model {self.model}", success=True)

    def _complete(self, r) -> str:
        base = os.environ.get("HUGGINGFACEHUB_API_BASE", DEFAULT_BASE).rstrip("/")
        params = {"return_full_text": False}
        if r.Tokens > 0:
            params["max_new_tokens"] = int(r.Tokens)
        if r.Temperature > 0:
            params["temperature"] = float(r.Temperature)
        if r.TopP > 0:
            params["top_p"] = float(r.TopP)
        if r.TopK > 0:
            params["top_k"] = int(r.TopK)
        stops = [s for s in r.StopPrompts if s]
        if stops:
            params["stop_sequences"] = stops
        body = json.dumps({"inputs": r.Prompt, "parameters": params, "options": {"wait_for_model": True}}).encode()
        req = urllib.request.Request(f"{base}/{self.model}", data=body, method="POST",
                                     headers={"Authorization": f"Bearer {self.token}",
                                              "Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=self.timeout) as resp:
            out = json.loads(resp.read().decode("utf-8"))
        if isinstance(out, dict) and "error" in out:
            raise RuntimeError(out["error"])
        text = out[0]["generated_text"] if isinstance(out, list) else out.get("generated_text", "")
        if r.Prompt and text.startswith(r.Prompt):  # servers that ignore return_full_text
            text = text[len(r.Prompt):]
        cut = min((text.find(s) for s in stops if s in text), default=-1)
        return text[:cut] if cut >= 0 else text

    def Predict(self, request, context):
        if not self.token:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "model not loaded")
        try:
            text = self._complete(request)
        except (urllib.error.URLError, OSError, RuntimeError, KeyError, IndexError, ValueError) as ex:
            context.abort(grpc.StatusCode.UNAVAILABLE, f"huggingface inference failed: {ex}")
        return pb.Reply(message=text.encode("utf-8"))

    def PredictStream(self, request, context):
        yield self.Predict(request, context)


def main(argv=None):
    worker_main(HuggingFaceServicer, argv)


if __name__ == "__main__":
    main()
