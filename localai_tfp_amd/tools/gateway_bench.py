"""Gateway capacity micro-benchmark (CPU only): a fake LLM worker streams tokens as fast as the
gateway can take them; measures SSE tokens/s through /v1/chat/completions at a given concurrency.
Isolates gateway + gRPC overhead from the engine."""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time

import yaml

from ..grpc import pb
from ..grpc.server import AioServer, BackendServicer


class FakeLLM(BackendServicer):
    def __init__(self, n_tokens: int, interval: float):
        super().__init__()
        self.n, self.dt = n_tokens, interval

    def LoadModel(self, request, context):
        return pb.Result(success=True)

    async def PredictStream(self, request, context):
        n = request.Tokens or self.n
        for i in range(n):
            if self.dt:
                await asyncio.sleep(self.dt)
            yield pb.Reply(message=b"tok ")
        yield pb.Reply(message=b"", tokens=n, prompt_tokens=10, timing_prompt_processing=1.0,
                       timing_token_generation=1.0)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=128)
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--interval", type=float, default=0.0, help="per-token delay in the fake worker (s)")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--profile", default="", help="write a cProfile of the gateway process here")
    a = ap.parse_args(argv)
    srv = AioServer(FakeLLM(a.tokens, a.interval), "127.0.0.1:0")
    work = tempfile.mkdtemp(prefix="gwbench")
    models = os.path.join(work, "models")
    os.makedirs(models)
    with open(os.path.join(models, "fake.yaml"), "w") as f:
        yaml.safe_dump({"name": "fake", "backend": "llama-cpp", "parameters": {"model": "fake"},
                        "template": {"use_tokenizer_template": True}}, f)
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, LOCALAI_GPUS="none")
    if a.profile:
        env["LOCALAI_CPROFILE"] = a.profile
    prof = []
    gw = subprocess.Popen([sys.executable, *prof, "-m", "localai_tfp_amd", "run", "--models-path", models, "--address",
                           f"127.0.0.1:{port}", "--disable-webui", "--log-level", "warning",
                           "--localai-config-dir", os.path.join(work, "cfg"),
                           "--generated-content-path", os.path.join(work, "gen"), "--upload-path", os.path.join(work, "up"),
                           "--external-grpc-backends", f"llama-cpp:127.0.0.1:{srv.port}"], env=env)
    try:
        import urllib.request
        for _ in range(200):
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=1)
                break
            except Exception:
                time.sleep(0.1)
        out = os.path.join(work, "lg.json")
        subprocess.run([sys.executable, "-m", "localai_tfp_amd.tools.loadgen", "--url", f"http://127.0.0.1:{port}",
                        "--model", "fake", "--concurrency", str(a.concurrency), "--gen-len", str(a.tokens),
                        "--duration", str(a.duration), "--out", out], check=True)
        recs = json.load(open(out))
        ok = [r for r in recs if r.get("ok")]
        chunks = sum(r["chunks"] for r in recs)
        t0 = min(r["t_send"] for r in recs)
        t1 = max(r["t_end"] for r in recs)
        ttft = sorted((r["t_first"] - r["t_send"]) * 1e3 for r in recs if r.get("t_first"))
        print(json.dumps({"chunks_per_s": round(chunks / (t1 - t0), 1), "requests_ok": len(ok),
                          "p50_ttft_ms": round(ttft[len(ttft) // 2], 2) if ttft else None}))
    finally:
        gw.terminate()
        gw.wait()
        srv.stop()


if __name__ == "__main__":
    main()
