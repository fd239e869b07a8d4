"""Gateway capacity benchmark (CPU only): how many SSE chunks/s one `local-ai run` gateway carries.

Fake LLM workers stand in for the GPUs, so the measurement isolates the serving path (HTTP/SSE gateway,
request middleware, gateway <-> worker transport) from the engine:

* `--transport mx` (default, what this framework's own workers use): each fake worker answers LoadModel with an
  `mxstream=<socket>` address (serving/mxstream.py) and emits, every `--step-ms`, ONE batch frame per gateway
  connection holding one token for every active request — the output pattern of the real engine
  (engine.BatchedSink: one frame per engine step).
* `--transport grpc`: the reference protocol, one PredictStream message per token.

`--replicas N` serves the model as `data_parallel: N` — N worker processes behind the one gateway address, as a user
deploys it (the gateway picks the least-loaded replica per request); `--gateway-workers G` runs that gateway as G
processes sharing the replicas (cli.py, serving/shared_backends.py); the load comes from `--loadgen-procs`
processes (the asyncio load generator tops out near 20-30k chunks/s per process).

Offered load per replica = concurrency / replicas / step_ms tokens/s (128 streams at a 9 ms step: 14.2k, the
per-GPU rate of the c128 bench); the gateway is the bound when chunks/s falls below replicas x that.

    python -m localai_tfp_amd.tools.gateway_bench --replicas 8 --concurrency 1024 --step-ms 9 --loadgen-procs 4
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

import yaml

from ..grpc import pb
from ..grpc.server import AioServer, BackendServicer


class FakeLLM(BackendServicer):
    """gRPC side of a fake worker: LoadModel advertises the mxstream socket; PredictStream is the per-token path."""

    def __init__(self, n_tokens: int, step_s: float, mx_path: str | None):
        super().__init__()
        self.n, self.dt = n_tokens, step_s
        self.mx = FakeMx(mx_path, step_s) if mx_path else None

    def LoadModel(self, request, context):
        return pb.Result(success=True, message=f"mxstream={self.mx.path}" if self.mx else "")

    def Predict(self, request, context):
        n = request.Tokens or self.n
        return pb.Reply(message=b"tok " * n, tokens=n, prompt_tokens=10)

    async def PredictStream(self, request, context):
        n = request.Tokens or self.n
        for _ in range(n):
            if self.dt:
                await asyncio.sleep(self.dt)
            yield pb.Reply(message=b"tok ")
        yield pb.Reply(message=b"", tokens=n, prompt_tokens=10, timing_prompt_processing=1.0,
                       timing_token_generation=1.0)


class FakeMx:
    """mxstream server of a fake worker: one step thread emits a batch frame per connection every step."""

    def __init__(self, path: str, step_s: float):
        from ..serving import mxstream as MX
        self.MX = MX
        self.path = path
        self.step = step_s
        self.lock = threading.Lock()
        self.active: dict = {}  # (conn, rid) -> [remaining, generated]
        if os.path.exists(path):
            os.unlink(path)
        self.lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.lsock.bind(path)
        self.lsock.listen(64)
        threading.Thread(target=self._accept, daemon=True).start()
        threading.Thread(target=self._steps, daemon=True).start()

    def _accept(self):
        while True:
            s, _ = self.lsock.accept()
            s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
            threading.Thread(target=self._serve, args=(s,), daemon=True).start()

    def _serve(self, s):
        MX = self.MX
        try:
            while True:
                hdr = MX._recv_exact(s, MX._HDR.size)
                if hdr is None:
                    return
                ln, typ = MX._HDR.unpack(hdr)
                body = MX._recv_exact(s, ln - 1) if ln > 1 else b""
                if body is None:
                    return
                (rid,) = MX._U64.unpack_from(body, 0)
                with self.lock:
                    if typ == MX.T_SUBMIT:
                        opts = pb.PredictOptions.FromString(body[8:])
                        self.active[(s, rid)] = [opts.Tokens or 256, 0]
                    elif typ == MX.T_ABORT:
                        self.active.pop((s, rid), None)
        except OSError:
            pass
        finally:
            with self.lock:
                for k in [k for k in self.active if k[0] is s]:
                    del self.active[k]

    def _steps(self):
        MX = self.MX
        nxt = time.monotonic()
        while True:
            nxt += self.step
            time.sleep(max(0.0, nxt - time.monotonic()))
            per: dict = {}
            with self.lock:
                for (s, rid), st in list(self.active.items()):
                    st[0] -= 1
                    st[1] += 1
                    fin = st[0] <= 0
                    per.setdefault(s, []).append((rid, MX.F_FINISHED if fin else 0, st[1], 10, 1.0, 1.0, b"tok "))
                    if fin:
                        del self.active[(s, rid)]
            for s, recs in per.items():
                try:
                    s.sendall(MX.pack_batch(recs))
                except OSError:
                    pass


def worker_main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--addr", required=True)
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--step-ms", type=float, default=9.0)
    ap.add_argument("--transport", default="mx")
    a = ap.parse_args(argv)
    port = a.addr.rsplit(":", 1)[-1]
    mx = os.path.join(tempfile.gettempdir(), f"gwbench-mx-{os.getpid()}-{port}.sock") if a.transport == "mx" else None
    srv = AioServer(FakeLLM(a.tokens, a.step_ms / 1e3, mx), a.addr)
    mark = os.environ.get("GWBENCH_MARK")
    if mark:  # one file per started worker (the bench reports how many replicas the gateway processes spawned)
        open(os.path.join(mark, f"worker-{os.getpid()}"), "w").close()
    print(f"fake worker on {a.addr} ({a.transport})", flush=True)
    threading.Event().wait()
    srv.stop()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_bench(replicas: int = 1, concurrency: int = 128, tokens: int = 256, step_ms: float = 9.0,
              transport: str = "mx", duration: float = 10.0, loadgen_procs: int = 1, profile: str = "",
              gateway_workers: int = 1) -> dict:
    work = tempfile.mkdtemp(prefix="gwbench")
    models = os.path.join(work, "models")
    os.makedirs(models)
    # the fake worker executable the gateway spawns per replica (`--external-grpc-backends name:<file>`)
    launcher = os.path.join(work, "fake_worker")
    with open(launcher, "w") as f:
        f.write(f"#!{sys.executable}\nimport sys\nfrom localai_tfp_amd.tools.gateway_bench import worker_main\n"
                f"worker_main(sys.argv[1:] + ['--tokens', '{tokens}', '--step-ms', '{step_ms}', "
                f"'--transport', '{transport}'])\n")
    os.chmod(launcher, 0o755)
    with open(os.path.join(models, "fake.yaml"), "w") as f:
        yaml.safe_dump({"name": "fake", "backend": "fake-llm", "parameters": {"model": "fake"},
                        "data_parallel": replicas, "template": {"use_tokenizer_template": True}}, f)
    port = _free_port()
    env = dict(os.environ, LOCALAI_GPUS="none",
               PYTHONPATH=os.pathsep.join(p for p in (os.path.dirname(os.path.dirname(os.path.dirname(
                   os.path.abspath(__file__)))), os.environ.get("PYTHONPATH", "")) if p))
    env["GWBENCH_MARK"] = work
    if profile:
        env["LOCALAI_CPROFILE"] = profile
    gw = subprocess.Popen([sys.executable, "-m", "localai_tfp_amd", "run", "--models-path", models, "--address",
                           f"127.0.0.1:{port}", "--disable-webui", "--log-level", "warning",
                           "--localai-config-dir", os.path.join(work, "cfg"),
                           "--generated-content-path", os.path.join(work, "gen"), "--upload-path", os.path.join(work, "up"),
                           "--external-grpc-backends", f"fake-llm:{launcher}",
                           "--gateway-workers", str(gateway_workers)], env=env)
    try:
        import urllib.request
        url = f"http://127.0.0.1:{port}"
        for _ in range(300):
            try:
                urllib.request.urlopen(url + "/readyz", timeout=1)
                break
            except Exception:
                time.sleep(0.1)
        # load the model (spawns the replicas) before the clock starts
        req = urllib.request.Request(url + "/v1/chat/completions", method="POST",
                                     data=json.dumps({"model": "fake", "max_tokens": 2, "messages": [
                                         {"role": "user", "content": "hi"}]}).encode(),
                                     headers={"Content-Type": "application/json"})
        urllib.request.urlopen(req, timeout=120).read()
        P = max(1, loadgen_procs)
        outs = [os.path.join(work, f"lg{i}.json") for i in range(P)]
        procs = [subprocess.Popen([sys.executable, "-m", "localai_tfp_amd.tools.loadgen", "--url", url,
                                   "--model", "fake", "--concurrency", str(concurrency // P + (i < concurrency % P)),
                                   "--gen-len", str(tokens), "--duration", str(duration), "--seed", str(i),
                                   "--stagger", "--out", outs[i]], env=env) for i in range(P)]
        for p in procs:
            if p.wait() != 0:
                raise RuntimeError("load generator failed")
        recs = [r for o in outs for r in json.load(open(o))]
    finally:
        gw.terminate()
        try:
            gw.wait(timeout=30)
        except subprocess.TimeoutExpired:
            gw.kill()
    # steady window: the middle of the run (all users active, no ramp / drain edges)
    t0 = min(r["t_send"] for r in recs)
    t1 = max(r["t_end"] for r in recs)
    w0, w1 = t0 + 0.2 * (t1 - t0), t0 + 0.9 * (t1 - t0)
    chunks = sum(1 for r in recs for t in r["t_chunks"] if w0 <= t < w1)
    ttft = sorted((r["t_first"] - r["t_send"]) * 1e3 for r in recs if r.get("t_first"))
    offered = replicas * (concurrency / replicas) / (step_ms / 1e3) if step_ms else None
    return {"replicas": replicas, "gateway_workers": gateway_workers, "transport": transport, "concurrency": concurrency, "step_ms": step_ms,
            "loadgen_procs": loadgen_procs, "chunks_per_s": round(chunks / (w1 - w0), 1),
            "offered_chunks_per_s": round(offered, 1) if offered else None,
            "requests_ok": sum(1 for r in recs if r.get("ok")),
            "p50_ttft_ms": round(ttft[len(ttft) // 2], 2) if ttft else None, "cpus": os.cpu_count(),
            "workers_started": sum(1 for f in os.listdir(work) if f.startswith("worker-"))}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=1, help="data_parallel replicas (fake workers) behind the gateway")
    ap.add_argument("--concurrency", type=int, default=128, help="total concurrent streams")
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--step-ms", type=float, default=9.0, help="fake engine step (one token per stream per step)")
    ap.add_argument("--transport", choices=("mx", "grpc"), default="mx")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--loadgen-procs", type=int, default=1)
    ap.add_argument("--profile", default="", help="write a cProfile of the gateway process here")
    ap.add_argument("--gateway-workers", type=int, default=1, help="`local-ai run --gateway-workers`")
    a = ap.parse_args(argv)
    print(json.dumps(run_bench(a.replicas, a.concurrency, a.tokens, a.step_ms, a.transport, a.duration,
                               a.loadgen_procs, a.profile, a.gateway_workers)))


if __name__ == "__main__":
    main()
