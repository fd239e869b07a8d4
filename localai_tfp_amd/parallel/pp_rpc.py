"""Remote layer split ("workers mode" / model sharding across hosts): pipeline stages over TCP.

Reference behaviour: llama.cpp's RPC backend — `rpc-server` processes started by
`local-ai worker llama-cpp-rpc` (core/cli/worker/worker_llamacpp.go:19-44, p2p variant
worker_p2p.go:31-115) become extra ggml devices of the LLM worker when `LLAMACPP_GRPC_SERVERS`
lists them (grpc-server.cpp:139-161, 2358-2361); each device holds a contiguous layer range and
activations hop devices at range boundaries.

MI355X-first redesign: ggml-rpc ships individual tensors and whole compute graphs over the wire
and executes them op by op. Here a stage is a complete engine slice: it loads its own layer range
of the model (from its own copy of the checkpoint — no weights over the network), owns the paged
KV cache of those layers, and runs them with the same fused HIP kernels as a local model. Per
engine step the leader sends one message — the host step plan (token positions, KV slots, block
tables: a few KB of int32) plus the hidden rows [T, H] fp32 — and receives the hidden rows back,
so a step costs one round trip per stage and the wire never carries graph structure.

Wire format (no pickle: a stage is a network service): 4-byte length + JSON header, then the raw
little-endian bytes of each array the header lists as {name: [dtype, shape]}.

Intra-node splits use tensor parallelism over RCCL/xGMI instead (parallel/tp.py); this path is for
capacity across hosts, like the reference's.
"""
from __future__ import annotations

import json
import logging
import socket
import socketserver
import struct
import threading

import numpy as np
import torch

log = logging.getLogger("localai_tfp_amd.pp_rpc")

_ARRAY_KEYS = ("tokens", "positions", "slots", "lidx", "dec_bt", "dec_lens", "pf_bt", "pf_cu", "pf_ctx")


# ------------------------------------------------------------------------------------------------ wire
def _recv_exact(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    mv = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(mv[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed the connection")
        got += k
    return buf


def send_msg(sock: socket.socket, header: dict, arrays: dict | None = None):
    arrays = arrays or {}
    meta = {k: [str(a.dtype), list(a.shape)] for k, a in arrays.items()}
    hb = json.dumps({**header, "_arrays": meta}).encode()
    parts = [struct.pack("<I", len(hb)), hb] + [np.ascontiguousarray(a).tobytes() for a in arrays.values()]
    sock.sendall(b"".join(parts))


def recv_msg(sock: socket.socket) -> tuple[dict, dict]:
    (n,) = struct.unpack("<I", _recv_exact(sock, 4))
    header = json.loads(bytes(_recv_exact(sock, n)))
    arrays = {}
    for k, (dt, shape) in header.pop("_arrays", {}).items():
        dtype = np.dtype(dt)
        if dtype.hasobject:
            raise ValueError("object arrays are not accepted")
        nbytes = int(np.prod(shape)) * dtype.itemsize if shape else dtype.itemsize
        arrays[k] = np.frombuffer(_recv_exact(sock, nbytes), dtype=dtype).reshape(shape)
    return header, arrays


# ------------------------------------------------------------------------------------------------ stage
class _Stage:
    """One loaded layer range with its KV cache and workspace."""

    def __init__(self, req: dict, device):
        from ..engine.kv_cache import KVCache
        from ..models.llama import Workspace
        from ..models.loader import _apply_overrides, _lora_attach, _lora_source, gguf_source, SYNTHETIC
        from ..models.llama import LlamaModel
        from ..engine.engine import kv_format_id, kv_torch_dtype
        model = req["model"]
        l0, l1 = req["layers"]
        if model.startswith("synthetic:"):
            import copy
            from ..models.synthetic import synthetic_source
            cfg = copy.deepcopy(SYNTHETIC[model.split(":", 1)[1]])
            _apply_overrides(cfg, req.get("overrides") or {})
            src = synthetic_source(cfg, "Q4_K_M", seed=1)
        else:
            from ..formats.gguf import GGUFReader
            from ..models.config import LlamaConfig
            r = GGUFReader(model)
            cfg = LlamaConfig.from_gguf_metadata(dict(r.metadata))
            _apply_overrides(cfg, req.get("overrides") or {})
            src = gguf_source(r)
        # LoRA adapters apply on every stage (adapter paths must resolve on the stage's host)
        ov = req.get("overrides") or {}
        self.model = _lora_attach(LlamaModel.load(cfg, _lora_source(src, ov, cfg), device, layer_range=(l0, l1),
                                                  stage=True), ov, cfg, 1, l0)
        self.cfg = cfg
        self.device = torch.device(device)
        self.kv = KVCache(l1 - l0, int(req["num_blocks"]), self.model.n_kv, int(req["block_size"]), cfg.head_dim,
                          self.device, kv_torch_dtype(req.get("kv_dtype", "bf16")),
                          kvf=kv_format_id(req.get("kv_dtype", "bf16")))
        self.ws = Workspace(cfg, int(req["max_tokens"]), int(req["max_seqs"]), self.device, 1, int(req["max_parts"]))

    def forward(self, header: dict, arrays: dict) -> np.ndarray:
        from ..models.llama import ForwardBatch
        dev = self.device
        t = {k: torch.from_numpy(np.ascontiguousarray(arrays[k])).to(dev) for k in _ARRAY_KEYS if k in arrays}
        nd = int(header["nd"])
        fb = ForwardBatch(t["tokens"], t["positions"], t["slots"], t["lidx"], n_decode=nd)
        if nd:
            fb.dec_block_tables, fb.dec_seq_lens = t["dec_bt"], t["dec_lens"]
            fb.dec_max_len = int(arrays["dec_lens"].max())
        if "pf_cu" in t:
            fb.pf_block_tables, fb.pf_cu_q, fb.pf_ctx_lens = t["pf_bt"], t["pf_cu"], t["pf_ctx"]
            cu = arrays["pf_cu"]
            fb.pf_q_lens_host = [int(cu[k + 1] - cu[k]) for k in range(len(cu) - 1)]
            fb.pf_ctx_lens_host = [int(x) for x in arrays["pf_ctx"]]
        T = fb.T
        h = arrays["hidden"]
        self.ws.h[:T].copy_(torch.from_numpy(np.ascontiguousarray(h)).to(dev))
        out = self.model.forward(fb, self.kv, self.ws)
        return out.float().cpu().numpy()


class StageServer:
    """`local-ai worker llama-cpp-rpc` / `python -m localai_tfp_amd.parallel.pp_rpc`: serves layer
    ranges to one leader at a time (a new `load` replaces the previous stage)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 50052, device: str | None = None):
        if device is None:
            device = "cuda:0" if torch.cuda.is_available() else "cpu"
        self.device = device
        self.stage: _Stage | None = None
        self._lock = threading.Lock()
        outer = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                outer._serve_conn(self.request)

        class Server(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self.server = Server((host, port), Handler)
        self.address = self.server.server_address

    def _serve_conn(self, sock: socket.socket):
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        while True:
            try:
                header, arrays = recv_msg(sock)
            except (ConnectionError, OSError):
                return
            op = header.get("op")
            try:
                with self._lock:
                    if op == "load":
                        self.stage = None
                        if self.device.startswith("cuda"):
                            torch.cuda.set_device(torch.device(self.device))
                        self.stage = _Stage(header, self.device)
                        send_msg(sock, {"ok": True, "layers": header["layers"]})
                    elif op == "forward":
                        if self.stage is None:
                            raise RuntimeError("no layers loaded")
                        send_msg(sock, {"ok": True}, {"hidden": self.stage.forward(header, arrays)})
                    elif op == "capacity":
                        send_msg(sock, {"ok": True, "free_bytes": _free_bytes(self.device)})
                    elif op == "close":
                        send_msg(sock, {"ok": True})
                        return
                    else:
                        raise ValueError(f"unknown op {op!r}")
            except Exception as ex:  # report to the leader, keep serving
                log.exception("stage op %s failed", op)
                send_msg(sock, {"ok": False, "error": f"{type(ex).__name__}: {ex}"})

    def serve_forever(self):
        log.info("layer-split stage listening on %s:%d (%s)", *self.address, self.device)
        self.server.serve_forever()

    def start(self):
        t = threading.Thread(target=self.server.serve_forever, daemon=True, name="pp-stage")
        t.start()
        return self

    def shutdown(self):
        self.server.shutdown()
        self.server.server_close()


def _free_bytes(device: str) -> int:
    if device.startswith("cuda"):
        free, _ = torch.cuda.mem_get_info(torch.device(device))
        return int(free)
    import psutil
    return int(psutil.virtual_memory().available)


# ------------------------------------------------------------------------------------------------ leader
class RemoteStages:
    """Leader-side client: the layer ranges after the local one, in order."""

    def __init__(self, model_ref: str, addrs: list[str], ranges: list[tuple[int, int]], overrides=None,
                 timeout: float = 600.0):
        self.model_ref, self.ranges, self.overrides = model_ref, ranges, overrides or {}
        self.socks = []
        for a in addrs:
            host, port = a.rsplit(":", 1)
            s = socket.create_connection((host, int(port)), timeout=timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.socks.append(s)
        self.addrs = addrs

    def _call(self, i: int, header: dict, arrays: dict | None = None):
        send_msg(self.socks[i], header, arrays)
        rh, ra = recv_msg(self.socks[i])
        if not rh.get("ok"):
            raise RuntimeError(f"layer-split stage {self.addrs[i]}: {rh.get('error')}")
        return rh, ra

    def setup_kv(self, num_blocks: int, block_size: int, kv_dtype: str, max_tokens: int, max_seqs: int,
                 max_parts: int) -> int:
        """Load every stage's layers + KV cache with the leader's block count (same block ids)."""
        for i, (l0, l1) in enumerate(self.ranges):
            self._call(i, {"op": "load", "model": self.model_ref, "layers": [l0, l1], "num_blocks": num_blocks,
                           "block_size": block_size, "kv_dtype": kv_dtype, "max_tokens": max_tokens,
                           "max_seqs": max_seqs, "max_parts": max_parts, "overrides": self.overrides})
        return num_blocks

    def run(self, fb, h: torch.Tensor):
        plan = fb.plan
        arrays = {k: np.asarray(plan[k]) for k in _ARRAY_KEYS if k in plan}
        x = h.float().cpu().numpy()
        for i in range(len(self.socks)):
            arrays["hidden"] = x
            _, ra = self._call(i, {"op": "forward", "nd": int(plan["nd"])}, arrays)
            x = ra["hidden"]
        h.copy_(torch.from_numpy(np.ascontiguousarray(x)).to(h.device))

    def close(self):
        for i, s in enumerate(self.socks):
            try:
                self._call(i, {"op": "close"})
            except Exception:
                pass
            s.close()


def split_layers(n_layers: int, n_parts: int, weights: list[float] | None = None) -> list[tuple[int, int]]:
    """Contiguous layer ranges proportional to `weights` (llama.cpp tensor_split / free memory)."""
    w = np.asarray(weights if weights else [1.0] * n_parts, np.float64)
    cuts = np.round(np.cumsum(w) / w.sum() * n_layers).astype(int)
    out, prev = [], 0
    for c in cuts:
        c = max(prev + 1, min(int(c), n_layers - (n_parts - len(out) - 1)))
        out.append((prev, c))
        prev = c
    out[-1] = (out[-1][0], n_layers)
    return out


def load_split(model_ref: str, servers: list[str], device, tensor_split: list[float] | None = None, overrides=None):
    """-> (leader LlamaModel holding the first range + embedding/head, tokenizer, cfg, metadata).
    `servers`: "host:port" stages, in pipeline order (LLAMACPP_GRPC_SERVERS)."""
    from ..models.loader import _apply_overrides, _lora_attach, _lora_source, gguf_source, SYNTHETIC
    from ..models.llama import LlamaModel
    from ..tokenizer import ByteTokenizer, from_gguf
    md = {}
    if model_ref.startswith("synthetic:"):
        import copy
        from ..models.synthetic import synthetic_source
        cfg = copy.deepcopy(SYNTHETIC[model_ref.split(":", 1)[1]])
        _apply_overrides(cfg, overrides or {})
        src = synthetic_source(cfg, "Q4_K_M", seed=1)
        tok = ByteTokenizer(cfg.vocab)
    else:
        from ..formats.gguf import GGUFReader
        from ..models.config import LlamaConfig
        r = GGUFReader(model_ref)
        md = dict(r.metadata)
        cfg = LlamaConfig.from_gguf_metadata(md)
        _apply_overrides(cfg, overrides or {})
        src = gguf_source(r)
        try:
            tok = from_gguf(md)
        except Exception:
            tok = ByteTokenizer(cfg.vocab)
    ranges = split_layers(cfg.n_layers, 1 + len(servers), tensor_split)
    ov = overrides or {}
    m = _lora_attach(LlamaModel.load(cfg, _lora_source(src, ov, cfg), device, layer_range=ranges[0]), ov, cfg, 1,
                     ranges[0][0])
    m.remote = RemoteStages(model_ref, servers, ranges[1:], overrides)
    log.info("layer split: local %s, remote %s", ranges[0], list(zip(servers, ranges[1:])))
    return m, tok, cfg, md


def main(argv=None):
    import argparse
    import os
    ap = argparse.ArgumentParser(description="layer-split pipeline stage (llama.cpp rpc-server equivalent)")
    ap.add_argument("--host", default=os.environ.get("LLAMACPP_RPC_HOST", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("LLAMACPP_RPC_PORT", "50052")))
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("LOCALAI_LOG_LEVEL", "INFO").upper())
    StageServer(a.host, a.port, a.device).serve_forever()


if __name__ == "__main__":
    main()
