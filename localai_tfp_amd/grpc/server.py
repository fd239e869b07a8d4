"""Serving side of the backend contract.

`BackendServicer` is the base every worker subclasses (LLM, embeddings, whisper, SD, stores, VAD,
TTS). Unimplemented RPCs answer UNIMPLEMENTED (reference: pkg/grpc/server.go falls through the
same way for Rerank/GetMetrics). `Status` defaults to READY/BUSY with RSS memory — the
reference's base.SingleThread behaviour (pkg/grpc/base/singlethread.go:13-52). Workers are
multi-request by default (`parallel = True`); `locking` workers serialise calls like the
reference's Go backends that return Locking() = true (pkg/grpc/server.go:33-36).
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
from concurrent import futures

import grpc

from . import FULL_SERVICE, METHODS, pb

MAX_MSG = 50 * 1024 * 1024  # 50 MB, as grpc-server.cpp:2641-2653 / pkg/grpc/client.go
log = logging.getLogger("localai_tfp_amd.grpc")


class BackendServicer:
    locking = False

    def __init__(self):
        self._lock = threading.Lock()
        self._busy = 0
        self._busy_lock = threading.Lock()

    # default implementations ------------------------------------------------------------------
    def Health(self, request, context):
        return pb.Reply(message=b"OK")

    def Status(self, request, context):
        try:
            import psutil
            rss = psutil.Process().memory_info().rss
        except Exception:
            rss = 0
        st = pb.STATE_BUSY if self._busy else pb.STATE_READY
        mem = pb.MemoryUsageData(total=rss)
        mem.breakdown["rss"] = rss
        return pb.StatusResponse(state=st, memory=mem)

    # plumbing -----------------------------------------------------------------------------------
    def _wrap_unary(self, fn):
        def h(req, ctx):
            with self._busy_lock:
                self._busy += 1
            try:
                if self.locking:
                    with self._lock:
                        return fn(req, ctx)
                return fn(req, ctx)
            finally:
                with self._busy_lock:
                    self._busy -= 1
        return h

    def _wrap_stream(self, fn):
        def h(req, ctx):
            with self._busy_lock:
                self._busy += 1
            try:
                if self.locking:
                    with self._lock:
                        yield from fn(req, ctx)
                else:
                    yield from fn(req, ctx)
            finally:
                with self._busy_lock:
                    self._busy -= 1
        return h

    def generic_handler(self):
        handlers = {}
        for name, (mname, req, resp, stream) in METHODS.items():
            req_cls, resp_cls = getattr(pb, req), getattr(pb, resp)
            fn = getattr(self, name, None)
            if fn is None:
                def fn(request, context, _n=name):
                    context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{_n} not implemented by this backend")
            if stream:
                handlers[name] = grpc.unary_stream_rpc_method_handler(
                    self._wrap_stream(fn), request_deserializer=req_cls.FromString,
                    response_serializer=resp_cls.SerializeToString)
            else:
                handlers[name] = grpc.unary_unary_rpc_method_handler(
                    self._wrap_unary(fn), request_deserializer=req_cls.FromString,
                    response_serializer=resp_cls.SerializeToString)
        return grpc.method_handlers_generic_handler(FULL_SERVICE, handlers)


def make_server(servicer: BackendServicer, addr: str, max_workers: int | None = None):
    max_workers = max_workers or int(os.environ.get("PYTHON_GRPC_MAX_WORKERS", "64"))
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_send_message_length", MAX_MSG),
                                  ("grpc.max_receive_message_length", MAX_MSG),
                                  ("grpc.so_reuseport", 0)])
    server.add_generic_rpc_handlers((servicer.generic_handler(),))
    port = server.add_insecure_port(addr)
    if port == 0:
        raise RuntimeError(f"could not bind {addr}")
    return server, port


def serve(servicer: BackendServicer, addr: str, max_workers: int | None = None, block: bool = True):
    server, port = make_server(servicer, addr, max_workers)
    server.start()
    log.info("backend %s listening on %s", type(servicer).__name__, addr)
    if not block:
        return server
    stop = threading.Event()

    def _sig(*_):
        stop.set()

    for s in (signal.SIGTERM, signal.SIGINT):
        try:
            signal.signal(s, _sig)
        except ValueError:
            pass
    while not stop.wait(0.5):
        pass
    server.stop(grace=2).wait()
    return server


def worker_main(servicer_factory, argv=None):
    """`python -m localai_tfp_amd.workers.<x> --addr host:port` entry (reference workers take
    the same flag: grpc-server.cpp:2655-2690, backend/python/*/backend.py)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--addr", default="127.0.0.1:50051")
    args, _ = ap.parse_known_args(argv)
    logging.basicConfig(level=os.environ.get("LOCALAI_LOG_LEVEL", "INFO").upper(),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    serve(servicer_factory(), args.addr)
