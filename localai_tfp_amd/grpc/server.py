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
import grpc.aio  # noqa: F401  (registers grpc.aio)
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


# ------------------------------------------------------------------------------------------------
# asyncio server: one event-loop thread multiplexes every stream (no thread per PredictStream);
# servicer methods may be coroutines / async generators, plain methods run in a thread pool.

class _Abort(Exception):
    def __init__(self, code, details):
        super().__init__(details)
        self.code, self.details = code, details


class _SyncCtx:
    """What a plain (thread-pool) handler sees instead of the grpc.aio context: abort() raises,
    the async wrapper turns it into the real abort on the event loop."""

    def __init__(self, ctx):
        self._ctx = ctx

    def abort(self, code, details=""):
        raise _Abort(code, details)

    def add_callback(self, fn):
        self._ctx.add_done_callback(lambda _c: fn())
        return True

    def is_active(self):
        return not self._ctx.done()

    def __getattr__(self, name):
        return getattr(self._ctx, name)


def aio_generic_handler(servicer: BackendServicer, executor):
    import asyncio
    import inspect

    handlers = {}
    for name, (mname, req, resp, stream) in METHODS.items():
        req_cls, resp_cls = getattr(pb, req), getattr(pb, resp)
        fn = getattr(servicer, name, None)
        if fn is None:
            async def h(request, context, _n=name):
                await context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{_n} not implemented by this backend")
            stream_h = None
        elif stream:
            if inspect.isasyncgenfunction(fn):
                async def stream_h(request, context, _fn=fn):
                    servicer._busy += 1
                    try:
                        async for r in _fn(request, context):
                            yield r
                    finally:
                        servicer._busy -= 1
            else:
                async def stream_h(request, context, _fn=fn):
                    loop = asyncio.get_running_loop()
                    servicer._busy += 1
                    try:
                        sc = _SyncCtx(context)
                        it = await loop.run_in_executor(executor, lambda: iter(_fn(request, sc)))
                        sentinel = object()
                        while True:
                            r = await loop.run_in_executor(executor, next, it, sentinel)
                            if r is sentinel:
                                break
                            yield r
                    except _Abort as ab:
                        await context.abort(ab.code, ab.details)
                    finally:
                        servicer._busy -= 1
        else:
            if inspect.iscoroutinefunction(fn):
                async def h(request, context, _fn=fn):
                    servicer._busy += 1
                    try:
                        return await _fn(request, context)
                    finally:
                        servicer._busy -= 1
            else:
                async def h(request, context, _fn=fn):
                    servicer._busy += 1
                    sc = _SyncCtx(context)

                    def call():
                        if servicer.locking:
                            with servicer._lock:
                                return _fn(request, sc)
                        return _fn(request, sc)
                    try:
                        return await asyncio.get_running_loop().run_in_executor(executor, call)
                    except _Abort as ab:
                        await context.abort(ab.code, ab.details)
                    finally:
                        servicer._busy -= 1
        if stream:
            if fn is None:
                async def stream_h(request, context, _n=name):
                    await context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{_n} not implemented by this backend")
                    yield None  # pragma: no cover
            handlers[name] = grpc.unary_stream_rpc_method_handler(
                stream_h, request_deserializer=req_cls.FromString, response_serializer=resp_cls.SerializeToString)
        else:
            handlers[name] = grpc.unary_unary_rpc_method_handler(
                h, request_deserializer=req_cls.FromString, response_serializer=resp_cls.SerializeToString)
    return grpc.method_handlers_generic_handler(FULL_SERVICE, handlers)


class AioServer:
    """grpc.aio server on a private event-loop thread (used by workers and in-process backends)."""

    def __init__(self, servicer: BackendServicer, addr: str, max_workers: int | None = None):
        import asyncio
        self.servicer = servicer
        self.loop = asyncio.new_event_loop()
        self.executor = futures.ThreadPoolExecutor(
            max_workers=max_workers or int(os.environ.get("PYTHON_GRPC_MAX_WORKERS", "64")))
        self._ready = threading.Event()
        self._err = None
        self.port = 0
        self.addr = addr
        self._t = threading.Thread(target=self._run, daemon=True, name="grpc-aio")
        self._t.start()
        self._ready.wait()
        if self._err:
            raise self._err

    def _run(self):
        import asyncio
        asyncio.set_event_loop(self.loop)
        servicer = self.servicer
        servicer.loop = self.loop

        async def start():
            self.server = grpc.aio.server(options=[("grpc.max_send_message_length", MAX_MSG),
                                                   ("grpc.max_receive_message_length", MAX_MSG),
                                                   ("grpc.so_reuseport", 0)])
            self.server.add_generic_rpc_handlers((aio_generic_handler(servicer, self.executor),))
            self.port = self.server.add_insecure_port(self.addr)
            if self.port == 0:
                raise RuntimeError(f"could not bind {self.addr}")
            servicer.bound_addr = f"{self.addr.rsplit(':', 1)[0]}:{self.port}"
            await self.server.start()
        try:
            self.loop.run_until_complete(start())
        except Exception as ex:
            self._err = ex
            self._ready.set()
            return
        self._ready.set()
        self.loop.run_forever()

    def stop(self, grace: float = 0):
        import asyncio
        if not self.loop.is_running():
            return
        fut = asyncio.run_coroutine_threadsafe(self.server.stop(grace), self.loop)
        try:
            fut.result(timeout=grace + 5)
        except Exception:
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)
        self._t.join(timeout=5)
        self.executor.shutdown(wait=False)


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
    server = AioServer(servicer, addr, max_workers)
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
    server.stop(grace=2)
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
