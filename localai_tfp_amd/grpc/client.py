"""Client side of the backend contract (reference: pkg/grpc/client.go).

Differences by design: one persistent channel per backend address (the reference dials a new
connection for every call, client.go:96-107), and calls are concurrent unless the backend config
asks for serialisation (`parallel=False` mirrors the reference's opMutex, client.go:53).
Busy/last-used bookkeeping feeds the WatchDog (pkg/model/watchdog.go)."""
from __future__ import annotations

import threading
import time

import grpc

from . import FULL_SERVICE, METHODS, pb
from .server import MAX_MSG


class BackendClient:
    def __init__(self, address: str, parallel: bool = True, watchdog=None):
        self.address = address
        self.parallel = parallel
        self.watchdog = watchdog
        self._chan = grpc.insecure_channel(address, options=[("grpc.max_send_message_length", MAX_MSG),
                                                             ("grpc.max_receive_message_length", MAX_MSG)])
        self._op_lock = threading.Lock()
        self._busy = 0
        self._bl = threading.Lock()
        self.last_used = time.time()
        self._stubs = {}
        for name, (_, req, resp, stream) in METHODS.items():
            path = f"/{FULL_SERVICE}/{name}"
            rs = getattr(pb, resp).FromString
            qs = getattr(pb, req).SerializeToString
            self._stubs[name] = (self._chan.unary_stream(path, request_serializer=qs, response_deserializer=rs)
                                 if stream else
                                 self._chan.unary_unary(path, request_serializer=qs, response_deserializer=rs))

    def close(self):
        self._chan.close()

    @property
    def busy(self) -> bool:
        return self._busy > 0

    def _enter(self):
        with self._bl:
            self._busy += 1
        self.last_used = time.time()
        if self.watchdog:
            self.watchdog.mark(self.address)

    def _exit(self):
        with self._bl:
            self._busy -= 1
        self.last_used = time.time()
        if self.watchdog and not self._busy:
            self.watchdog.unmark(self.address)

    def call(self, name: str, request, timeout: float | None = None, metadata=None):
        stub = self._stubs[name]
        self._enter()
        try:
            if self.parallel:
                return stub(request, timeout=timeout, metadata=metadata)
            with self._op_lock:
                return stub(request, timeout=timeout, metadata=metadata)
        finally:
            self._exit()

    def stream(self, name: str, request, timeout: float | None = None):
        stub = self._stubs[name]
        self._enter()
        lock = None if self.parallel else self._op_lock
        if lock:
            lock.acquire()
        try:
            yield from stub(request, timeout=timeout)
        finally:
            if lock:
                lock.release()
            self._exit()

    # convenience wrappers -------------------------------------------------------------------------
    def health(self, timeout: float = 10.0) -> bool:
        try:
            r = self._stubs["Health"](pb.HealthMessage(), timeout=timeout)
            return r.message == b"OK"
        except grpc.RpcError:
            return False

    def load_model(self, opts, timeout: float | None = None):
        return self.call("LoadModel", opts, timeout)

    def predict(self, opts, timeout=None):
        return self.call("Predict", opts, timeout)

    def predict_stream(self, opts, timeout=None):
        return self.stream("PredictStream", opts, timeout)

    def __getattr__(self, name):
        # pass-through for the remaining RPCs: client.Embedding(req), client.StoresFind(req), ...
        if name in METHODS:
            if METHODS[name][3]:
                return lambda req, timeout=None: self.stream(name, req, timeout)
            return lambda req, timeout=None: self.call(name, req, timeout)
        raise AttributeError(name)


class AsyncBackendClient:
    """grpc.aio twin of :class:`BackendClient` for the gateway's event loop (one channel per
    backend address and loop; streaming token replies never block a worker thread)."""

    def __init__(self, address: str, sync: BackendClient | None = None):
        import grpc.aio
        self.address = address
        self.sync = sync  # shares busy/last-used bookkeeping with the sync client (WatchDog)
        self._chan = grpc.aio.insecure_channel(address, options=[("grpc.max_send_message_length", MAX_MSG),
                                                                 ("grpc.max_receive_message_length", MAX_MSG)])
        self._stubs = {}
        for name, (_, req, resp, stream) in METHODS.items():
            path = f"/{FULL_SERVICE}/{name}"
            rs = getattr(pb, resp).FromString
            qs = getattr(pb, req).SerializeToString
            self._stubs[name] = (self._chan.unary_stream(path, request_serializer=qs, response_deserializer=rs)
                                 if stream else
                                 self._chan.unary_unary(path, request_serializer=qs, response_deserializer=rs))

    async def call(self, name: str, request, timeout: float | None = None):
        if self.sync:
            self.sync._enter()
        try:
            return await self._stubs[name](request, timeout=timeout)
        finally:
            if self.sync:
                self.sync._exit()

    async def stream(self, name: str, request, timeout: float | None = None):
        if self.sync:
            self.sync._enter()
        call = self._stubs[name](request, timeout=timeout)
        try:
            async for r in call:
                yield r
        finally:
            call.cancel()  # no-op when finished; aborts the backend request if the client went away
            if self.sync:
                self.sync._exit()

    async def close(self):
        await self._chan.close()
