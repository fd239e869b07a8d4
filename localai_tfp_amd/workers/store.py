"""local-store worker: in-memory vector store over the native store (csrc/runtime/store.cpp).

Behavioural parity: backend/go/stores/store.go:1-511 — StoresSet merge-insert (overwrite on equal
key), StoresDelete, StoresGet (missing keys skipped), StoresFind (cosine top-k, unit-norm fast
path). The reference is a sorted Go slice with a heap; here the rows live in one contiguous
float32 matrix in C++ so top-k is a single blocked GEMV + partial sort."""
from __future__ import annotations

import threading

import numpy as np

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main
from ..runtime_native import NativeStore


class StoreServicer(BackendServicer):
    def __init__(self, device=None):
        super().__init__()
        self.store = NativeStore()
        self._lock = threading.RLock()

    def LoadModel(self, request, context):
        return pb.Result(message="store ready", success=True)

    @staticmethod
    def _keys(ks):
        if not len(ks):
            return np.zeros((0, 0), np.float32)
        return np.asarray([list(k.Floats) for k in ks], np.float32)

    def StoresSet(self, request, context):
        if len(request.Keys) != len(request.Values):
            return pb.Result(message="keys and values must have the same length", success=False)
        if not len(request.Keys):
            return pb.Result(message="no keys", success=False)
        try:
            with self._lock:
                self.store.set(self._keys(request.Keys), [v.Bytes for v in request.Values])
        except ValueError as ex:
            return pb.Result(message=str(ex), success=False)
        return pb.Result(success=True)

    def StoresDelete(self, request, context):
        with self._lock:
            if len(self.store) and len(request.Keys):
                self.store.delete(self._keys(request.Keys))
        return pb.Result(success=True)

    def StoresGet(self, request, context):
        with self._lock:
            if not len(self.store) or not len(request.Keys):
                return pb.StoresGetResult()
            ks, vs = self.store.get(self._keys(request.Keys))
        return pb.StoresGetResult(Keys=[pb.StoresKey(Floats=k.tolist()) for k in ks],
                                  Values=[pb.StoresValue(Bytes=v) for v in vs])

    def StoresFind(self, request, context):
        q = np.asarray(list(request.Key.Floats), np.float32)
        with self._lock:
            if not len(self.store):
                return pb.StoresFindResult()
            if q.size != self.store.dim:
                context.abort(3, f"key dimension {q.size} does not match store dimension {self.store.dim}")
            ks, vs, sims = self.store.find(q, max(1, int(request.TopK)))
        return pb.StoresFindResult(Keys=[pb.StoresKey(Floats=k.tolist()) for k in ks],
                                   Values=[pb.StoresValue(Bytes=v) for v in vs], Similarities=sims)


def main(argv=None):
    worker_main(StoreServicer, argv)


if __name__ == "__main__":
    main()
