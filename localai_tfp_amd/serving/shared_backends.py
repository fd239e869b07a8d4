"""Cross-process registry of running backends, for the multi-process gateway (`local-ai run --gateway-workers N`).

One Python gateway process carries ~20k SSE chunks/s (uvicorn's h11 HTTP/1.1 and the per-chunk ASGI send are
pure Python; profiles/r5_gateway_capacity.md) — less than a single MI355X produces at c128, and an eighth of what
`data_parallel: 8` needs. The reference's Go gateway is multi-threaded (core/http/app.go:53); the MI355X form is N
gateway processes accepting on one SO_REUSEPORT socket that SHARE the model's worker processes instead of
spawning their own (which would load every model N times):

* the first process to load a model spawns its replicas as usual (it owns them: watchdog, unload, shutdown) and
  publishes `{owner pid, backend, replicas: [{address, mxstream socket}]}` here;
* every other process attaches to the published replicas (gRPC clients + its own mxstream connection per worker
  — a worker's mxstream server takes any number of gateway connections) and never stops them;
* an attached process re-validates the entry at most once per second and drops its clients when the owner
  unloaded the model or exited (the next request then loads / attaches again).

Entries are JSON files updated under an fcntl lock per model, so concurrent first requests in two processes still
spawn the model once.
"""
from __future__ import annotations

import contextlib
import fcntl
import hashlib
import json
import os
import time


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


class SharedBackends:
    def __init__(self, root: str):
        self.root = root
        os.makedirs(root, exist_ok=True)
        self.pid = os.getpid()

    def _path(self, name: str) -> str:
        return os.path.join(self.root, hashlib.sha1(name.encode()).hexdigest()[:20] + ".json")

    @contextlib.contextmanager
    def locked(self, name: str):
        with open(self._path(name) + ".lock", "a") as f:
            fcntl.flock(f, fcntl.LOCK_EX)
            try:
                yield
            finally:
                fcntl.flock(f, fcntl.LOCK_UN)

    def read(self, name: str) -> dict | None:
        """The live entry of `name` (owner process running), else None."""
        try:
            with open(self._path(name)) as f:
                e = json.load(f)
        except (OSError, ValueError):
            return None
        if e.get("name") != name or not _alive(int(e.get("owner", 0))):
            return None
        return e

    def publish(self, name: str, backend: str, replicas) -> dict:
        e = {"name": name, "owner": self.pid, "backend": backend, "t": time.time(),
             "replicas": [{"address": r.address, "mx_path": r.mx_path} for r in replicas]}
        p = self._path(name)
        tmp = f"{p}.{self.pid}.tmp"
        with open(tmp, "w") as f:
            json.dump(e, f)
        os.replace(tmp, p)
        return e

    def withdraw(self, name: str):
        """Remove `name`'s entry if this process owns it."""
        with self.locked(name):
            try:
                with open(self._path(name)) as f:
                    e = json.load(f)
            except (OSError, ValueError):
                return
            if int(e.get("owner", 0)) == self.pid:
                with contextlib.suppress(OSError):
                    os.unlink(self._path(name))

    @staticmethod
    def same(a: dict | None, b: dict | None) -> bool:
        return bool(a and b and a["owner"] == b["owner"] and a["replicas"] == b["replicas"])
