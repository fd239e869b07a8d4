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

Watchdog activity: only the owner runs the WatchDog, but SO_REUSEPORT hands most connections to the
siblings. Every attached process therefore reports its use of each replica address in a small per-process
activity file ({last use, requests in flight}, rewritten when the in-flight count changes and at most once a
second otherwise); the owner's idle / busy checks fold the live siblings' activity into its own before killing.
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

    # ---------------------------------------------------------------- watchdog activity of attached processes
    def _act_path(self, address: str, pid: int | None = None) -> str:
        h = hashlib.sha1(address.encode()).hexdigest()[:20]
        return os.path.join(self.root, f"{h}.act.{pid if pid is not None else self.pid}")

    def report(self, address: str, last: float, busy: int):
        p = self._act_path(address)
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"last": last, "busy": busy}, f)
        os.replace(tmp, p)

    def activity(self, address: str) -> tuple[float, bool]:
        """(latest use, any request in flight) of `address` over the live attached processes (not this one)."""
        prefix = os.path.basename(self._act_path(address, 0))[:-1]
        last, busy = 0.0, False
        try:
            names = os.listdir(self.root)
        except OSError:
            return last, busy
        for n in names:
            if not n.startswith(prefix) or n.endswith(".tmp"):
                continue
            try:
                pid = int(n[len(prefix):])
            except ValueError:
                continue
            if pid == self.pid or not _alive(pid):
                continue
            try:
                with open(os.path.join(self.root, n)) as f:
                    a = json.load(f)
            except (OSError, ValueError):
                continue
            last = max(last, float(a.get("last", 0.0)))
            busy = busy or int(a.get("busy", 0)) > 0
        return last, busy

    @staticmethod
    def same(a: dict | None, b: dict | None) -> bool:
        return bool(a and b and a["owner"] == b["owner"] and a["replicas"] == b["replicas"])


class ActivityReporter:
    """Watchdog stand-in for a client of an ATTACHED replica: mark / unmark report this process's use of the
    address to the owner through SharedBackends.report (the owner's WatchDog reads it)."""

    def __init__(self, shared: SharedBackends, min_interval: float = 1.0):
        self.shared, self.min_interval = shared, min_interval
        self._busy: dict[str, int] = {}
        self._sent: dict[str, float] = {}

    def _send(self, address: str, force: bool):
        now = time.time()
        if force or now - self._sent.get(address, 0.0) >= self.min_interval:
            self._sent[address] = now
            try:
                self.shared.report(address, now, self._busy.get(address, 0))
            except OSError:
                pass

    def mark(self, address: str):
        n = self._busy.get(address, 0)
        self._busy[address] = n + 1
        self._send(address, force=n == 0)

    def unmark(self, address: str):
        self._busy[address] = 0
        self._send(address, force=True)
