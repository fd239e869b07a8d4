"""Backend process management: spawn/health/LoadModel, data-parallel replicas across GPUs, GPU
placement, external backends, single-active-backend, WatchDog.

Behavioural parity target:
  * pkg/model/loader.go:20-188    ModelLoader (models map, LoadModel under a mutex, CheckIsLoaded,
                                   ShutdownModel, StopAllGRPC)
  * pkg/model/initializers.go     backend aliases (:24-41), autodetect order (:498-559), external
                                   backends as address or executable (:307-331), spawn on a free port,
                                   20 x 2 s Health readiness loop, then LoadModel(ModelOptions) (:282-420)
  * pkg/model/process.go:21-158   child process lifecycle, stdout/stderr tailing, delete waits while busy
  * pkg/model/watchdog.go:19-156  busy / idle timeouts

MI355X-first differences: one worker process per GPU. A model config may ask for
``data_parallel: N`` replicas that are placed on N distinct GPUs through HIP_VISIBLE_DEVICES and
load-balanced by in-flight requests at the gateway (the reference's federated least-used routing,
core/p2p/federated.go:77, done intra-node). ``tensor_parallel_size: N`` workers are launched with
torch.distributed.run over N GPUs; rank 0 serves gRPC.
"""
from __future__ import annotations

import collections
import logging
import os
import socket
import subprocess
import sys
import threading
import time

from .. import workers as W
from ..grpc import pb
from ..grpc.client import BackendClient
from .options import model_options

log = logging.getLogger("localai_tfp_amd.loader")


class BackendLoadError(RuntimeError):
    pass


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> list[int]:
    env = os.environ.get("LOCALAI_GPUS") or os.environ.get("HIP_VISIBLE_DEVICES") or ""
    if env:
        return [int(x) for x in env.split(",") if x.strip().isdigit()]
    try:
        import torch
        return list(range(torch.cuda.device_count()))
    except Exception:
        return []


class Replica:
    """One worker process (or in-process server / external address) serving one model copy."""

    def __init__(self, address: str, client: BackendClient, proc: subprocess.Popen | None = None,
                 gpus: tuple = (), server=None, servicer=None):
        self.address, self.client, self.proc, self.gpus = address, client, proc, gpus
        self.server, self.servicer = server, servicer
        self.log_tail: collections.deque[str] = collections.deque(maxlen=200)
        self._aclients: dict[int, object] = {}
        self.mx_path = ""  # mxstream socket advertised by the worker's LoadModel reply
        self._mxclients: dict[int, object] = {}

    def mxclient(self):
        """Batched token channel (serving/mxstream.py) bound to the running loop, or None."""
        if not self.mx_path:
            return None
        import asyncio
        from .mxstream import StreamClient
        key = id(asyncio.get_running_loop())
        c = self._mxclients.get(key)
        if c is None:
            c = self._mxclients[key] = StreamClient(self.mx_path)
        return c

    def aclient(self):
        """Async client bound to the running event loop (gateway request path)."""
        import asyncio
        from ..grpc.client import AsyncBackendClient
        key = id(asyncio.get_running_loop())
        c = self._aclients.get(key)
        if c is None:
            c = self._aclients[key] = AsyncBackendClient(self.address, self.client)
        return c

    @property
    def inflight(self) -> int:
        return self.client._busy

    def alive(self) -> bool:
        return self.proc is None or self.proc.poll() is None

    def stop(self, force: bool = False, wait_busy_s: float = 120.0):
        # process.go deleteProcess: wait while the backend is busy unless forced
        t0 = time.time()
        while not force and self.client.busy and time.time() - t0 < wait_busy_s:
            time.sleep(0.25)
        try:
            self.client.close()
        except Exception:
            pass
        if self.server is not None:
            eng = getattr(self.servicer, "engine", None)
            if eng is not None and hasattr(eng, "shutdown"):
                eng.shutdown()
            self.server.stop()
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=15)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(timeout=5)


class LoadedModel:
    def __init__(self, name: str, backend: str, replicas: list[Replica]):
        self.name, self.backend, self.replicas = name, backend, replicas
        self._rr = 0
        self._lock = threading.Lock()
        self.shared: dict | None = None  # registry entry this process attached to (another gateway owns it)
        self._checked = 0.0

    def pick(self) -> BackendClient:
        return self.pick_replica().client

    def apick(self):
        return self.pick_replica().aclient()

    def pick_replica(self) -> Replica:
        """Least in-flight replica (ties round-robin)."""
        with self._lock:
            n = len(self.replicas)
            best = None
            for k in range(n):
                r = self.replicas[(self._rr + k) % n]
                if best is None or r.inflight < best.inflight:
                    best = r
            self._rr = (self._rr + 1) % n
            return best

    @property
    def client(self) -> BackendClient:
        return self.pick()

    def alive(self) -> bool:
        return all(r.alive() for r in self.replicas)

    def stop(self, force=False):
        for r in self.replicas:
            r.stop(force)


from .shared_backends import ActivityReporter  # noqa: E402


class WatchDog:
    """Kills backends busy for longer than busy_timeout or idle for longer than idle_timeout."""

    def __init__(self, loader: "ModelLoader", busy_timeout: float = 300.0, idle_timeout: float = 900.0,
                 busy_check: bool = True, idle_check: bool = True, interval: float = 30.0):
        self.loader = loader
        self.busy_timeout, self.idle_timeout = busy_timeout, idle_timeout
        self.busy_check, self.idle_check = busy_check, idle_check
        self.interval = interval
        self.busy_since: dict[str, float] = {}
        self.last_used: dict[str, float] = {}
        self.addr_model: dict[str, str] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._t: threading.Thread | None = None

    def add(self, address: str, model: str):
        with self._lock:
            self.addr_model[address] = model
            self.last_used[address] = time.time()

    def remove(self, address: str):
        with self._lock:
            self.addr_model.pop(address, None)
            self.busy_since.pop(address, None)
            self.last_used.pop(address, None)

    def mark(self, address: str):
        with self._lock:
            self.busy_since.setdefault(address, time.time())
            self.last_used[address] = time.time()

    def unmark(self, address: str):
        with self._lock:
            self.busy_since.pop(address, None)
            self.last_used[address] = time.time()

    def check_once(self, now: float | None = None) -> list[str]:
        now = now or time.time()
        victims = set()
        shared = getattr(self.loader, "shared", None)
        with self._lock:
            if self.busy_check:
                for a, t in self.busy_since.items():
                    if now - t > self.busy_timeout:
                        log.warning("watchdog: %s busy for %.0fs, killing", a, now - t)
                        victims.add(self.addr_model.get(a))
            if self.idle_check:
                for a, t in self.last_used.items():
                    if a in self.busy_since:
                        continue
                    if shared is not None and now - t > self.idle_timeout:
                        # sibling gateway processes serve this replica too: their use counts
                        s_last, s_busy = shared.activity(a)
                        if s_busy:
                            continue
                        t = max(t, s_last)
                    if now - t > self.idle_timeout:
                        log.warning("watchdog: %s idle for %.0fs, killing", a, now - t)
                        victims.add(self.addr_model.get(a))
        victims.discard(None)
        for m in victims:
            self.loader.shutdown_model(m, force=True)
        return sorted(victims)

    def start(self):
        if self._t is None:
            self._t = threading.Thread(target=self._run, daemon=True, name="watchdog")
            self._t.start()

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self.check_once()
            except Exception:
                log.exception("watchdog check failed")

    def stop(self):
        self._stop.set()


def _module_for(backend: str) -> str:
    mod = W.WORKERS.get(W.resolve(backend))
    if mod is None:
        raise BackendLoadError(f"unknown backend {backend!r}")
    return mod


def guess_backend(cfg, model_path: str) -> list[str]:
    """Candidate backends when the config names none (initializers.go:498-559 tries them all)."""
    m = cfg.parameters.model or ""
    full = os.path.join(model_path, m)
    low = m.lower()
    if low.startswith("synthetic:"):
        return ["bert-embeddings"] if low.startswith("synthetic:bert") else ["llama-cpp"]
    if low.endswith(".onnx"):
        return ["piper", "silero-vad"]
    if low.endswith(".gguf") and os.path.isfile(full):
        try:
            from ..formats.gguf import GGUFReader
            arch = str(GGUFReader(full).metadata.get("general.architecture", ""))
            if arch in ("bert", "nomic-bert", "jina-bert-v2"):
                return ["bert-embeddings"]
            if arch == "whisper":
                return ["whisper"]
        except Exception:
            pass
        return ["llama-cpp"]
    if "whisper" in low or low.startswith("ggml-"):
        return ["whisper", "llama-cpp"]
    return list(W.AUTODETECT_ORDER)


class ModelLoader:
    def __init__(self, app, inproc: bool | None = None):
        self.app = app
        self.models: dict[str, LoadedModel] = {}
        self._lock = threading.RLock()
        self._loading: dict[str, threading.Lock] = collections.defaultdict(threading.Lock)
        self.inproc = inproc if inproc is not None else os.environ.get("LOCALAI_INPROC_BACKENDS", "") == "1"
        self.gpus = visible_gpus()
        self._gpu_load: dict[int, int] = {g: 0 for g in self.gpus}
        # multi-process gateway (cli.py --gateway-workers): backends shared with the sibling gateway processes
        reg = os.environ.get("LOCALAI_BACKEND_REGISTRY", "")
        self.shared = None
        if reg:
            from .shared_backends import SharedBackends
            self.shared = SharedBackends(reg)
            if getattr(app, "watchdog_idle", False):
                log.info("watchdog: idle checks of shared replicas include the sibling gateway processes' activity")
        self.watchdog: WatchDog | None = None
        if getattr(app, "watchdog_busy", False) or getattr(app, "watchdog_idle", False):
            self.watchdog = WatchDog(self, app.watchdog_busy_timeout_s, app.watchdog_idle_timeout_s,
                                     app.watchdog_busy, app.watchdog_idle)
            self.watchdog.start()

    # ------------------------------------------------------------------ queries
    def get(self, name: str) -> LoadedModel | None:
        with self._lock:
            m = self.models.get(name)
        if m is not None and m.shared is not None and time.time() - m._checked > 1.0:
            m._checked = time.time()
            if not self.shared.same(self.shared.read(name), m.shared):
                log.info("shared backend for %s was unloaded by its owner; detaching", name)
                self.shutdown_model(name, force=True)
                return None
        if m is not None and not m.alive():
            log.warning("backend for %s died; removing", name)
            self.shutdown_model(name, force=True)
            return None
        return m

    def list_loaded(self) -> list[str]:
        with self._lock:
            return sorted(self.models)

    def check_is_loaded(self, name: str) -> LoadedModel | None:
        m = self.get(name)
        if m is None:
            return None
        if not all(r.client.health(timeout=120) for r in m.replicas):
            log.warning("backend for %s failed health check; removing", name)
            self.shutdown_model(name, force=True)
            return None
        return m

    # ------------------------------------------------------------------ load
    def load(self, cfg, backend: str | None = None) -> LoadedModel:
        name = cfg.name or cfg.parameters.model
        m = self.get(name)
        if m is not None:
            return m
        with self._loading[name]:
            m = self.get(name)
            if m is not None:
                return m
            if getattr(self.app, "single_active_backend", False):
                for other in self.list_loaded():
                    self.shutdown_model(other)
            if self.shared is not None:
                with self.shared.locked(name):
                    e = self.shared.read(name)
                    if e is not None and e["owner"] != self.shared.pid:
                        m = self._attach(name, e)
                    else:
                        m = self._load_candidates(cfg, name, backend)
                        self.shared.publish(name, m.backend, m.replicas)
            else:
                m = self._load_candidates(cfg, name, backend)
            with self._lock:
                self.models[name] = m
            return m

    def _attach(self, name: str, e: dict) -> LoadedModel:
        """Clients to the replicas another gateway process published (it owns and stops them)."""
        parallel = bool(getattr(self.app, "parallel_backend_requests", True))
        reps = []
        for r in e["replicas"]:
            rep_ = Replica(r["address"], BackendClient(r["address"], parallel=parallel,
                                                       watchdog=ActivityReporter(self.shared)))
            rep_.mx_path = r["mx_path"] if r["mx_path"] and os.path.exists(r["mx_path"]) else ""
            reps.append(rep_)
        m = LoadedModel(name, e["backend"], reps)
        m.shared, m._checked = e, time.time()
        log.info("attached %s: %d replica(s) owned by gateway process %d", name, len(reps), e["owner"])
        return m

    def _load_candidates(self, cfg, name: str, backend: str | None) -> LoadedModel:
        cands = [backend or cfg.backend] if (backend or cfg.backend) else guess_backend(cfg, self.app.models_path)
        errs = []
        for b in cands:
            try:
                m = self._load_with(cfg, name, b)
                break
            except Exception as ex:
                errs.append(f"{b}: {ex}")
                log.warning("loading %s with %s failed: %s", name, b, ex)
        else:
            raise BackendLoadError(f"could not load model {name!r}: " + "; ".join(errs))
        return m

    def _assign_gpus(self, n: int) -> list[int]:
        if not self.gpus:
            return []
        order = sorted(self.gpus, key=lambda g: (self._gpu_load[g], g))
        got = order[:n] if n <= len(order) else [order[i % len(order)] for i in range(n)]
        for g in got:
            self._gpu_load[g] += 1
        return got

    def _release_gpus(self, gpus):
        for g in gpus:
            if g in self._gpu_load:
                self._gpu_load[g] = max(0, self._gpu_load[g] - 1)

    def _load_with(self, cfg, name: str, backend: str) -> LoadedModel:
        backend = W.resolve(backend)
        opts = model_options(cfg, self.app, self.app.models_path)
        if backend == "piper":  # pkg/model/initializers.go:451-453: espeak-ng data under the backend assets
            opts.LibrarySearchPath = os.path.join(getattr(self.app, "backend_assets_path", "") or "",
                                                  "backend-assets", "espeak-ng-data")
        ext = (getattr(self.app, "external_grpc_backends", None) or {}).get(backend)
        parallel = bool(getattr(self.app, "parallel_backend_requests", True))
        tp = max(1, int(cfg.tensor_parallel_size or 1))
        dp = max(1, int(getattr(cfg, "data_parallel", 0) or 1))
        replicas: list[Replica] = []
        try:
            if ext and ":" in ext and not os.path.exists(ext):
                # external backend at fixed address(es): no process to manage; "host:port|host:port|..." lists
                # externally started data-parallel replicas of one model
                for addr in ext.split("|"):
                    replicas.append(self._connect(addr.strip(), parallel))
            else:
                for _ in range(dp):
                    gpus = tuple(self._assign_gpus(tp))
                    if self.inproc and tp == 1:
                        replicas.append(self._start_inproc(backend, parallel, gpus))
                    else:
                        replicas.append(self._spawn(backend, ext, parallel, gpus, tp))
            attempts = cfg.grpc.attempts or 20
            sleep = cfg.grpc.attempts_sleep_time or 2
            for r in replicas:
                self._wait_healthy(r, attempts, sleep)
                res = r.client.load_model(opts)
                if not res.success:
                    raise BackendLoadError(res.message or "LoadModel failed")
                for part in (res.message or "").split(";"):
                    k, _, v = part.strip().partition("=")
                    if k == "mxstream" and v and os.path.exists(v):
                        r.mx_path = v
                if self.watchdog:
                    self.watchdog.add(r.address, name)
                    r.client.watchdog = self.watchdog
        except Exception:
            for r in replicas:
                r.stop(force=True)
                self._release_gpus(r.gpus)
            raise
        log.info("loaded %s with backend %s (%d replica(s), tp=%d)", name, backend, len(replicas), tp)
        return LoadedModel(name, backend, replicas)

    def _connect(self, address: str, parallel: bool) -> Replica:
        return Replica(address, BackendClient(address, parallel=parallel))

    def _start_inproc(self, backend: str, parallel: bool, gpus) -> Replica:
        import importlib
        from ..grpc.server import AioServer
        mod = importlib.import_module(_module_for(backend))
        servicer_cls = next(getattr(mod, n) for n in dir(mod) if n.endswith("Servicer") and n != "BackendServicer")
        dev = None
        if gpus:
            dev = f"cuda:{gpus[0]}"
        try:
            svc = servicer_cls(device=dev)
        except TypeError:
            svc = servicer_cls()
        if hasattr(svc, "backend"):
            svc.backend = backend
        server = AioServer(svc, "127.0.0.1:0")
        addr = f"127.0.0.1:{server.port}"
        return Replica(addr, BackendClient(addr, parallel=parallel), None, tuple(gpus), server, svc)

    def _spawn(self, backend: str, ext: str | None, parallel: bool, gpus, tp: int) -> Replica:
        port = free_port()
        addr = f"127.0.0.1:{port}"
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["MX_BACKEND_NAME"] = backend
        if gpus:
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
        if ext:  # external backend executable: `<file> --addr host:port`
            cmd = [ext, "--addr", addr]
        elif tp > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tp}",
                   "--master-addr", "127.0.0.1", f"--master-port={free_port()}", "-m", _module_for(backend),
                   "--addr", addr]
        else:
            cmd = [sys.executable, "-m", _module_for(backend), "--addr", addr]
        log.info("spawning %s on %s (gpus=%s)", backend, addr, gpus or "-")
        proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                start_new_session=True)
        r = Replica(addr, BackendClient(addr, parallel=parallel), proc, tuple(gpus))

        def tail():
            for line in proc.stdout:
                line = line.rstrip()
                r.log_tail.append(line)
                log.debug("[%s] %s", addr, line)
        threading.Thread(target=tail, daemon=True, name=f"tail-{port}").start()
        return r

    def _wait_healthy(self, r: Replica, attempts: int, sleep: float):
        for i in range(attempts):
            if not r.alive():
                raise BackendLoadError(f"backend process exited: {' | '.join(list(r.log_tail)[-5:])}")
            if r.client.health(timeout=max(2.0, sleep)):
                return
            time.sleep(sleep)
        raise BackendLoadError(f"backend at {r.address} not healthy after {attempts} attempts")

    # ------------------------------------------------------------------ shutdown
    def shutdown_model(self, name: str, force: bool | None = None) -> bool:
        with self._lock:
            m = self.models.pop(name, None)
        if m is None:
            return False
        force = force if force is not None else getattr(self.app, "force_backend_shutdown", False)
        if m.shared is not None:  # attached: the owning gateway process stops the workers
            for r in m.replicas:
                try:
                    r.client.close()
                except Exception:
                    pass
            return True
        if self.shared is not None:
            self.shared.withdraw(name)
        for r in m.replicas:
            if self.watchdog:
                self.watchdog.remove(r.address)
            r.stop(force)
            self._release_gpus(r.gpus)
        return True

    def stop_all(self):
        for n in self.list_loaded():
            self.shutdown_model(n, force=True)
        if self.watchdog:
            self.watchdog.stop()

    def status(self, name: str):
        m = self.get(name)
        if m is None:
            return None
        return m.pick().Status(pb.HealthMessage(), timeout=10)
