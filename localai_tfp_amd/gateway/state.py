"""Gateway application state and bootstrap (behavioural parity: core/application/startup.go:20-164,
application.go:9-39, config_file_watcher.go:29-180, services/list_models.go:17-63)."""
from __future__ import annotations

import json
import logging
import os
import threading
import time

from ..config.app_config import ApplicationConfig
from ..config.loader import ModelConfigLoader
from ..config.model_config import FLAG_ANY
from ..serving.model_loader import ModelLoader
from ..templates.evaluator import Evaluator
from .inference import Inference

log = logging.getLogger("localai_tfp_amd.gateway")

# list_models.go LOOSE_ONLY / SKIP_IF_CONFIGURED / SKIP_ALWAYS / ALWAYS_INCLUDE
SKIP_IF_CONFIGURED, SKIP_ALWAYS, ALWAYS_INCLUDE, LOOSE_ONLY = 0, 1, 2, 3


class JSONStore:
    """Tiny persisted list (files / assistants metadata), like utils.SaveConfig/ReadConfig."""

    def __init__(self, path: str):
        self.path = path
        self.items: list[dict] = []
        self._lock = threading.Lock()
        try:
            with open(path) as f:
                self.items = json.load(f)
        except (FileNotFoundError, ValueError):
            self.items = []

    def save(self):
        with self._lock:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(self.items, f)
            os.replace(tmp, self.path)


class Application:
    def __init__(self, cfg: ApplicationConfig | None = None, inproc: bool | None = None):
        self.cfg = cfg or ApplicationConfig()
        c = self.cfg
        c.ensure_dirs()
        self.configs = ModelConfigLoader(c.models_path, c.context_size, c.threads, c.f16, c.debug)
        self.configs.load_from_path()
        if c.config_file and os.path.exists(c.config_file):
            self.configs.load_multiple_single_file(c.config_file)
        self.loader = ModelLoader(c, inproc)
        self.evaluator = Evaluator(c.models_path)
        self.inference = Inference(self)
        from ..gallery import GalleryService
        self.gallery = GalleryService(c.models_path, c.galleries, on_change=self.reload_configs,
                                      enforce_scan=c.enforce_predownload_scans)
        self.files = JSONStore(os.path.join(c.upload_dir, "uploadedFiles.json"))
        self.assistants = JSONStore(os.path.join(c.config_dir, "assistants.json"))
        self.assistant_files = JSONStore(os.path.join(c.config_dir, "assistantsFile.json"))
        self.api_keys = list(c.api_keys)
        self._file_keys: list[str] = []
        self.started = time.time()
        self._watch_stop = threading.Event()
        self.p2p = None
        if c.p2p:
            from .. import p2p as P
            if not c.p2p_token:
                c.p2p_token = P.generate_token(c.p2p_dht_interval, c.p2p_otp_interval)
                log.info("p2p enabled without a token; generated network token: %s", c.p2p_token)
            me = P.self_node(c.address, P.FEDERATED_ID if c.federated else P.WORKER_ID)
            self.p2p = P.P2PNode(c.p2p_token, c.p2p_network_id, list(c.p2p_peers), me,
                                 lan_discovery=c.p2p_lan_discovery, discovery_targets=list(c.p2p_discovery_targets))

    # ------------------------------------------------------------------ startup
    def startup(self):
        c = self.cfg
        for m in c.models:  # `run <url|gallery-id>` positional args (pkg/startup/model_preload.go)
            try:
                from .startup import install_models
                install_models(self, [m])
            except Exception as ex:
                log.error("failed to install %s: %s", m, ex)
        try:
            self.configs.preload()
        except Exception as ex:
            log.error("preload failed: %s", ex)
        self._load_dynamic_config()
        threading.Thread(target=self._watch_config_dir, daemon=True, name="config-watch").start()
        for name in c.load_to_memory:
            cfg = self.configs.load_by_name(name)
            log.info("loading %s into memory", name)
            self.loader.load(cfg)

    def reload_configs(self):
        self.configs.load_from_path()

    def _load_dynamic_config(self):
        """config_dir/api_keys.json and external_backends.json are hot-reloaded (config_file_watcher.go)."""
        d = self.cfg.config_dir
        try:
            with open(os.path.join(d, "api_keys.json")) as f:
                keys = json.load(f)
            self._file_keys = [k for k in keys if isinstance(k, str)]
        except (FileNotFoundError, ValueError):
            self._file_keys = []
        try:
            with open(os.path.join(d, "external_backends.json")) as f:
                eb = json.load(f)
            if isinstance(eb, dict):
                self.cfg.external_grpc_backends.update(eb)
        except (FileNotFoundError, ValueError):
            pass

    def _watch_config_dir(self):
        last = None
        d = self.cfg.config_dir
        while not self._watch_stop.wait(2.0):
            try:
                st = tuple(os.path.getmtime(os.path.join(d, f)) if os.path.exists(os.path.join(d, f)) else 0
                           for f in ("api_keys.json", "external_backends.json"))
            except OSError:
                continue
            if st != last:
                last = st
                self._load_dynamic_config()

    @property
    def all_api_keys(self) -> list[str]:
        return self.api_keys + self._file_keys

    def shutdown(self):
        self._watch_stop.set()
        if self.p2p is not None:
            self.p2p.stop()
        self.gallery.close()
        self.loader.stop_all()

    # ------------------------------------------------------------------ listing
    def list_models(self, flt=None, policy: int = SKIP_IF_CONFIGURED) -> list[str]:
        flt = flt or (lambda _c: True)
        names = []
        seen = set()
        if policy != LOOSE_ONLY:
            for c in self.configs.all():
                if flt(c):
                    names.append(c.name)
                seen.add(c.name)
                seen.add(c.parameters.model)
        if policy in (SKIP_IF_CONFIGURED, ALWAYS_INCLUDE, LOOSE_ONLY):
            for f in self.configs.loose_model_files():
                if policy == ALWAYS_INCLUDE or f not in seen:
                    if f not in names:
                        names.append(f)
        return names

    def model_exists(self, name: str) -> bool:
        return name in self.list_models(policy=ALWAYS_INCLUDE) or self.loader.get(name) is not None

    def first_model_for(self, flag: int) -> str:
        for c in self.configs.all():
            if flag == FLAG_ANY or c.has_usecases(flag):
                return c.name
        loose = self.configs.loose_model_files()
        return loose[0] if loose else ""
