"""Model-config registry (reference: core/config/backend_config_loader.go:21-370).

* `load_from_path(models_dir)`: every `*.yaml|*.yml` file (one config each) in the models dir;
* `load_multiple_single_file(path)`: a YAML list of configs (`--config-file`);
* `load_by_name(name)`: the config called `name`, else `<models>/<name>.yaml`, else a synthetic
  config with `parameters.model = name` (so a bare GGUF in the models dir just works), with
  SetDefaults + GGUF guessing applied;
* `preload()`: downloads `download_files`, URL models and mmproj into the models dir.
"""
from __future__ import annotations

import logging
import os
import threading
from pathlib import Path

import yaml

from .model_config import ModelConfig

log = logging.getLogger("localai_tfp_amd.config")

MODEL_EXTS_SKIP = {".yaml", ".yml", ".tmpl", ".json", ".md", ".txt", ".partial", ".keep", ".sha256"}


class ModelConfigLoader:
    def __init__(self, model_path: str = "models", ctx_size: int = 0, threads: int = 0, f16: bool = False,
                 debug: bool = False):
        self.model_path = str(model_path)
        self.ctx_size, self.threads, self.f16, self.debug = ctx_size, threads, f16, debug
        self._configs: dict[str, ModelConfig] = {}
        self._implicit: dict[str, ModelConfig] = {}
        self._lock = threading.RLock()

    # ---------------------------------------------------------------- loading
    def _defaults(self, c: ModelConfig):
        c.set_defaults(self.ctx_size, self.threads, self.f16, self.debug, self.model_path)

    def read_file(self, path: str | Path) -> list[ModelConfig]:
        with open(path, "r", encoding="utf-8") as f:
            data = yaml.safe_load(f)
        if data is None:
            return []
        items = data if isinstance(data, list) else [data]
        out = []
        for d in items:
            if not isinstance(d, dict):
                continue
            c = ModelConfig.from_dict(d)
            c.source_file = str(path)
            self._defaults(c)
            out.append(c)
        return out

    def load_config_file(self, path: str | Path):
        cs = self.read_file(path)
        for c in cs:
            if not c.validate():
                raise ValueError(f"invalid model config {path}")
            with self._lock:
                self._configs[c.name] = c

    def load_multiple_single_file(self, path: str | Path):
        for c in self.read_file(path):
            if c.validate():
                with self._lock:
                    self._configs[c.name] = c

    def load_from_path(self, path: str | None = None):
        p = Path(path or self.model_path)
        if not p.is_dir():
            return
        for f in sorted(p.iterdir()):
            if f.suffix not in (".yaml", ".yml") or f.name.startswith("."):
                continue
            try:
                for c in self.read_file(f):
                    if c.validate() and c.name:
                        with self._lock:
                            self._configs[c.name] = c
                    else:
                        log.warning("skipping invalid config %s", f)
            except Exception as ex:
                log.warning("cannot load %s: %s", f, ex)

    def load_by_name(self, name: str) -> ModelConfig:
        with self._lock:
            c = self._configs.get(name)
        if c is None:
            cand = Path(self.model_path) / f"{name}.yaml"
            if cand.exists():
                self.load_config_file(cand)
                with self._lock:
                    c = self._configs.get(name)
        if c is not None:
            return c.copy()  # defaults were applied when the file was read
        # implicit config for a bare model file; cached so the GGUF header is parsed once, not per request
        with self._lock:
            c = self._implicit.get(name)
        if c is None:
            c = ModelConfig(name=name)
            c.parameters.model = name
            self._defaults(c)
            with self._lock:
                self._implicit[name] = c
        return c.copy()

    # ---------------------------------------------------------------- queries
    def get(self, name: str) -> ModelConfig | None:
        with self._lock:
            c = self._configs.get(name)
            return c.copy() if c else None

    def all(self) -> list[ModelConfig]:
        with self._lock:
            return [c for _, c in sorted(self._configs.items())]

    def names(self) -> list[str]:
        with self._lock:
            return sorted(self._configs)

    def remove(self, name: str):
        with self._lock:
            self._configs.pop(name, None)

    def add(self, c: ModelConfig):
        with self._lock:
            self._configs[c.name] = c

    def filtered(self, flt) -> list[ModelConfig]:
        return [c for c in self.all() if flt(c)]

    def loose_model_files(self) -> list[str]:
        """Model files in the models dir that no config references (listed by /v1/models too)."""
        p = Path(self.model_path)
        if not p.is_dir():
            return []
        referenced = {c.parameters.model for c in self.all()} | set(self.names())
        out = []
        for f in sorted(p.iterdir()):
            if f.is_dir() or f.name.startswith(".") or f.suffix in MODEL_EXTS_SKIP:
                continue
            if f.name not in referenced:
                out.append(f.name)
        return out

    # ---------------------------------------------------------------- preload (downloads)
    def preload(self, progress=None):
        from ..gallery.downloader import download_file, looks_like_url, resolve_url
        for c in self.all():
            for f in c.download_files:
                fn = f.get("filename", "")
                uri = f.get("uri", "")
                sha = f.get("sha256", "")
                dst = Path(self.model_path) / fn
                if dst.exists() or not uri:
                    continue
                download_file(resolve_url(uri), dst, sha, progress=progress)
            m = c.parameters.model
            if m and looks_like_url(m):
                import hashlib
                fname = hashlib.md5(m.encode()).hexdigest()
                dst = Path(self.model_path) / fname
                if not dst.exists():
                    download_file(resolve_url(m), dst, "", progress=progress)
                c.parameters.model = fname
            if c.mmproj and looks_like_url(c.mmproj):
                import hashlib
                fname = hashlib.md5(c.mmproj.encode()).hexdigest()
                dst = Path(self.model_path) / fname
                if not dst.exists():
                    download_file(resolve_url(c.mmproj), dst, "", progress=progress)
                c.mmproj = fname


# filters (backend_config_filter.go:7-35)
def no_filter(_c):
    return True


def by_usecase(flag: int):
    return lambda c: c.has_usecases(flag)


def by_name_regex(pattern: str):
    import re
    rx = re.compile(pattern)
    return lambda c: bool(rx.search(c.name))
