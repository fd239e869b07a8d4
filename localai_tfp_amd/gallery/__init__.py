"""Model gallery: index listing, install (files + prompt templates + merged YAML config), delete,
and an asynchronous job service with progress (behavioural parity: core/gallery/gallery.go:19-266,
models.go:99-221, request.go:13-76; core/services/gallery.go:18-215)."""
from __future__ import annotations

import copy
import logging
import os
import queue
import threading
import uuid
from dataclasses import dataclass, field

import yaml

from . import downloader as _dl
from .downloader import DownloadError, download_file, read_uri, verify_path  # noqa: F401

log = logging.getLogger("localai_tfp_amd.gallery")


@dataclass
class Gallery:
    name: str
    url: str

    @classmethod
    def parse(cls, v) -> "Gallery":
        if isinstance(v, Gallery):
            return v
        return cls(v.get("name", ""), v.get("url", ""))


@dataclass
class GalleryModel:
    name: str = ""
    url: str = ""
    description: str = ""
    license: str = ""
    urls: list = field(default_factory=list)
    icon: str = ""
    tags: list = field(default_factory=list)
    files: list = field(default_factory=list)  # [{filename, sha256, uri}]
    config_file: dict = field(default_factory=dict)
    overrides: dict = field(default_factory=dict)
    gallery: Gallery | None = None
    installed: bool = False

    @property
    def id(self) -> str:
        return f"{self.gallery.name if self.gallery else ''}@{self.name}"

    @classmethod
    def from_dict(cls, d: dict, gallery: Gallery | None = None) -> "GalleryModel":
        return cls(name=d.get("name", ""), url=d.get("url", ""), description=d.get("description", ""),
                   license=d.get("license", ""), urls=list(d.get("urls") or []), icon=d.get("icon", ""),
                   tags=list(d.get("tags") or []), files=list(d.get("files") or []),
                   config_file=dict(d.get("config_file") or {}), overrides=dict(d.get("overrides") or {}),
                   gallery=gallery)

    def to_dict(self) -> dict:
        d = {"name": self.name, "url": self.url, "description": self.description, "license": self.license,
             "urls": self.urls, "icon": self.icon, "tags": self.tags, "files": self.files,
             "installed": self.installed}
        if self.config_file:
            d["config_file"] = self.config_file
        if self.overrides:
            d["overrides"] = self.overrides
        if self.gallery:
            d["gallery"] = {"name": self.gallery.name, "url": self.gallery.url}
        return d


@dataclass
class ModelInstallConfig:
    """The per-model YAML a gallery `url:` points at (models.go:47-56)."""
    name: str = ""
    description: str = ""
    icon: str = ""
    license: str = ""
    urls: list = field(default_factory=list)
    config_file: str = ""
    files: list = field(default_factory=list)
    prompt_templates: list = field(default_factory=list)  # [{name, content}]

    @classmethod
    def from_yaml(cls, data: bytes | str) -> "ModelInstallConfig":
        d = yaml.safe_load(data) or {}
        return cls(name=d.get("name", ""), description=d.get("description", ""), icon=d.get("icon", ""),
                   license=d.get("license", ""), urls=list(d.get("urls") or []),
                   config_file=d.get("config_file") or "", files=list(d.get("files") or []),
                   prompt_templates=list(d.get("prompt_templates") or []))

    def to_dict(self) -> dict:
        return {"name": self.name, "description": self.description, "icon": self.icon, "license": self.license,
                "urls": self.urls, "config_file": self.config_file, "files": self.files,
                "prompt_templates": self.prompt_templates}


def gallery_file_name(name: str) -> str:
    return f"._gallery_{name}.yaml"


def _safe_name(name: str) -> str:
    return name.replace(os.sep, "__")


def deep_merge(dst: dict, src: dict) -> dict:
    """mergo.Merge(..., WithOverride): src wins, maps merge recursively."""
    for k, v in (src or {}).items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            deep_merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


# ------------------------------------------------------------------------------------------------
# listing

def gallery_models(g: Gallery, base_path: str) -> list[GalleryModel]:
    data = read_uri(g.url, base_path)
    items = yaml.safe_load(data) or []
    out = []
    for d in items:
        m = GalleryModel.from_dict(d, g)
        m.installed = os.path.exists(os.path.join(base_path, gallery_file_name(_safe_name(m.name))))
        out.append(m)
    return out


def available_models(galleries, base_path: str) -> list[GalleryModel]:
    out = []
    for g in galleries:
        g = Gallery.parse(g)
        try:
            out.extend(gallery_models(g, base_path))
        except Exception as ex:
            log.warning("gallery %s (%s) unavailable: %s", g.name, g.url, ex)
    return out


def find_model(models: list[GalleryModel], name: str) -> GalleryModel | None:
    name = _safe_name(name)
    for m in models:
        if ("@" in name and name.lower() == m.id.lower()) or ("@" not in name and m.name.lower() == name.lower()):
            return m
    return None


def search(models: list[GalleryModel], term: str) -> list[GalleryModel]:
    return [m for m in models if term in m.name or term in m.description or
            (m.gallery and term in m.gallery.name) or term in ",".join(m.tags)]


def paginate(models: list, page: int, per_page: int) -> list:
    start = max(0, (page - 1) * per_page)
    return models[start:start + per_page]


# ------------------------------------------------------------------------------------------------
# install / delete

def install_model(base_path: str, name_override: str, cfg: ModelInstallConfig, overrides: dict | None,
                  progress=None, enforce_scan: bool = False) -> str:
    """Download the files (each behind the HF safety scan when enforce_scan: core/gallery/models.go:121-126),
    write prompt templates, the merged model YAML and the gallery record."""
    os.makedirs(base_path, exist_ok=True)
    for i, f in enumerate(cfg.files):
        dst = verify_path(f["filename"], base_path)
        if enforce_scan and f.get("uri"):
            _dl.enforce_scan(f["uri"], name_override or cfg.name)
        download_file(f.get("uri", ""), dst, f.get("sha256", ""), i, len(cfg.files), progress)
    for t in cfg.prompt_templates:
        dst = verify_path(t["name"] + ".tmpl", base_path)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, "w") as fh:
            fh.write(t.get("content", ""))
    name = name_override or cfg.name
    cfg_path = verify_path(name + ".yaml", base_path)
    if overrides or cfg.config_file:
        cm = yaml.safe_load(cfg.config_file) if cfg.config_file else {}
        cm = cm or {}
        cm["name"] = name
        deep_merge(cm, overrides or {})
        from ..config.model_config import ModelConfig
        mc = ModelConfig.from_dict(copy.deepcopy(cm))
        if not mc.validate():
            raise ValueError(f"gallery config for {name!r} failed validation")
        with open(cfg_path, "w") as fh:
            yaml.safe_dump(cm, fh, sort_keys=False)
    with open(verify_path(gallery_file_name(name), base_path), "w") as fh:
        yaml.safe_dump(cfg.to_dict(), fh, sort_keys=False)
    return name


def install_from_gallery(galleries, name: str, base_path: str, req: GalleryModel | None = None,
                         progress=None, enforce_scan: bool = False) -> str:
    models = available_models(galleries, base_path)
    m = find_model(models, name)
    if m is None:
        raise KeyError(f"no model found with name {name!r}")
    return apply_gallery_model(m, base_path, req, progress, enforce_scan)


def apply_gallery_model(m: GalleryModel, base_path: str, req: GalleryModel | None = None, progress=None,
                        enforce_scan: bool = False) -> str:
    req = req or GalleryModel()
    if m.url:
        cfg = ModelInstallConfig.from_yaml(read_uri(m.url, base_path))
        cfg.description, cfg.license = m.description, m.license
    elif m.config_file:
        cfg = ModelInstallConfig(name=m.name, description=m.description, license=m.license, urls=list(m.urls),
                                 config_file=yaml.safe_dump(m.config_file))
    else:
        raise ValueError(f"invalid gallery model {m.name!r}: neither url nor config_file")
    cfg.urls = list(cfg.urls) + list(m.urls)
    cfg.icon = m.icon
    cfg.files = list(cfg.files) + list(req.files) + list(m.files)
    ov = deep_merge(copy.deepcopy(m.overrides), req.overrides)
    return install_model(base_path, req.name or m.name, cfg, ov, progress, enforce_scan)


def safety_scan_installed(galleries, base_path: str) -> list[tuple[str, str, dict]]:
    """`local-ai util hf-scan` without arguments (core/gallery/gallery.go:243-262): every installed gallery
    model's files through the HF scan. Returns [(model, uri, scan record)] of the flagged ones."""
    bad = []
    for m in available_models(galleries, base_path):
        if not m.installed:
            continue
        files = list(m.files)
        try:
            files += local_model_config(base_path, m.name).files
        except (OSError, ValueError):
            pass
        for uri in dict.fromkeys(f.get("uri", "") for f in files):
            if not uri:
                continue
            try:
                _dl.hf_scan(uri)
            except _dl.UnsafeFilesFound as ex:
                bad.append((m.name, uri, ex.result))
            except (_dl.DownloadError, OSError, ValueError):
                pass
    return bad


def local_model_config(base_path: str, name: str) -> ModelInstallConfig:
    with open(os.path.join(base_path, gallery_file_name(_safe_name(name)))) as fh:
        return ModelInstallConfig.from_yaml(fh.read())


def delete_model(base_path: str, name: str, additional_files=()) -> None:
    name = _safe_name(name)
    cfg_file = verify_path(name + ".yaml", base_path)
    gal_file = verify_path(gallery_file_name(name), base_path)
    files = []
    try:
        gc = local_model_config(base_path, name)
        files += [verify_path(f["filename"], base_path) for f in gc.files]
    except FileNotFoundError:
        pass
    files += [verify_path(f, base_path) for f in additional_files]
    files += [cfg_file, gal_file]
    errs = []
    for f in dict.fromkeys(files):
        try:
            os.remove(f)
        except FileNotFoundError as ex:
            errs.append(str(ex))
    if errs and len(errs) == len(dict.fromkeys(files)):
        raise FileNotFoundError("; ".join(errs))


# ------------------------------------------------------------------------------------------------
# async job service (core/services/gallery.go)

@dataclass
class OpStatus:
    deletion: bool = False
    file_name: str = ""
    error: str | None = None
    processed: bool = False
    message: str = ""
    progress: float = 0.0
    total_file_size: str = ""
    downloaded_file_size: str = ""
    gallery_element_name: str = ""

    def to_dict(self):
        return {"deletion": self.deletion, "file_name": self.file_name, "error": self.error,
                "processed": self.processed, "message": self.message, "progress": self.progress,
                "file_size": self.total_file_size, "downloaded_size": self.downloaded_file_size,
                "gallery_element_name": self.gallery_element_name}


@dataclass
class GalleryOp:
    id: str
    gallery_model_name: str = ""
    req: GalleryModel | None = None
    config_url: str = ""
    delete: bool = False
    galleries: list = field(default_factory=list)


class GalleryService:
    def __init__(self, base_path: str, galleries=None, on_change=None, enforce_scan: bool = False):
        self.base_path = base_path
        self.enforce_scan = enforce_scan  # HF safety scan before every download (EnforcePredownloadScans)
        self.galleries = [Gallery.parse(g) for g in (galleries or [])]
        self.status: dict[str, OpStatus] = {}
        self.q: queue.Queue[GalleryOp | None] = queue.Queue()
        self.on_change = on_change  # e.g. reload model configs after an install
        self._lock = threading.Lock()
        self._t = threading.Thread(target=self._loop, daemon=True, name="gallery-jobs")
        self._t.start()

    def submit(self, name: str = "", req: GalleryModel | None = None, config_url: str = "",
               delete: bool = False) -> str:
        uid = str(uuid.uuid4())
        self._set(uid, OpStatus(message="waiting", gallery_element_name=name))
        self.q.put(GalleryOp(uid, name, req, config_url, delete, self.galleries))
        return uid

    def get_status(self, uid: str) -> OpStatus | None:
        with self._lock:
            return self.status.get(uid)

    def all_status(self) -> dict:
        with self._lock:
            return dict(self.status)

    def _set(self, uid, st: OpStatus):
        with self._lock:
            self.status[uid] = st

    def close(self):
        self.q.put(None)

    def _loop(self):
        while True:
            op = self.q.get()
            if op is None:
                return
            st = OpStatus(deletion=op.delete, gallery_element_name=op.gallery_model_name, message="processing")
            self._set(op.id, st)

            def progress(fname, cur, total, pct, st=st):
                st.file_name, st.downloaded_file_size, st.total_file_size = fname, cur, total
                st.progress = pct
                st.message = "processing"

            try:
                if op.delete:
                    delete_model(self.base_path, op.gallery_model_name)
                elif op.config_url:
                    cfg = ModelInstallConfig.from_yaml(read_uri(op.config_url, self.base_path))
                    req = op.req or GalleryModel()
                    cfg.files += req.files
                    install_model(self.base_path, req.name or cfg.name, cfg, req.overrides, progress, self.enforce_scan)
                elif op.req is not None and (op.req.url or op.req.config_file) and not op.gallery_model_name:
                    apply_gallery_model(op.req, self.base_path, op.req, progress, self.enforce_scan)
                else:
                    install_from_gallery(op.galleries, op.gallery_model_name, self.base_path, op.req, progress,
                                         self.enforce_scan)
                if self.on_change:
                    self.on_change()
                st.progress, st.processed, st.message = 100.0, True, "completed"
            except Exception as ex:
                log.error("gallery job %s failed: %s", op.id, ex)
                st.error, st.processed, st.message = str(ex), True, f"error: {ex}"
