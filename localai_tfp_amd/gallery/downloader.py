"""URI schemes and resumable downloads (behavioural parity: pkg/downloader/uri.go:24-417,
pkg/oci/*.go for ollama/OCI registries, pkg/utils/path.go for path hardening).

Schemes: ``huggingface://owner/repo/file[@branch]`` (also ``hf://``, ``hf.co/``),
``github:org/repo/path[@branch]`` (also ``github://``), ``ollama://model[:tag]``,
``oci://registry/repo[:tag]``, ``file://`` (restricted to a trusted base path) and http(s).

Downloads stream into ``<file>.partial`` and resume with a ``Range`` header when the server
advertises ``Accept-Ranges: bytes``; the sha256 is verified before the atomic rename.
"""
from __future__ import annotations

import hashlib
import json
import logging
import os
import re
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable

log = logging.getLogger("localai_tfp_amd.downloader")

HF_PREFIXES = ("huggingface://", "hf://", "hf.co/")
GITHUB_PREFIXES = ("github://", "github:")
OCI_PREFIX, OLLAMA_PREFIX, LOCAL_PREFIX = "oci://", "ollama://", "file://"
URL_PREFIXES = ("http://", "https://", *HF_PREFIXES, *GITHUB_PREFIXES, OLLAMA_PREFIX, OCI_PREFIX)

ProgressFn = Callable[[str, str, str, float], None]  # (file_name, current_h, total_h, percent)


class DownloadError(RuntimeError):
    pass


def looks_like_url(s: str) -> bool:
    return s.startswith(URL_PREFIXES)


def looks_like_oci(s: str) -> bool:
    return s.startswith((OCI_PREFIX, OLLAMA_PREFIX))


def _split_branch(s: str) -> tuple[str, str]:
    if "@" in s:
        a, b = s.split("@", 1)
        return a, b
    return s, "main"


def resolve_url(uri: str) -> str:
    for p in GITHUB_PREFIXES:
        if uri.startswith(p):
            path, branch = _split_branch(uri[len(p):])
            parts = path.split("/")
            org, proj, rest = parts[0], parts[1], "/".join(parts[2:])
            return f"https://raw.githubusercontent.com/{org}/{proj}/{branch}/{rest}"
    for p in HF_PREFIXES:
        if uri.startswith(p):
            repo = uri[len(p):]
            parts = repo.split("/")
            owner, name = parts[0], parts[1]
            path, branch = _split_branch("/".join(parts[2:]))
            return f"https://huggingface.co/{owner}/{name}/resolve/{branch}/{path}"
    return uri


def filename_from_url(uri: str) -> str:
    u = uri.split("@", 1)[0]
    base = os.path.basename(urllib.parse.unquote(urllib.parse.urlparse(u).path))
    if base:
        return base
    f = hashlib.md5(uri.encode()).hexdigest()
    return f + ".yaml" if uri.endswith((".yaml", ".yml")) else f


def verify_path(rel: str, base: str) -> str:
    """Reject paths that escape `base` (utils.VerifyPath / InTrustedRoot)."""
    full = os.path.realpath(os.path.join(base, rel))
    root = os.path.realpath(base)
    if full != root and not full.startswith(root + os.sep):
        raise DownloadError(f"path {rel!r} escapes {base!r}")
    return full


def human(n: float) -> str:
    for unit in ("B", "KiB", "MiB", "GiB", "TiB"):
        if n < 1024 or unit == "TiB":
            return f"{n:.1f} {unit}" if unit != "B" else f"{int(n)} B"
        n /= 1024
    return str(n)


def _open(url: str, headers: dict | None = None, method: str = "GET", timeout: float = 60):
    req = urllib.request.Request(url, headers=headers or {}, method=method)
    tok = os.environ.get("HF_TOKEN") or os.environ.get("HUGGINGFACE_HUB_TOKEN")
    if tok and "huggingface.co" in url:
        req.add_header("Authorization", f"Bearer {tok}")
    return urllib.request.urlopen(req, timeout=timeout)


def read_uri(uri: str, base_path: str = "", authorization: str = "") -> bytes:
    """Fetch a small resource (gallery index / model config) fully into memory."""
    url = resolve_url(uri)
    if url.startswith(LOCAL_PREFIX):
        path = url[len(LOCAL_PREFIX):]
        if base_path:
            real = os.path.realpath(path)
            root = os.path.realpath(base_path)
            if not (real == root or real.startswith(root + os.sep)):
                raise DownloadError(f"file URL {path!r} is outside the trusted base path")
        with open(path, "rb") as f:
            return f.read()
    if os.path.isfile(url):
        with open(url, "rb") as f:
            return f.read()
    h = {"Authorization": authorization} if authorization else {}
    with _open(url, h) as r:
        return r.read()


# ------------------------------------------------------------------------------------------------
# HuggingFace safety scan (pkg/downloader/huggingface.go:24-47): best effort, HF-hosted files only

class NonHuggingFaceFile(DownloadError):
    pass


class UnsafeFilesFound(DownloadError):
    def __init__(self, msg: str, result: dict):
        super().__init__(msg)
        self.result = result


def hf_api_base() -> str:
    """Scan API root; LOCALAI_HF_API points it at a mirror (or a stand-in server in the tests)."""
    return os.environ.get("LOCALAI_HF_API", "https://huggingface.co").rstrip("/")


def hf_scan(uri: str, timeout: float = 10.0) -> dict:
    """GET {api}/api/models/<owner>/<repo>/scan for a file hosted on huggingface.co. Returns the scan record
    (repositoryId, revision, hasUnsafeFile, clamAVInfectedFiles, dangerousPickles, scansDone); raises
    NonHuggingFaceFile for other hosts and UnsafeFilesFound (carrying the record) when the repo is flagged."""
    parts = resolve_url(uri).split("/")
    if len(parts) <= 4 or parts[2] != "huggingface.co":
        raise NonHuggingFaceFile(f"not a huggingface repo: {uri}")
    url = f"{hf_api_base()}/api/models/{parts[3]}/{parts[4]}/scan"
    with _open(url, timeout=timeout) as r:
        if r.status != 200:
            raise DownloadError(f"unexpected status code during HuggingFace scan: {r.status}")
        res = json.loads(r.read() or b"{}")
    if res.get("hasUnsafeFile"):
        raise UnsafeFilesFound(f"unsafe files found in {parts[3]}/{parts[4]}", res)
    return res


def enforce_scan(uri: str, model: str = "") -> None:
    """Pre-download gate: refuse a file of a flagged HF repo. Like the reference, only a positive finding blocks;
    a non-HF host, an unreachable API or a malformed answer lets the download proceed."""
    try:
        hf_scan(uri)
    except UnsafeFilesFound as ex:
        log.error("model %s: %s (clamAV: %s, pickles: %s)", model or "?", ex,
                  ex.result.get("clamAVInfectedFiles") or [], ex.result.get("dangerousPickles") or [])
        raise
    except (DownloadError, OSError, ValueError) as ex:
        log.debug("scan skipped for %s: %s", uri, ex)


def _sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def download_file(uri: str, file_path: str, sha256: str = "", file_n: int = 0, total_files: int = 1,
                  progress: ProgressFn | None = None, chunk: int = 1 << 22) -> None:
    """DownloadFile: skip if present with matching hash; resumable `.partial`; sha256 check."""
    file_path = os.fspath(file_path)
    if looks_like_oci(uri):
        return _download_oci(uri, file_path, progress)
    if os.path.exists(file_path):
        if not sha256 or _sha256_file(file_path).lower() == sha256.lower():
            return
        log.warning("%s: sha256 mismatch, re-downloading", file_path)
        os.remove(file_path)
    os.makedirs(os.path.dirname(os.path.abspath(file_path)) or ".", exist_ok=True)
    url = resolve_url(uri)
    part = file_path + ".partial"
    if url.startswith(LOCAL_PREFIX) or os.path.isfile(url):
        src = url[len(LOCAL_PREFIX):] if url.startswith(LOCAL_PREFIX) else url
        total = os.path.getsize(src)
        with open(src, "rb") as fi, open(part, "wb") as fo:
            done = 0
            for b in iter(lambda: fi.read(chunk), b""):
                fo.write(b)
                done += len(b)
                if progress:
                    progress(file_path, human(done), human(total), _pct(done, total, file_n, total_files))
    else:
        start = os.path.getsize(part) if os.path.exists(part) else 0
        headers = {}
        if start:
            try:
                with _open(url, method="HEAD") as r:
                    if r.headers.get("Accept-Ranges") == "bytes":
                        headers["Range"] = f"bytes={start}-"
                    else:
                        start = 0
            except Exception:
                start = 0
        with _open(url, headers) as r:
            if start and r.status != 206:
                start = 0
            total = int(r.headers.get("Content-Length") or 0) + start
            with open(part, "ab" if start else "wb") as fo:
                done = start
                last = 0.0
                while True:
                    b = r.read(chunk)
                    if not b:
                        break
                    fo.write(b)
                    done += len(b)
                    if progress and time.monotonic() - last > 0.5:
                        last = time.monotonic()
                        progress(file_path, human(done), human(total), _pct(done, total, file_n, total_files))
    if sha256:
        got = _sha256_file(part)
        if got.lower() != sha256.lower():
            os.remove(part)
            raise DownloadError(f"sha256 mismatch for {file_path}: expected {sha256}, got {got}")
    os.replace(part, file_path)
    if progress:
        sz = os.path.getsize(file_path)
        progress(file_path, human(sz), human(sz), _pct(1, 1, file_n, total_files))


def _pct(done, total, file_n, total_files) -> float:
    frac = done / total if total else 0.0
    return 100.0 * (file_n + frac) / max(1, total_files)


# ------------------------------------------------------------------------------------------------
# ollama / OCI registries (pkg/oci/ollama.go, image.go): fetch the manifest, download the model layer

def _registry_parts(uri: str) -> tuple[str, str, str]:
    if uri.startswith(OLLAMA_PREFIX):
        ref = uri[len(OLLAMA_PREFIX):]
        name, tag = (ref.rsplit(":", 1) + ["latest"])[:2] if ":" in ref else (ref, "latest")
        if "/" not in name:
            name = "library/" + name
        return "registry.ollama.ai", name, tag
    ref = uri[len(OCI_PREFIX):]
    reg, _, rest = ref.partition("/")
    name, tag = (rest.rsplit(":", 1) if ":" in rest else (rest, "latest"))
    return reg, name, tag


def _download_oci(uri: str, file_path: str, progress: ProgressFn | None):
    reg, name, tag = _registry_parts(uri)
    accept = ("application/vnd.docker.distribution.manifest.v2+json,"
              "application/vnd.oci.image.manifest.v1+json")
    headers = {"Accept": accept}
    man_url = f"https://{reg}/v2/{name}/manifests/{tag}"
    try:
        with _open(man_url, headers) as r:
            man = json.loads(r.read())
    except urllib.error.HTTPError as e:
        if e.code != 401:
            raise
        # bearer token flow
        m = re.search(r'realm="([^"]+)",service="([^"]+)"', e.headers.get("WWW-Authenticate", ""))
        if not m:
            raise
        tok_url = f"{m.group(1)}?service={m.group(2)}&scope=repository:{name}:pull"
        with _open(tok_url) as r:
            tok = json.loads(r.read()).get("token", "")
        headers["Authorization"] = f"Bearer {tok}"
        with _open(man_url, headers) as r:
            man = json.loads(r.read())
    layers = man.get("layers", [])
    layer = next((l for l in layers if l.get("mediaType", "").endswith("image.model")), None) or \
        max(layers, key=lambda l: l.get("size", 0))
    digest = layer["digest"]
    blob = f"https://{reg}/v2/{name}/blobs/{digest}"
    sha = digest.split(":", 1)[1] if digest.startswith("sha256:") else ""
    h = {k: v for k, v in headers.items() if k == "Authorization"}
    part = file_path + ".partial"
    with _open(blob, h) as r, open(part, "wb") as fo:
        total = int(layer.get("size", 0))
        done = 0
        for b in iter(lambda: r.read(1 << 22), b""):
            fo.write(b)
            done += len(b)
            if progress:
                progress(file_path, human(done), human(total), 100.0 * done / max(1, total))
    if sha and _sha256_file(part) != sha:
        os.remove(part)
        raise DownloadError(f"digest mismatch for {uri}")
    os.replace(part, file_path)
