"""`local-ai run <model...>` positional arguments: URLs, gallery ids, OCI refs
(behavioural parity: pkg/startup/model_preload.go:20-138)."""
from __future__ import annotations

import logging
import os

import yaml

from ..gallery import GalleryModel, ModelInstallConfig, apply_gallery_model, install_from_gallery, install_model
from ..gallery.downloader import download_file, filename_from_url, looks_like_oci, looks_like_url, read_uri

log = logging.getLogger("localai_tfp_amd.startup")


def install_models(app, refs: list[str]) -> list[str]:
    """Each ref is (a) a URL to a model YAML config, (b) a URL/OCI/ollama ref to a model file,
    (c) `gallery@name` or a bare gallery model name. Returns the installed model names."""
    base = app.cfg.models_path
    out = []
    for ref in refs:
        if looks_like_url(ref) and not looks_like_oci(ref) and ref.endswith((".yaml", ".yml")):
            d = yaml.safe_load(read_uri(ref, base)) or {}
            if "config_file" in d or "files" in d:
                cfg = ModelInstallConfig.from_yaml(yaml.safe_dump(d))
                out.append(install_model(base, "", cfg, {}, enforce_scan=app.cfg.enforce_predownload_scans))
            else:
                name = d.get("name") or os.path.splitext(filename_from_url(ref))[0]
                with open(os.path.join(base, name + ".yaml"), "w") as f:
                    yaml.safe_dump(d, f)
                out.append(name)
        elif looks_like_url(ref):
            fname = filename_from_url(ref)
            if looks_like_oci(ref):
                fname = ref.split("://", 1)[1].replace("/", "__").replace(":", "-")
            dst = os.path.join(base, fname)
            if not os.path.exists(dst):
                download_file(ref, dst)
            out.append(fname)
        elif os.path.exists(ref) and ref.endswith((".yaml", ".yml")):
            with open(ref) as f:
                d = yaml.safe_load(f) or {}
            name = d.get("name") or os.path.splitext(os.path.basename(ref))[0]
            with open(os.path.join(base, name + ".yaml"), "w") as f:
                yaml.safe_dump(d, f)
            out.append(name)
        else:
            out.append(install_from_gallery(app.gallery.galleries, ref, base,
                                            enforce_scan=app.cfg.enforce_predownload_scans))
        app.reload_configs()
    return out
