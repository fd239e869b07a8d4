"""HuggingFace safety scan (reference pkg/downloader/huggingface.go:24-47, core/gallery/models.go:121-126,
core/cli/util.go:75-107) against a local stand-in for the HF scan API (no egress here): flagged repos block gallery
installs before any byte is downloaded, `util hf-scan` reports them, non-HF hosts pass unscanned."""
import json
import os
import subprocess
import sys
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest
import yaml

from localai_tfp_amd.gallery import GalleryService, ModelInstallConfig, install_model
from localai_tfp_amd.gallery import downloader as D

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Scan(BaseHTTPRequestHandler):
    hits = []

    def do_GET(self):
        _Scan.hits.append(self.path)
        if self.path.startswith("/api/models/"):
            owner, repo = self.path.split("/")[3:5]
            bad = owner == "evil"
            rec = {"repositoryId": f"{owner}/{repo}", "revision": "abc", "hasUnsafeFile": bad,
                   "clamAVInfectedFiles": ["x.bin"] if bad else [], "dangerousPickles": ["model.pkl"] if bad else [],
                   "scansDone": True}
            body = json.dumps(rec).encode()
        elif self.path == "/files/weights.bin":
            body = b"\x00" * 1024
        else:
            self.send_response(404)
            self.end_headers()
            return
        self.send_response(200)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.fixture()
def scan_api(monkeypatch):
    srv = HTTPServer(("127.0.0.1", 0), _Scan)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_port}"
    monkeypatch.setenv("LOCALAI_HF_API", base)
    _Scan.hits.clear()
    yield base
    srv.shutdown()


def test_scan_record_and_verdicts(scan_api):
    rec = D.hf_scan("huggingface://good/model/file.gguf")
    assert rec["repositoryId"] == "good/model" and not rec["hasUnsafeFile"]
    with pytest.raises(D.UnsafeFilesFound) as ei:
        D.hf_scan("hf://evil/model/file.gguf@main")
    assert ei.value.result["dangerousPickles"] == ["model.pkl"]
    assert _Scan.hits[-1] == "/api/models/evil/model/scan"
    with pytest.raises(D.NonHuggingFaceFile):
        D.hf_scan("github:org/repo/file.yaml")


def test_install_refuses_flagged_repo_before_download(scan_api, tmp_path):
    cfg = ModelInstallConfig(name="m", files=[{"filename": "w.gguf", "uri": "huggingface://evil/repo/w.gguf"}])
    with pytest.raises(D.UnsafeFilesFound):
        install_model(str(tmp_path), "", cfg, {}, enforce_scan=True)
    assert not (tmp_path / "w.gguf").exists() and not (tmp_path / "w.gguf.partial").exists()
    # non-HF files are not scanned and download normally
    cfg2 = ModelInstallConfig(name="m2", files=[{"filename": "w.bin", "uri": f"{scan_api}/files/weights.bin"}])
    install_model(str(tmp_path), "", cfg2, {}, enforce_scan=True)
    assert (tmp_path / "w.bin").stat().st_size == 1024


def test_scan_unreachable_api_does_not_block(monkeypatch, tmp_path, scan_api):
    monkeypatch.setenv("LOCALAI_HF_API", "http://127.0.0.1:9")  # closed port: the reference ignores such errors
    D.enforce_scan("huggingface://evil/repo/w.gguf", "m")  # no raise


def test_gallery_job_reports_unsafe(scan_api, tmp_path):
    (tmp_path / "models").mkdir()
    gal = tmp_path / "models" / "gallery.yaml"  # file:// galleries must sit under the models path
    gal.write_text(yaml.safe_dump([{"name": "bad-model", "config_file": {"backend": "llama-cpp"},
                                    "files": [{"filename": "b.gguf", "uri": "huggingface://evil/r/b.gguf"}]}]))
    svc = GalleryService(str(tmp_path / "models"), [{"name": "g", "url": f"file://{gal}"}], enforce_scan=True)
    try:
        uid = svc.submit("g@bad-model")
        import time
        t0 = time.time()
        while not (svc.get_status(uid) and svc.get_status(uid).processed) and time.time() - t0 < 30:
            time.sleep(0.05)
        st = svc.get_status(uid)
        assert st.processed and st.error and "unsafe" in st.error
    finally:
        svc.close()


def test_util_hf_scan_cli(scan_api, tmp_path):
    env = dict(os.environ, LOCALAI_HF_API=scan_api)
    run = lambda *a: subprocess.run([sys.executable, "-m", "localai_tfp_amd", "util", "hf-scan", *a], env=env,
                                    cwd=ROOT, capture_output=True, text=True, timeout=120)
    p = run("huggingface://good/a/x.gguf")
    assert p.returncode == 0 and "No security warnings" in p.stdout
    p = run("huggingface://good/a/x.gguf", "huggingface://evil/b/y.gguf")
    assert p.returncode == 1 and "evil/b" in p.stdout and "model.pkl" in p.stdout
    # no arguments: the installed gallery models' files
    models = tmp_path / "models"
    models.mkdir()
    gal = models / "gallery.yaml"
    gal.write_text(yaml.safe_dump([{"name": "bad-model", "config_file": {"backend": "llama-cpp"},
                                    "files": [{"filename": "b.gguf", "uri": "huggingface://evil/r/b.gguf"}]}]))
    (models / "._gallery_bad-model.yaml").write_text(yaml.safe_dump({"name": "bad-model", "files": []}))
    gals = json.dumps([{"name": "g", "url": f"file://{gal}"}])
    p = run("--models-path", str(models), "--galleries", gals)
    assert p.returncode == 1 and "bad-model" in p.stdout, p.stdout + p.stderr
