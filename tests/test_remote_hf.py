"""`huggingface` backend (reference backend/go/llm/langchain): remote HF Inference API client, driven
through the HTTP gateway against a local stand-in for the Inference API (no egress here)."""
import json
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest
import yaml
from fastapi.testclient import TestClient

from localai_tfp_amd.config.app_config import ApplicationConfig
from localai_tfp_amd.gateway.app import create_app


class _HF(BaseHTTPRequestHandler):
    seen = []

    def do_POST(self):
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        _HF.seen.append((self.path, self.headers.get("Authorization"), body))
        txt = "remote says hello STOP and more"
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.end_headers()
        self.wfile.write(json.dumps([{"generated_text": txt}]).encode())

    def log_message(self, *a):
        pass


@pytest.fixture()
def hf_server(monkeypatch):
    srv = HTTPServer(("127.0.0.1", 0), _HF)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    monkeypatch.setenv("HUGGINGFACEHUB_API_BASE", f"http://127.0.0.1:{srv.server_port}/models")
    yield srv
    srv.shutdown()


def _app(tmp_path):
    models = tmp_path / "models"
    models.mkdir()
    (models / "hf.yaml").write_text(yaml.safe_dump({
        "name": "hf", "backend": "huggingface",
        "parameters": {"model": "gpt2", "temperature": 0.5, "max_tokens": 16},
        "stopwords": ["STOP"], "template": {"completion": "{{.Input}}"},
    }))
    cfg = ApplicationConfig(models_path=str(models), generated_content_dir=str(tmp_path / "gen"),
                            upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"), api_keys=[])
    return create_app(cfg, inproc=True)


def test_hf_backend_completion(tmp_path, hf_server, monkeypatch):
    monkeypatch.setenv("HUGGINGFACEHUB_API_TOKEN", "hf_test")
    _HF.seen.clear()
    app = _app(tmp_path)
    with TestClient(app) as c:
        r = c.post("/v1/completions", json={"model": "hf", "prompt": "say hi"})
        assert r.status_code == 200, r.text
        assert r.json()["choices"][0]["text"] == "remote says hello "
    app.state.localai.shutdown()
    path, auth, body = _HF.seen[0]
    assert path == "/models/gpt2" and auth == "Bearer hf_test"
    assert body["inputs"] == "say hi"
    assert body["parameters"]["max_new_tokens"] == 16 and body["parameters"]["stop_sequences"] == ["STOP"]


def test_hf_backend_requires_token(tmp_path, hf_server, monkeypatch):
    monkeypatch.delenv("HUGGINGFACEHUB_API_TOKEN", raising=False)
    app = _app(tmp_path)
    with TestClient(app, raise_server_exceptions=False) as c:
        r = c.post("/v1/completions", json={"model": "hf", "prompt": "say hi"})
        assert r.status_code >= 400
    app.state.localai.shutdown()
