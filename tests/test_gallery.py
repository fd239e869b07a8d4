"""Gallery + downloader (cases modelled on core/gallery/*_test.go and pkg/downloader/uri_test.go),
exercised with file-based galleries: there is no network here."""
import hashlib
import os
import time

import pytest
import yaml

from localai_tfp_amd import gallery as G
from localai_tfp_amd.gallery import downloader as D


def test_resolve_url_schemes():
    assert D.resolve_url("github:go-skynet/model-gallery/gpt4all-j.yaml") == \
        "https://raw.githubusercontent.com/go-skynet/model-gallery/main/gpt4all-j.yaml"
    assert D.resolve_url("github:go-skynet/model-gallery/gpt4all-j.yaml@dev") == \
        "https://raw.githubusercontent.com/go-skynet/model-gallery/dev/gpt4all-j.yaml"
    assert D.resolve_url("huggingface://TheBloke/x-GGUF/x.Q4_K_M.gguf") == \
        "https://huggingface.co/TheBloke/x-GGUF/resolve/main/x.Q4_K_M.gguf"
    assert D.resolve_url("hf://a/b/c.gguf@rev") == "https://huggingface.co/a/b/resolve/rev/c.gguf"
    assert D.resolve_url("https://example.com/a") == "https://example.com/a"
    assert D.looks_like_url("ollama://llama3") and D.looks_like_oci("oci://reg/x:1") and not D.looks_like_url("/tmp/x")
    assert D.filename_from_url("https://h/a/b/model.gguf?x=1") == "model.gguf"
    assert D._registry_parts("ollama://gemma:2b") == ("registry.ollama.ai", "library/gemma", "2b")


def test_download_sha_and_path_guard(tmp_path):
    src = tmp_path / "src.bin"
    src.write_bytes(os.urandom(10000))
    sha = hashlib.sha256(src.read_bytes()).hexdigest()
    dst = tmp_path / "out" / "m.bin"
    seen = []
    D.download_file("file://" + str(src), dst, sha, progress=lambda *a: seen.append(a))
    assert dst.read_bytes() == src.read_bytes() and seen[-1][3] == pytest.approx(100.0)
    with pytest.raises(D.DownloadError):
        D.download_file("file://" + str(src), tmp_path / "bad.bin", "0" * 64)
    assert not (tmp_path / "bad.bin").exists() and not (tmp_path / "bad.bin.partial").exists()
    with pytest.raises(D.DownloadError):
        D.verify_path("../escape", str(tmp_path / "out"))
    with pytest.raises(D.DownloadError):
        D.read_uri("file:///etc/hostname", str(tmp_path))


def _make_gallery(tmp_path):
    blob = tmp_path / "srv" / "weights.gguf"
    blob.parent.mkdir(parents=True)
    blob.write_bytes(b"GGUF" + b"\0" * 100)
    sha = hashlib.sha256(blob.read_bytes()).hexdigest()
    model_cfg = {
        "name": "tiny", "description": "d", "license": "mit",
        "config_file": yaml.safe_dump({"backend": "llama-cpp", "parameters": {"model": "weights.gguf", "temperature": 0.2},
                                       "template": {"chat": "tiny-chat"}}),
        "files": [{"filename": "weights.gguf", "sha256": sha, "uri": "file://" + str(blob)}],
        "prompt_templates": [{"name": "tiny-chat", "content": "{{.Input}}"}],
    }
    (tmp_path / "srv" / "tiny.yaml").write_text(yaml.safe_dump(model_cfg))
    index = [{"name": "tiny", "url": "file://" + str(tmp_path / "srv" / "tiny.yaml"), "tags": ["llm", "q4"],
              "overrides": {"parameters": {"top_k": 7}}},
             {"name": "inline", "config_file": {"backend": "whisper", "parameters": {"model": "w.bin"}},
              "description": "speech"}]
    (tmp_path / "srv" / "index.yaml").write_text(yaml.safe_dump(index))
    return [G.Gallery("test", "file://" + str(tmp_path / "srv" / "index.yaml"))]


def test_list_install_delete(tmp_path):
    base = str(tmp_path / "models")
    gals = _make_gallery(tmp_path / "models")  # file:// sources must live under the models path
    models = G.available_models(gals, base)
    assert [m.name for m in models] == ["tiny", "inline"] and not any(m.installed for m in models)
    assert G.find_model(models, "test@tiny").name == "tiny"
    assert [m.name for m in G.search(models, "speech")] == ["inline"]
    assert G.paginate(models, 2, 1)[0].name == "inline"

    req = G.GalleryModel(overrides={"parameters": {"temperature": 0.5}})
    name = G.install_from_gallery(gals, "tiny", base, req)
    assert name == "tiny"
    cfg = yaml.safe_load(open(os.path.join(base, "tiny.yaml")))
    assert cfg["name"] == "tiny" and cfg["parameters"] == {"model": "weights.gguf", "temperature": 0.5, "top_k": 7}
    assert open(os.path.join(base, "tiny-chat.tmpl")).read() == "{{.Input}}"
    assert os.path.exists(os.path.join(base, "weights.gguf"))
    assert os.path.exists(os.path.join(base, G.gallery_file_name("tiny")))

    G.delete_model(base, "tiny")
    assert not os.path.exists(os.path.join(base, "weights.gguf"))
    assert not os.path.exists(os.path.join(base, "tiny.yaml"))


def test_job_service(tmp_path):
    base = str(tmp_path / "models")
    gals = _make_gallery(tmp_path / "models")
    changed = []
    svc = G.GalleryService(base, gals, on_change=lambda: changed.append(1))
    uid = svc.submit("inline")
    bad = svc.submit("does-not-exist")
    deadline = time.time() + 10
    while time.time() < deadline and not (svc.get_status(uid).processed and svc.get_status(bad).processed):
        time.sleep(0.02)
    st = svc.get_status(uid)
    assert st.processed and st.error is None and st.progress == 100.0, st
    assert yaml.safe_load(open(os.path.join(base, "inline.yaml")))["backend"] == "whisper"
    assert svc.get_status(bad).error and changed == [1]
    svc.close()
