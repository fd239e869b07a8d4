"""`local-ai` command line (behavioural parity: main.go:20-122 .env search, core/cli/cli.go:8-18,
run.go:19-203 flags + env aliases, models.go:34-59, util.go:17-109, tts.go:17, transcript.go:15,
soundgeneration.go:18, worker/*.go, federated.go:10-23).

    python -m localai_tfp_amd run [models...] [--address :8080] [--models-path ./models] ...
    python -m localai_tfp_amd models list|install <id>
    python -m localai_tfp_amd tts|transcript|sound-generation ...
    python -m localai_tfp_amd util gguf-info <file> | usecase-heuristic <model>
    python -m localai_tfp_amd worker llm --addr 127.0.0.1:50051
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys

ENV_FILES = [".env", "localai.env", os.path.expanduser("~/.config/localai.env"), "/etc/localai.env"]


def load_env_files():
    """main.go:36-52: first-found wins per variable; existing env is never overridden."""
    for path in ENV_FILES:
        try:
            with open(path) as f:
                for line in f:
                    line = line.strip()
                    if not line or line.startswith("#") or "=" not in line:
                        continue
                    k, _, v = line.partition("=")
                    os.environ.setdefault(k.strip(), v.strip().strip('"').strip("'"))
        except OSError:
            continue


def _bool_env(names, default=False):
    for n in names:
        if n in os.environ:
            return os.environ[n].lower() in ("1", "true", "yes", "on")
    return default


def add_run_args(ap: argparse.ArgumentParser):
    ap.add_argument("models", nargs="*", help="model URLs / gallery ids / config files to install at start")
    ap.add_argument("--models-path")
    ap.add_argument("--address")
    ap.add_argument("--backend-assets-path")
    ap.add_argument("--generated-content-path")
    ap.add_argument("--upload-path")
    ap.add_argument("--localai-config-dir")
    ap.add_argument("--config-file", "--models-config-file", dest="config_file")
    ap.add_argument("--galleries", help="JSON list of galleries")
    ap.add_argument("--autoload-galleries", action="store_true", default=None)
    ap.add_argument("--gateway-workers", type=int, default=None,
                    help="gateway processes accepting on the address (SO_REUSEPORT) and sharing the backends "
                         "(env LOCALAI_GATEWAY_WORKERS; default 1): one Python gateway carries ~20k SSE chunks/s")
    ap.add_argument("--preload-models", help="JSON list of gallery models to apply at start")
    ap.add_argument("--preload-models-config")
    ap.add_argument("--f16", action="store_true", default=None)
    ap.add_argument("--threads", "-t", type=int)
    ap.add_argument("--context-size", type=int)
    ap.add_argument("--cors", action="store_true", default=None)
    ap.add_argument("--cors-allow-origins")
    ap.add_argument("--csrf", action="store_true", default=None)
    ap.add_argument("--upload-limit", type=int)
    ap.add_argument("--api-keys", nargs="*")
    ap.add_argument("--disable-webui", action="store_true", default=None)
    ap.add_argument("--opaque-errors", action="store_true", default=None)
    ap.add_argument("--use-subtle-key-comparison", action="store_true", default=None)
    ap.add_argument("--disable-api-key-requirement-for-http-get", action="store_true", default=None)
    ap.add_argument("--disable-metrics-endpoint", action="store_true", default=None)
    ap.add_argument("--p2p", action="store_true", default=None)
    ap.add_argument("--p2ptoken")
    ap.add_argument("--p2p-dht-interval", type=int)
    ap.add_argument("--p2p-otp-interval", type=int)
    ap.add_argument("--parallel-requests", action="store_true", default=None)
    ap.add_argument("--single-active-backend", action="store_true", default=None)
    ap.add_argument("--preload-backend-only", action="store_true", default=None)
    ap.add_argument("--external-grpc-backends", nargs="*", help="name:host:port or name:/path/to/executable")
    ap.add_argument("--enable-watchdog-idle", action="store_true", default=None)
    ap.add_argument("--watchdog-idle-timeout")
    ap.add_argument("--enable-watchdog-busy", action="store_true", default=None)
    ap.add_argument("--watchdog-busy-timeout")
    ap.add_argument("--federated", action="store_true", default=None)
    ap.add_argument("--p2p-peers", help="comma-separated federator / peer URLs to announce this node to")
    ap.add_argument("--disable-gallery-endpoint", action="store_true", default=None)
    ap.add_argument("--machine-tag")
    ap.add_argument("--load-to-memory", nargs="*")
    ap.add_argument("--log-level", default=os.environ.get("LOCALAI_LOG_LEVEL", "info"))
    ap.add_argument("--gpus", help="comma-separated GPU indices available to backends")


def app_config_from_args(a):
    from .config.app_config import ApplicationConfig, _duration
    c = ApplicationConfig()
    simple = {"models_path": "models_path", "address": "address", "backend_assets_path": "backend_assets_path",
              "generated_content_path": "generated_content_dir", "upload_path": "upload_dir",
              "localai_config_dir": "config_dir", "config_file": "config_file", "threads": "threads",
              "context_size": "context_size", "cors_allow_origins": "cors_allow_origins",
              "upload_limit": "upload_limit_mb", "machine_tag": "machine_tag", "p2ptoken": "p2p_token",
              "p2p_dht_interval": "p2p_dht_interval", "p2p_otp_interval": "p2p_otp_interval",
              "gpus": "gpus"}
    for src, dst in simple.items():
        v = getattr(a, src, None)
        if v is not None:
            setattr(c, dst, v)
    flags = {"f16": "f16", "cors": "cors", "csrf": "csrf", "disable_webui": "disable_webui",
             "opaque_errors": "opaque_errors", "use_subtle_key_comparison": "use_subtle_key_comparison",
             "disable_api_key_requirement_for_http_get": "disable_api_key_requirement_for_http_get",
             "disable_metrics_endpoint": "disable_metrics_endpoint", "p2p": "p2p",
             "parallel_requests": "parallel_backend_requests", "single_active_backend": "single_active_backend",
             "preload_backend_only": "preload_backend_only", "enable_watchdog_idle": "watchdog_idle",
             "enable_watchdog_busy": "watchdog_busy", "federated": "federated",
             "disable_gallery_endpoint": "disable_gallery_endpoint", "autoload_galleries": "autoload_galleries"}
    for src, dst in flags.items():
        v = getattr(a, src, None)
        if v is not None:
            setattr(c, dst, bool(v))
    if a.api_keys:
        c.api_keys = list(a.api_keys)
    if a.watchdog_idle_timeout:
        c.watchdog_idle_timeout_s = _duration(a.watchdog_idle_timeout)
    if a.watchdog_busy_timeout:
        c.watchdog_busy_timeout_s = _duration(a.watchdog_busy_timeout)
    gal = a.galleries or os.environ.get("LOCALAI_GALLERIES") or os.environ.get("GALLERIES")
    if gal:
        c.galleries = json.loads(gal)
    ext = list(a.external_grpc_backends or [])
    env_ext = os.environ.get("LOCALAI_EXTERNAL_GRPC_BACKENDS") or os.environ.get("EXTERNAL_GRPC_BACKENDS")
    if env_ext:
        ext += [e for e in env_ext.split(",") if e]
    for e in ext:
        name, _, target = e.partition(":")
        c.external_grpc_backends[name] = target
    if a.load_to_memory:
        c.load_to_memory = list(a.load_to_memory)
    models = list(a.models or [])
    env_models = os.environ.get("LOCALAI_MODELS") or os.environ.get("MODELS")
    if env_models:
        models += [m for m in env_models.split(",") if m]
    c.models = models
    if a.gpus:
        os.environ["LOCALAI_GPUS"] = a.gpus
    if a.p2p_peers:
        c.p2p_peers = [x for x in a.p2p_peers.split(",") if x]
    return c


def _listen_socket(host: str, port: int, reuse_port: bool):
    import socket
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if reuse_port:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.set_inheritable(True)
    return s


def _spawn_gateway_followers(a, n: int, registry: str) -> list:
    """n sibling gateway processes: same arguments, same address (SO_REUSEPORT), backends shared through
    `registry` (serving/shared_backends.py); gallery preloads and p2p stay with this (primary) process."""
    import subprocess
    env = dict(os.environ, LOCALAI_BACKEND_REGISTRY=registry, LOCALAI_GATEWAY_FOLLOWER=str(os.getpid()),
               LOCALAI_GATEWAY_WORKERS="1")
    argv = [x for x in a._argv]
    return [subprocess.Popen([sys.executable, "-m", "localai_tfp_amd", *argv], env=env) for _ in range(n)]


def _watch_parent(ppid: int):
    """A follower gateway ends with its primary (SIGTERM to itself: uvicorn's graceful shutdown)."""
    import signal
    import threading
    import time as _t

    def run():
        while True:
            _t.sleep(1.0)
            if os.getppid() != ppid:
                os.kill(os.getpid(), signal.SIGTERM)
                return
    threading.Thread(target=run, daemon=True, name="gateway-parent-watch").start()


def cmd_run(a):
    import uvicorn
    from .gateway.app import create_app
    c = app_config_from_args(a)
    follower = os.environ.get("LOCALAI_GATEWAY_FOLLOWER", "")
    nw = a.gateway_workers if a.gateway_workers is not None else int(os.environ.get("LOCALAI_GATEWAY_WORKERS", "1") or 1)
    followers = []
    if follower:
        c.p2p = c.federated = False
        a.preload_models = a.preload_models_config = None
        _watch_parent(int(follower))
    elif nw > 1:
        import tempfile
        reg = os.path.join(c.config_dir or tempfile.gettempdir(), f".gateway-backends-{os.getpid()}")
        os.environ["LOCALAI_BACKEND_REGISTRY"] = reg
    app = create_app(c)
    st = app.state.localai
    if a.preload_models:
        from .gallery import GalleryModel
        for m in json.loads(a.preload_models):
            st.gallery.submit(name=m.get("id", ""), req=GalleryModel.from_dict(m))
    if a.preload_models_config:
        import yaml
        with open(a.preload_models_config) as f:
            for m in yaml.safe_load(f) or []:
                from .gallery import GalleryModel
                st.gallery.submit(name=m.get("id", ""), req=GalleryModel.from_dict(m))
    if c.preload_backend_only:
        st.startup()
        import signal
        signal.sigwait({signal.SIGINT, signal.SIGTERM})
        st.shutdown()
        return 0
    host, port = c.host_port
    level = a.log_level.lower() if a.log_level else "info"
    if not follower and nw <= 1:
        uvicorn.run(app, host=host, port=port, log_level=level, access_log=level == "debug", timeout_keep_alive=60)
        return 0
    sock = _listen_socket(host, port, True)
    if not follower:
        followers = _spawn_gateway_followers(a, nw - 1, os.environ["LOCALAI_BACKEND_REGISTRY"])
    try:
        uvicorn.Server(uvicorn.Config(app, log_level=level, access_log=level == "debug",
                                      timeout_keep_alive=60)).run(sockets=[sock])
    finally:
        for p in followers:
            p.terminate()
        for p in followers:
            try:
                p.wait(timeout=30)
            except Exception:
                p.kill()
        if not follower:
            import shutil
            shutil.rmtree(os.environ.get("LOCALAI_BACKEND_REGISTRY", ""), ignore_errors=True)
    return 0


def cmd_models(a):
    from .config.app_config import ApplicationConfig
    from .gallery import Gallery, available_models, install_from_gallery
    c = ApplicationConfig()
    if a.models_path:
        c.models_path = a.models_path
    gal = a.galleries or os.environ.get("LOCALAI_GALLERIES") or os.environ.get("GALLERIES") or "[]"
    gals = [Gallery.parse(g) for g in json.loads(gal)]
    if a.models_cmd == "list":
        for m in available_models(gals, c.models_path):
            print(("* " if m.installed else "  ") + f"{m.gallery.name}@{m.name}")
    else:
        for name in a.names:
            install_from_gallery(gals, name, c.models_path,
                                 progress=lambda f, cur, tot, pct: print(f"\r{f} {cur}/{tot} {pct:.1f}%", end=""),
                                 enforce_scan=not a.disable_predownload_scan)
            print(f"\ninstalled {name}")
    return 0


def _standalone_app(models_path: str | None):
    from .config.app_config import ApplicationConfig
    from .gateway.state import Application
    c = ApplicationConfig()
    if models_path:
        c.models_path = models_path
    return Application(c)


def cmd_tts(a):
    import asyncio
    from .gateway.media import run_tts
    st = _standalone_app(a.models_path)
    try:
        path = asyncio.run(run_tts(st, {"input": " ".join(a.text), "voice": a.voice or "", "backend": a.backend or "",
                                        "language": a.language or ""}, a.model))
        if a.output_file:
            os.replace(path, a.output_file)
            path = a.output_file
        print(path)
    finally:
        st.shutdown()
    return 0


def cmd_transcript(a):
    import asyncio
    st = _standalone_app(a.models_path)
    try:
        cfg = st.configs.load_by_name(a.model)
        if not cfg.backend:
            cfg.backend = a.backend or "whisper"
        r = asyncio.run(st.inference.transcribe(cfg, a.filename, a.language or "", a.translate, a.threads or 0))
        for s in r.segments:
            print(s.text)
    finally:
        st.shutdown()
    return 0


def cmd_sound(a):
    import asyncio
    st = _standalone_app(a.models_path)
    try:
        cfg = st.configs.load_by_name(a.model)
        if a.backend:
            cfg.backend = a.backend
        out = a.output_file or "sound.wav"
        kw = dict(text=" ".join(a.text), model=cfg.parameters.model, dst=os.path.abspath(out))
        if a.duration:
            kw["duration"] = a.duration
        if a.temperature:
            kw["temperature"] = a.temperature
        asyncio.run(st.inference.sound(cfg, **kw))
        print(out)
    finally:
        st.shutdown()
    return 0


def cmd_util(a):
    if a.util_cmd == "gguf-info":
        from .formats.gguf import GGUFReader
        r = GGUFReader(a.file)
        for k, v in r.metadata.items():
            if isinstance(v, list) and len(v) > 16:
                v = f"[{len(v)} items]"
            print(f"{k}: {v}")
        if a.header_only:
            return 0
        for name, ti in r.tensors.items():
            print(f"tensor {name} {ti.qtype.name if hasattr(ti.qtype, 'name') else ti.qtype} {list(ti.shape)}")
    elif a.util_cmd == "usecase-heuristic":
        from .config.loader import ModelConfigLoader
        from .config.model_config import USECASE_FLAGS
        cl = ModelConfigLoader(a.models_path or "models")
        cl.load_from_path()
        for name in a.names or cl.names():
            c = cl.load_by_name(name)
            flags = [k for k, v in USECASE_FLAGS.items() if v and c.has_usecases(v)]
            print(f"{name}: {', '.join(flags) or '-'}")
    elif a.util_cmd == "hf-scan":
        return _hf_scan(a)
    return 0


def _hf_scan(a) -> int:
    """`local-ai util hf-scan [uri...]` (core/cli/util.go:75-107): best-effort HF safety scan of the given URIs, or
    of every installed gallery model's files. Exit status 1 when anything is flagged."""
    from .gallery import Gallery, safety_scan_installed
    from .gallery import downloader as D
    print("LocalAI security scanner - BEST EFFORT, limited to models hosted on huggingface.co", file=sys.stderr)
    bad = []
    if not a.uris:
        gal = a.galleries or os.environ.get("LOCALAI_GALLERIES") or os.environ.get("GALLERIES") or "[]"
        models_path = a.models_path or os.environ.get("LOCALAI_MODELS_PATH") or os.environ.get("MODELS_PATH") or "models"
        bad = safety_scan_installed([Gallery.parse(g) for g in json.loads(gal)], models_path)
    for uri in a.uris:
        try:
            D.hf_scan(uri)
        except D.UnsafeFilesFound as ex:
            bad.append(("", uri, ex.result))
        except (D.DownloadError, OSError, ValueError) as ex:
            print(f"{uri}: not scanned ({ex})", file=sys.stderr)
    for model, uri, res in bad:
        print(f"! WARNING ! known-unsafe files in {res.get('repositoryId') or uri}{' (model ' + model + ')' if model else ''}: "
              f"clamAV={res.get('clamAVInfectedFiles') or []} pickles={res.get('dangerousPickles') or []}")
    if not bad:
        print("No security warnings were detected. This is a BEST EFFORT tool; not every issue is detected.")
    return 1 if bad else 0


def cmd_federated(a):
    """`local-ai federated` (core/cli/federated.go): the load-balancing proxy over announced nodes."""
    from . import p2p as P
    token = a.p2ptoken or os.environ.get("LOCALAI_P2P_TOKEN") or os.environ.get("TOKEN") or ""
    reg = P.Registry(token, a.network_id or os.environ.get("LOCALAI_P2P_NETWORK_ID", ""))
    for n in (a.nodes or "").split(","):
        if n:  # static nodes (id=host:port or host:port), kept online by re-adding
            nid, _, addr = n.rpartition("=")
            reg.add(P.NodeData(id=nid or addr, address=addr, service=P.FEDERATED_ID))
    fs = P.FederatedServer(a.address, reg, P.FEDERATED_ID, load_balanced=a.load_balanced,
                           worker_target=a.target_worker or "")
    if a.nodes:
        import threading
        import time

        def keep():
            while True:
                for nd in reg.nodes(P.FEDERATED_ID):
                    reg.add(nd)
                time.sleep(10)
        threading.Thread(target=keep, daemon=True).start()
    fs.serve_forever()
    return 0


def cmd_explorer(a):
    """`local-ai explorer` (core/cli/explorer.go): network directory + discovery loop."""
    import uvicorn
    from .p2p.explorer import Database, DiscoveryServer, create_explorer_app
    db = Database(a.pool_database)
    ds = DiscoveryServer(db, a.connection_timeout, a.connection_error_threshold)
    if a.only_sync:
        ds.run_once()
        return 0
    if a.with_sync:
        ds.start()
    host, _, port = a.address.rpartition(":")
    uvicorn.run(create_explorer_app(db), host=host or "0.0.0.0", port=int(port))
    return 0


def cmd_worker(a):
    from . import workers as W
    import importlib
    if a.kind in ("llama-cpp-rpc", "rpc"):
        # layer-split stage (reference `local-ai worker llama-cpp-rpc`, worker_llamacpp.go:19-44)
        from .parallel import pp_rpc
        host, port = a.addr.rsplit(":", 1)
        pp_rpc.main(["--host", host, "--port", port])
        return 0
    mod = importlib.import_module(W.WORKERS[W.resolve(a.kind)])
    mod.main(["--addr", a.addr])
    return 0


def main(argv=None):
    load_env_files()
    ap = argparse.ArgumentParser(prog="local-ai", description="MI355X-native LocalAI")
    sub = ap.add_subparsers(dest="cmd")
    add_run_args(sub.add_parser("run", help="start the API server"))
    m = sub.add_parser("models", help="manage gallery models")
    m.add_argument("models_cmd", choices=["list", "install"])
    m.add_argument("names", nargs="*")
    m.add_argument("--models-path")
    m.add_argument("--galleries")
    m.add_argument("--disable-predownload-scan", action="store_true",
                   default=_bool_env(["LOCALAI_DISABLE_PREDOWNLOAD_SCAN"]))
    t = sub.add_parser("tts", help="text to speech")
    t.add_argument("text", nargs="+")
    t.add_argument("--model", "-m", required=True)
    t.add_argument("--backend", "-b")
    t.add_argument("--voice", "-v")
    t.add_argument("--language", "-l")
    t.add_argument("--output-file", "-o")
    t.add_argument("--models-path")
    tr = sub.add_parser("transcript", help="speech to text")
    tr.add_argument("filename")
    tr.add_argument("--model", "-m", required=True)
    tr.add_argument("--backend", "-b")
    tr.add_argument("--language", "-l")
    tr.add_argument("--translate", action="store_true")
    tr.add_argument("--threads", type=int)
    tr.add_argument("--models-path")
    sg = sub.add_parser("sound-generation", help="text to sound")
    sg.add_argument("text", nargs="+")
    sg.add_argument("--model", "-m", required=True)
    sg.add_argument("--backend", "-b")
    sg.add_argument("--duration", type=float)
    sg.add_argument("--temperature", type=float)
    sg.add_argument("--output-file", "-o")
    sg.add_argument("--models-path")
    u = sub.add_parser("util", help="utilities")
    usub = u.add_subparsers(dest="util_cmd")
    gi = usub.add_parser("gguf-info")
    gi.add_argument("file")
    gi.add_argument("--header-only", action="store_true")
    uh = usub.add_parser("usecase-heuristic")
    uh.add_argument("names", nargs="*")
    uh.add_argument("--models-path")
    hs = usub.add_parser("hf-scan", help="check models for known security issues (best effort, huggingface only)")
    hs.add_argument("uris", nargs="*")
    hs.add_argument("--models-path")
    hs.add_argument("--galleries")
    fd = sub.add_parser("federated", help="run the federated load-balancing proxy")
    fd.add_argument("--address", default=os.environ.get("LOCALAI_ADDRESS", "0.0.0.0:8080"))
    fd.add_argument("--p2ptoken")
    fd.add_argument("--network-id")
    fd.add_argument("--load-balanced", action="store_true",
                    default=_bool_env(["LOCALAI_LOAD_BALANCED", "LOAD_BALANCED"]))
    fd.add_argument("--target-worker", default=os.environ.get("LOCALAI_TARGET_WORKER", ""))
    fd.add_argument("--nodes", default=os.environ.get("LOCALAI_FEDERATED_NODES", ""),
                    help="static nodes: id=host:port,...")
    ex = sub.add_parser("explorer", help="run the p2p network explorer")
    ex.add_argument("--address", default=os.environ.get("LOCALAI_ADDRESS", "0.0.0.0:8080"))
    ex.add_argument("--pool-database", default=os.environ.get("LOCALAI_POOL_DATABASE", "explorer.json"))
    ex.add_argument("--connection-timeout", type=float, default=50.0)
    ex.add_argument("--connection-error-threshold", type=int, default=3)
    ex.add_argument("--with-sync", action="store_true")
    ex.add_argument("--only-sync", action="store_true")
    w = sub.add_parser("worker", help="run a single backend worker process")
    w.add_argument("kind", help="backend name, e.g. llama-cpp, whisper, bert-embeddings; llama-cpp-rpc = layer-split stage")
    w.add_argument("--addr", default="127.0.0.1:50051")
    a = ap.parse_args(argv)
    a._argv = list(argv) if argv is not None else sys.argv[1:]
    logging.basicConfig(level=getattr(logging, str(getattr(a, "log_level", "info") or "info").upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    fn = {"run": cmd_run, "models": cmd_models, "tts": cmd_tts, "transcript": cmd_transcript,
          "sound-generation": cmd_sound, "util": cmd_util, "worker": cmd_worker,
          "federated": cmd_federated, "explorer": cmd_explorer}.get(a.cmd)
    if fn is None:
        ap.print_help()
        return 1
    return fn(a)


if __name__ == "__main__":
    sys.exit(main())
