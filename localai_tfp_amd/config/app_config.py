"""Application-wide settings (reference: core/config/application_config.go:14-371 and the `run`
command flags + LOCALAI_* env aliases, core/cli/run.go:19-73)."""
from __future__ import annotations

import os
from dataclasses import dataclass, field


def _env(name, default, cast=str):
    for n in ([name] if isinstance(name, str) else name):
        v = os.environ.get(n)
        if v is not None and v != "":
            if cast is bool:
                return v.lower() in ("1", "true", "yes", "on")
            if cast is list:
                return [x for x in (s.strip() for s in v.replace(";", ",").split(",")) if x]
            return cast(v)
    return default


@dataclass
class ApplicationConfig:
    models_path: str = field(default_factory=lambda: _env(["LOCALAI_MODELS_PATH", "MODELS_PATH"], "models"))
    backend_assets_path: str = field(default_factory=lambda: _env(["LOCALAI_BACKEND_ASSETS_PATH", "BACKEND_ASSETS_PATH"], "/tmp/localai/backend_data"))
    generated_content_dir: str = field(default_factory=lambda: _env(["LOCALAI_GENERATED_CONTENT_PATH", "GENERATED_CONTENT_PATH"], "/tmp/generated/content"))
    upload_dir: str = field(default_factory=lambda: _env(["LOCALAI_UPLOAD_PATH", "UPLOAD_PATH"], "/tmp/localai/upload"))
    config_dir: str = field(default_factory=lambda: _env(["LOCALAI_CONFIG_DIR", "CONFIG_DIR"], "/tmp/localai/config"))
    config_file: str = field(default_factory=lambda: _env(["LOCALAI_MODELS_CONFIG_FILE", "CONFIG_FILE"], ""))
    galleries: list = field(default_factory=list)
    autoload_galleries: bool = field(default_factory=lambda: _env(["LOCALAI_AUTOLOAD_GALLERIES", "AUTOLOAD_GALLERIES"], False, bool))
    preload_models: list = field(default_factory=list)
    models: list = field(default_factory=list)  # positional `run` args: URLs / gallery ids
    address: str = field(default_factory=lambda: _env(["LOCALAI_ADDRESS", "ADDRESS"], ":8080"))
    cors: bool = field(default_factory=lambda: _env(["LOCALAI_CORS", "CORS"], False, bool))
    cors_allow_origins: str = field(default_factory=lambda: _env(["LOCALAI_CORS_ALLOW_ORIGINS", "CORS_ALLOW_ORIGINS"], ""))
    csrf: bool = field(default_factory=lambda: _env(["LOCALAI_CSRF"], False, bool))
    upload_limit_mb: int = field(default_factory=lambda: _env(["LOCALAI_UPLOAD_LIMIT", "UPLOAD_LIMIT"], 15, int))
    api_keys: list = field(default_factory=lambda: _env(["LOCALAI_API_KEY", "API_KEY"], [], list))
    disable_webui: bool = field(default_factory=lambda: _env(["LOCALAI_DISABLE_WEBUI", "DISABLE_WEBUI"], False, bool))
    disable_gallery_endpoint: bool = field(default_factory=lambda: _env(["LOCALAI_DISABLE_GALLERY_ENDPOINT"], False, bool))
    disable_metrics_endpoint: bool = field(default_factory=lambda: _env(["LOCALAI_DISABLE_METRICS_ENDPOINT"], False, bool))
    disable_api_key_requirement_for_http_get: bool = field(default_factory=lambda: _env(["LOCALAI_DISABLE_API_KEY_REQUIREMENT_FOR_HTTP_GET"], False, bool))
    http_get_exempted_endpoints: list = field(default_factory=lambda: _env(["LOCALAI_HTTP_GET_EXEMPTED_ENDPOINTS"], [r"^/$", r"^/browse/?$", r"^/talk/?$", r"^/p2p/?$", r"^/chat/?$", r"^/text2image/?$", r"^/tts/?$", r"^/static/.*$", r"^/swagger.*$"], list))
    use_subtle_key_comparison: bool = field(default_factory=lambda: _env(["LOCALAI_SUBTLE_KEY_COMPARISON"], False, bool))
    opaque_errors: bool = field(default_factory=lambda: _env(["LOCALAI_OPAQUE_ERRORS"], False, bool))
    machine_tag: str = field(default_factory=lambda: _env(["LOCALAI_MACHINE_TAG", "MACHINE_TAG"], ""))
    # inference
    context_size: int = field(default_factory=lambda: _env(["LOCALAI_CONTEXT_SIZE", "CONTEXT_SIZE"], 0, int))
    threads: int = field(default_factory=lambda: _env(["LOCALAI_THREADS", "THREADS"], 0, int))
    f16: bool = field(default_factory=lambda: _env(["LOCALAI_F16", "F16"], False, bool))
    debug: bool = field(default_factory=lambda: _env(["LOCALAI_LOG_LEVEL", "LOG_LEVEL"], "info") == "debug")
    parallel_backend_requests: bool = field(default_factory=lambda: _env(["LOCALAI_PARALLEL_REQUESTS", "PARALLEL_REQUESTS"], True, bool))
    single_active_backend: bool = field(default_factory=lambda: _env(["LOCALAI_SINGLE_ACTIVE_BACKEND", "SINGLE_ACTIVE_BACKEND"], False, bool))
    preload_backend_only: bool = field(default_factory=lambda: _env(["LOCALAI_PRELOAD_BACKEND_ONLY", "PRELOAD_BACKEND_ONLY"], False, bool))
    external_grpc_backends: dict = field(default_factory=dict)
    load_to_memory: list = field(default_factory=lambda: _env(["LOCALAI_LOAD_TO_MEMORY", "LOAD_TO_MEMORY"], [], list))
    # watchdog (core/cli/run.go:65-68)
    watchdog_idle: bool = field(default_factory=lambda: _env(["LOCALAI_WATCHDOG_IDLE", "WATCHDOG_IDLE"], False, bool))
    watchdog_idle_timeout_s: float = field(default_factory=lambda: _duration(_env(["LOCALAI_WATCHDOG_IDLE_TIMEOUT", "WATCHDOG_IDLE_TIMEOUT"], "15m")))
    watchdog_busy: bool = field(default_factory=lambda: _env(["LOCALAI_WATCHDOG_BUSY", "WATCHDOG_BUSY"], False, bool))
    watchdog_busy_timeout_s: float = field(default_factory=lambda: _duration(_env(["LOCALAI_WATCHDOG_BUSY_TIMEOUT", "WATCHDOG_BUSY_TIMEOUT"], "5m")))
    force_backend_shutdown: bool = field(default_factory=lambda: _env(["LOCALAI_FORCE_BACKEND_SHUTDOWN"], False, bool))
    # p2p / federation
    p2p: bool = field(default_factory=lambda: _env(["LOCALAI_P2P", "P2P"], False, bool))
    p2p_token: str = field(default_factory=lambda: _env(["LOCALAI_P2P_TOKEN", "P2P_TOKEN", "TOKEN"], ""))
    p2p_network_id: str = field(default_factory=lambda: _env(["LOCALAI_P2P_NETWORK_ID", "P2P_NETWORK_ID"], ""))
    # intervals written into a generated token (core/cli/run.go:57-58)
    p2p_dht_interval: int = field(default_factory=lambda: _env(["LOCALAI_P2P_DHT_INTERVAL", "P2P_DHT_INTERVAL"], 360, int))
    p2p_otp_interval: int = field(default_factory=lambda: _env(["LOCALAI_P2P_OTP_INTERVAL", "P2P_OTP_INTERVAL"], 9000, int))
    # federator / peer URLs this instance announces itself to (libp2p discovery replacement)
    p2p_peers: list = field(default_factory=lambda: _env(["LOCALAI_P2P_PEERS", "P2P_PEERS"], [], list))
    # LAN discovery beacons (the reference's libp2p mDNS, on by default with p2p); unicast targets for
    # networks without multicast
    p2p_lan_discovery: bool = field(default_factory=lambda: not _env(["LOCALAI_P2P_DISABLE_LAN_DISCOVERY"], False, bool))
    p2p_discovery_targets: list = field(default_factory=lambda: _env(["LOCALAI_P2P_DISCOVERY_TARGETS"], [], list))
    federated: bool = field(default_factory=lambda: _env(["LOCALAI_FEDERATED", "FEDERATED"], False, bool))
    # MI355X specifics
    gpus: str = field(default_factory=lambda: _env(["LOCALAI_GPUS", "HIP_VISIBLE_DEVICES"], ""))
    # best-effort HF safety scan before every gallery download (core/cli/run.go:50 DisablePredownloadScan)
    enforce_predownload_scans: bool = field(
        default_factory=lambda: not _env(["LOCALAI_DISABLE_PREDOWNLOAD_SCAN"], False, bool))
    version: str = "v0.1.0-mi355x"

    @property
    def host_port(self) -> tuple[str, int]:
        a = self.address
        if a.startswith(":"):
            return "0.0.0.0", int(a[1:])
        h, _, p = a.rpartition(":")
        return h or "0.0.0.0", int(p)

    def ensure_dirs(self):
        for d in (self.models_path, self.generated_content_dir, self.upload_dir, self.config_dir):
            if d:
                os.makedirs(d, exist_ok=True)
        for sub in ("audio", "images", "videos"):
            os.makedirs(os.path.join(self.generated_content_dir, sub), exist_ok=True)


def _duration(s) -> float:
    """Go-style duration string ("15m", "1h30m", "45s") -> seconds."""
    if isinstance(s, (int, float)):
        return float(s)
    import re
    total = 0.0
    for num, unit in re.findall(r"([\d.]+)(ms|h|m|s)", str(s)):
        total += float(num) * {"h": 3600, "m": 60, "s": 1, "ms": 1e-3}[unit]
    return total or float(s or 0)
