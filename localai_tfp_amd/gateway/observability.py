"""Prometheus metrics of the gateway (reference: core/services/metrics.go:13-54 — the `api_call`
latency histogram), extended with the serving metrics an LLM deployment is operated on:

* client-observed latency per model: time to first token and time per output token of every
  streamed completion (histograms), output tokens and requests (counters);
* engine state of every loaded backend, scraped from its Status RPC on each /metrics request
  (KV-cache blocks used / total, running / waiting sequences, engine steps, busy seconds, generated
  and prompt tokens, weights and KV bytes) as gauges;
* GPU utilisation, HBM use, power and temperature through AMD SMI (amdsmi, the driver interface —
  no HIP context is created in the gateway), also served on /system.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time

log = logging.getLogger("localai_tfp_amd.gateway")

try:
    import prometheus_client as prom
    REGISTRY = prom.CollectorRegistry()
    API_LATENCY = prom.Histogram("api_call", "duration of API calls", ["method", "path"], registry=REGISTRY,
                                 buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120))
    TTFT = prom.Histogram("localai_time_to_first_token_seconds", "time from request to the first streamed token",
                          ["model"], registry=REGISTRY,
                          buckets=(0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2, 4, 8, 16, 32))
    TPOT = prom.Histogram("localai_time_per_output_token_seconds", "mean inter-token time of a streamed completion",
                          ["model"], registry=REGISTRY,
                          buckets=(0.002, 0.005, 0.01, 0.015, 0.02, 0.03, 0.05, 0.075, 0.1, 0.2, 0.5, 1))
    OUT_TOKENS = prom.Counter("localai_output_tokens", "streamed output tokens", ["model"], registry=REGISTRY)
    REQUESTS = prom.Counter("localai_completion_requests", "streamed completion requests", ["model", "status"],
                            registry=REGISTRY)
    BACKEND = prom.Gauge("localai_backend_state", "engine state of a loaded backend (Status RPC breakdown)",
                         ["model", "key"], registry=REGISTRY)
    GPU = prom.Gauge("localai_gpu", "AMD SMI GPU metrics", ["gpu", "key"], registry=REGISTRY)
except ImportError:  # pragma: no cover
    prom = REGISTRY = API_LATENCY = TTFT = TPOT = OUT_TOKENS = REQUESTS = BACKEND = GPU = None


class StreamTimer:
    """Per-request timing of a streamed completion: chunk(n) for every content chunk, close(ok)."""

    def __init__(self, model: str):
        self.model = model or "unknown"
        self.t0 = time.perf_counter()
        self.t_first = None
        self.t_last = None
        self.n = 0

    def chunk(self, n_tokens: int = 1):
        now = time.perf_counter()
        if self.t_first is None:
            self.t_first = now
            if TTFT is not None:
                TTFT.labels(self.model).observe(now - self.t0)
        self.t_last = now
        self.n += max(0, int(n_tokens))

    def close(self, ok: bool = True):
        if prom is None:
            return
        REQUESTS.labels(self.model, "ok" if ok else "error").inc()
        if self.n:
            OUT_TOKENS.labels(self.model).inc(self.n)
        if self.t_first is not None and self.n > 1:
            TPOT.labels(self.model).observe((self.t_last - self.t_first) / (self.n - 1))


# ---------------------------------------------------------------- engine state of loaded backends
async def scrape_backends(app_state, timeout: float = 2.0):
    """Status RPC of every loaded model's first replica -> localai_backend_state{model,key}."""
    if BACKEND is None:
        return
    from ..grpc import pb
    loader = app_state.loader
    for name in loader.list_loaded():
        m = loader.get(name)
        if m is None or not getattr(m, "replicas", None):
            continue
        client = m.replicas[0].client
        try:
            st = await asyncio.wait_for(asyncio.to_thread(client.call, "Status", pb.HealthMessage(), timeout),
                                        timeout + 0.5)
        except Exception as ex:  # a busy or dead backend must not fail the scrape
            log.debug("status scrape of %s failed: %s", name, ex)
            continue
        BACKEND.labels(name, "state").set(int(st.state))
        for k, v in st.memory.breakdown.items():
            BACKEND.labels(name, k).set(float(v))


# ---------------------------------------------------------------- AMD SMI
_SMI = {"ok": None, "handles": []}


def gpu_metrics() -> list[dict]:
    """[{index, name, gfx_busy_percent, vram_used, vram_total, power_w, temp_c}] via amdsmi (empty list
    when AMD SMI is unavailable or MX_NO_SMI=1)."""
    if os.environ.get("MX_NO_SMI") == "1":
        return []
    try:
        import amdsmi
    except Exception:
        return []
    if _SMI["ok"] is None:
        try:
            amdsmi.amdsmi_init()
            _SMI["handles"] = list(amdsmi.amdsmi_get_processor_handles())
            _SMI["ok"] = True
        except Exception as ex:
            log.debug("amdsmi unavailable: %s", ex)
            _SMI["ok"] = False
    if not _SMI["ok"]:
        return []
    out = []
    for i, h in enumerate(_SMI["handles"]):
        d = {"index": i}

        def grab(key, fn):
            try:
                d[key] = fn()
            except Exception:
                pass
        grab("name", lambda: amdsmi.amdsmi_get_gpu_asic_info(h).get("market_name"))
        grab("gfx_busy_percent", lambda: amdsmi.amdsmi_get_gpu_activity(h).get("gfx_activity"))
        grab("vram_used", lambda: amdsmi.amdsmi_get_gpu_vram_usage(h).get("vram_used"))
        grab("vram_total", lambda: amdsmi.amdsmi_get_gpu_vram_usage(h).get("vram_total"))
        grab("power_w", lambda: amdsmi.amdsmi_get_power_info(h).get("average_socket_power"))
        grab("temp_c", lambda: amdsmi.amdsmi_get_temp_metric(h, amdsmi.AmdSmiTemperatureType.HOTSPOT,
                                                             amdsmi.AmdSmiTemperatureMetric.CURRENT))
        out.append(d)
    return out


def export_gpu_metrics():
    if GPU is None:
        return
    for d in gpu_metrics():
        for k, v in d.items():
            if k in ("index", "name") or not isinstance(v, (int, float)):
                continue
            GPU.labels(str(d["index"]), k).set(float(v))
