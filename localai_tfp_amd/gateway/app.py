"""HTTP application: FastAPI app, middleware chain and route registration.

Behavioural parity: core/http/app.go:53-215 (JSON error handler / opaque errors, middleware order:
machine tag, request logging, recover, metrics, health, key auth, CORS, CSRF), auth
middleware/auth.go:18-97 (API keys, constant-time compare option, GET exemptions by regex,
keys hot-reloaded from api_keys.json), metrics services/metrics.go:13-54, health
routes/health.go:5-13."""
from __future__ import annotations

import contextlib
import hmac
import logging
import re
import time

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse

from ..config.app_config import ApplicationConfig
from .request import RequestError
from .state import Application

log = logging.getLogger("localai_tfp_amd.gateway")

try:
    import prometheus_client as prom
    _REGISTRY = prom.CollectorRegistry()
    API_LATENCY = prom.Histogram("api_call", "duration of API calls", ["method", "path"], registry=_REGISTRY,
                                 buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120))
except ImportError:  # pragma: no cover
    prom = None
    _REGISTRY = None
    API_LATENCY = None


def _error(status: int, msg: str, typ: str = "invalid_request_error") -> JSONResponse:
    return JSONResponse({"error": {"code": status, "message": msg, "type": typ}}, status_code=status)


def create_app(cfg: ApplicationConfig | None = None, inproc: bool | None = None, startup: bool = True) -> FastAPI:
    state = Application(cfg, inproc)
    c = state.cfg
    @contextlib.asynccontextmanager
    async def lifespan(_app):
        if startup:
            import asyncio
            await asyncio.get_running_loop().run_in_executor(None, state.startup)
        yield
        state.shutdown()

    app = FastAPI(title="LocalAI (MI355X-native)", version=c.version, docs_url="/swagger/index.html",
                  openapi_url="/swagger/doc.json", lifespan=lifespan)
    app.state.localai = state

    # ---------------------------------------------------------------- errors
    @app.exception_handler(RequestError)
    async def _req_err(request: Request, ex: RequestError):
        if c.opaque_errors:
            return PlainTextResponse("", status_code=ex.status)
        return _error(ex.status, str(ex))

    @app.exception_handler(Exception)
    async def _any_err(request: Request, ex: Exception):
        log.exception("request failed: %s %s", request.method, request.url.path)
        if c.opaque_errors:
            return PlainTextResponse("", status_code=500)
        return _error(500, str(ex), "server_error")

    # ---------------------------------------------------------------- middleware (outermost last)
    exempt = [re.compile(p) for p in c.http_get_exempted_endpoints]
    health_paths = {"/healthz", "/readyz"}

    @app.middleware("http")
    async def auth_mw(request: Request, call_next):
        keys = state.all_api_keys
        path = request.url.path
        if keys and path not in health_paths:
            if not (request.method == "GET" and (c.disable_api_key_requirement_for_http_get or
                                                 any(r.match(path) for r in exempt))):
                auth = request.headers.get("authorization", "")
                tok = auth[7:] if auth.lower().startswith("bearer ") else (
                    request.headers.get("x-api-key") or request.headers.get("xi-api-key") or "")
                if c.use_subtle_key_comparison:
                    ok = any(hmac.compare_digest(tok.encode(), k.encode()) for k in keys)
                else:
                    ok = tok in keys
                if not ok:
                    if c.opaque_errors:
                        return PlainTextResponse("", status_code=401)
                    return _error(401, "An authentication key is required", "invalid_request_error")
        return await call_next(request)

    if not c.disable_metrics_endpoint and API_LATENCY is not None:
        @app.middleware("http")
        async def metrics_mw(request: Request, call_next):
            t0 = time.perf_counter()
            resp = await call_next(request)
            path = request.url.path
            if path != "/metrics":
                API_LATENCY.labels(request.method, path).observe(time.perf_counter() - t0)
            return resp

    if c.machine_tag:
        @app.middleware("http")
        async def tag_mw(request: Request, call_next):
            resp = await call_next(request)
            resp.headers["Machine-Tag"] = c.machine_tag
            return resp

    if c.cors:
        from fastapi.middleware.cors import CORSMiddleware
        origins = [o.strip() for o in c.cors_allow_origins.split(",") if o.strip()] or ["*"]
        app.add_middleware(CORSMiddleware, allow_origins=origins, allow_methods=["*"], allow_headers=["*"])

    # ---------------------------------------------------------------- routes
    @app.get("/healthz")
    @app.get("/readyz")
    async def health():
        return PlainTextResponse("OK")

    @app.get("/version")
    async def version():
        return {"version": c.version}

    @app.get("/metrics")
    async def metrics():
        if prom is None:
            return PlainTextResponse("", status_code=404)
        return PlainTextResponse(prom.generate_latest(_REGISTRY).decode(), media_type=prom.CONTENT_TYPE_LATEST)

    from . import localai as localai_routes
    from . import media as media_routes
    from . import openai as openai_routes
    from . import assistants as assistant_routes
    from . import thirdparty as thirdparty_routes
    app.include_router(openai_routes.router)
    app.include_router(media_routes.router)
    app.include_router(assistant_routes.router)
    app.include_router(localai_routes.router)
    app.include_router(thirdparty_routes.router)
    if not c.disable_webui:
        from . import ui as ui_routes
        app.include_router(ui_routes.router)
    return app
