"""HTTP application: FastAPI app, middleware chain and route registration.

Behavioural parity: core/http/app.go:53-215 (JSON error handler / opaque errors, middleware order:
machine tag, request logging, recover, metrics, health, key auth, CORS, CSRF), auth
middleware/auth.go:18-97 (API keys, constant-time compare option, GET exemptions by regex,
keys hot-reloaded from api_keys.json), metrics services/metrics.go:13-54, health
routes/health.go:5-13."""
from __future__ import annotations

import contextlib
import hmac
import asyncio
import logging
import re
import time

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse

from ..config.app_config import ApplicationConfig
from .request import RequestError
from .state import Application

log = logging.getLogger("localai_tfp_amd.gateway")

from .observability import API_LATENCY, REGISTRY as _REGISTRY, prom

def _error(status: int, msg: str, typ: str = "invalid_request_error") -> JSONResponse:
    return JSONResponse({"error": {"code": status, "message": msg, "type": typ}}, status_code=status)


class GatewayMiddleware:
    """Pure-ASGI middleware (auth + latency metrics + machine tag). Starlette's BaseHTTPMiddleware
    pushes every streamed body chunk through an anyio memory stream, which dominated the gateway's
    CPU profile under SSE load; this one only wraps `send` when it has to."""

    def __init__(self, app, state, exempt, health_paths):
        self.app, self.state, self.exempt, self.health = app, state, exempt, health_paths
        c = state.cfg
        self.cfg = c
        self.metrics = API_LATENCY if (not c.disable_metrics_endpoint and API_LATENCY is not None) else None
        self.tag = c.machine_tag.encode() if c.machine_tag else None

    def _authorized(self, scope) -> bool:
        keys = self.state.all_api_keys
        path = scope["path"]
        if not keys or path in self.health:
            return True
        c = self.cfg
        if scope["method"] == "GET" and (c.disable_api_key_requirement_for_http_get or
                                         any(r.match(path) for r in self.exempt)):
            return True
        hdr = {k: v for k, v in scope["headers"] if k in (b"authorization", b"x-api-key", b"xi-api-key")}
        auth = hdr.get(b"authorization", b"").decode("latin-1")
        if auth.lower().startswith("bearer "):
            tok = auth[7:]
        else:
            tok = (hdr.get(b"x-api-key") or hdr.get(b"xi-api-key") or b"").decode("latin-1")
        if c.use_subtle_key_comparison:
            return any(hmac.compare_digest(tok.encode(), k.encode()) for k in keys)
        return tok in keys

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        if not self._authorized(scope):
            resp = PlainTextResponse("", status_code=401) if self.cfg.opaque_errors else \
                _error(401, "An authentication key is required", "invalid_request_error")
            return await resp(scope, receive, send)
        if self.tag is not None:
            inner_send = send

            async def send(msg, _s=inner_send):
                if msg["type"] == "http.response.start":
                    msg = dict(msg)
                    msg["headers"] = list(msg.get("headers", [])) + [(b"machine-tag", self.tag)]
                await _s(msg)
        if self.metrics is None or scope["path"] == "/metrics":
            return await self.app(scope, receive, send)
        t0 = time.perf_counter()
        try:
            await self.app(scope, receive, send)
        finally:
            self.metrics.labels(scope["method"], scope["path"]).observe(time.perf_counter() - t0)


def create_app(cfg: ApplicationConfig | None = None, inproc: bool | None = None, startup: bool = True) -> FastAPI:
    state = Application(cfg, inproc)
    c = state.cfg
    @contextlib.asynccontextmanager
    async def lifespan(_app):
        import os
        prof = None
        if os.environ.get("LOCALAI_CPROFILE"):  # diagnostics: profile the serving process
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        if startup:
            import asyncio
            await asyncio.get_running_loop().run_in_executor(None, state.startup)
        yield
        state.shutdown()
        if prof is not None:
            prof.disable()
            prof.dump_stats(os.environ["LOCALAI_CPROFILE"])

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

    app.add_middleware(GatewayMiddleware, state=state, exempt=exempt, health_paths=health_paths)

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
        from . import observability as obs
        await obs.scrape_backends(state)
        await asyncio.to_thread(obs.export_gpu_metrics)
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
