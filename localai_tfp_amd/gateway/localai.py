"""LocalAI-specific endpoints: gallery jobs, stores, VAD, backend monitor/shutdown, tokenize,
system info, p2p, token metrics.

Behavioural parity: core/http/routes/localai.go:15-96; endpoints/localai/gallery.go:30-213,
stores.go:12-125, vad.go:19, backend_monitor.go:14,35, tokenize.go:17, system.go:14, p2p.go:14,28,
get_token_metrics.go:24; services/backend_monitor.go:18-140; core/backend/stores.go."""
from __future__ import annotations

import os

from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse, Response

from ..config.model_config import FLAG_TOKENIZE, FLAG_VAD, ModelConfig
from ..grpc import pb
from .openai import app_of
from .request import RequestError

router = APIRouter()


# ------------------------------------------------------------------------------------------------
# gallery (G14)

def _gallery_enabled(a):
    if a.cfg.disable_gallery_endpoint:
        raise RequestError("gallery endpoint disabled", 404)


@router.post("/models/apply")
async def models_apply(request: Request):
    from ..gallery import GalleryModel
    a = app_of(request)
    _gallery_enabled(a)
    body = await request.json()
    req = GalleryModel.from_dict(body)
    gid = body.get("id", "")
    if gid:
        uid = a.gallery.submit(name=gid, req=req)
    elif body.get("config_url"):
        uid = a.gallery.submit(req=req, config_url=body["config_url"])
    else:
        uid = a.gallery.submit(req=req)
    return {"uuid": uid, "status": f"{str(request.base_url).rstrip('/')}/models/jobs/{uid}"}


@router.post("/models/delete/{name}")
async def models_delete(request: Request, name: str):
    a = app_of(request)
    _gallery_enabled(a)
    uid = a.gallery.submit(name=name, delete=True)
    a.loader.shutdown_model(name)
    a.configs.remove(name)
    return {"uuid": uid, "status": f"{str(request.base_url).rstrip('/')}/models/jobs/{uid}"}


@router.get("/models/available")
async def models_available(request: Request):
    import asyncio
    from ..gallery import available_models
    a = app_of(request)
    _gallery_enabled(a)
    ms = await asyncio.get_running_loop().run_in_executor(None, available_models, a.gallery.galleries,
                                                         a.cfg.models_path)
    return [m.to_dict() for m in ms]


@router.get("/models/galleries")
async def galleries_list(request: Request):
    a = app_of(request)
    return [{"name": g.name, "url": g.url} for g in a.gallery.galleries]


@router.post("/models/galleries")
async def galleries_add(request: Request):
    from ..gallery import Gallery
    a = app_of(request)
    body = await request.json()
    g = Gallery.parse(body)
    if any(x.name == g.name for x in a.gallery.galleries):
        raise RequestError(f"gallery {g.name!r} already exists")
    a.gallery.galleries.append(g)
    return [{"name": x.name, "url": x.url} for x in a.gallery.galleries]


@router.delete("/models/galleries")
async def galleries_del(request: Request):
    a = app_of(request)
    body = await request.json()
    name = body.get("name", "")
    before = len(a.gallery.galleries)
    a.gallery.galleries = [g for g in a.gallery.galleries if g.name != name]
    if len(a.gallery.galleries) == before:
        raise RequestError(f"gallery {name!r} not found", 404)
    return [{"name": x.name, "url": x.url} for x in a.gallery.galleries]


@router.get("/models/jobs/{uid}")
async def job(request: Request, uid: str):
    st = app_of(request).gallery.get_status(uid)
    if st is None:
        raise RequestError("could not find any status for ID", 404)
    return st.to_dict()


@router.get("/models/jobs")
async def jobs(request: Request):
    return {k: v.to_dict() for k, v in app_of(request).gallery.all_status().items()}


# ------------------------------------------------------------------------------------------------
# stores (G24 / N11)

def _store_cfg(name: str) -> ModelConfig:
    c = ModelConfig(name=f"__store__{name or 'default'}", backend="local-store")
    c.parameters.model = name or "default"
    c.set_defaults()
    return c


def _keys(ks):
    return [pb.StoresKey(Floats=[float(x) for x in k]) for k in ks]


@router.post("/stores/set")
async def stores_set(request: Request):
    a = app_of(request)
    b = await request.json()
    r = await a.inference.rpc(_store_cfg(b.get("store", "")), "StoresSet", pb.StoresSetOptions(
        Keys=_keys(b.get("keys", [])), Values=[pb.StoresValue(Bytes=str(v).encode()) for v in b.get("values", [])]))
    if not r.success:
        raise RequestError(r.message or "set failed", 500)
    return Response(status_code=200)


@router.post("/stores/delete")
async def stores_delete(request: Request):
    a = app_of(request)
    b = await request.json()
    r = await a.inference.rpc(_store_cfg(b.get("store", "")), "StoresDelete",
                              pb.StoresDeleteOptions(Keys=_keys(b.get("keys", []))))
    if not r.success:
        raise RequestError(r.message or "delete failed", 500)
    return Response(status_code=200)


@router.post("/stores/get")
async def stores_get(request: Request):
    a = app_of(request)
    b = await request.json()
    r = await a.inference.rpc(_store_cfg(b.get("store", "")), "StoresGet",
                              pb.StoresGetOptions(Keys=_keys(b.get("keys", []))))
    return {"keys": [list(k.Floats) for k in r.Keys], "values": [v.Bytes.decode(errors="replace") for v in r.Values]}


@router.post("/stores/find")
async def stores_find(request: Request):
    a = app_of(request)
    b = await request.json()
    r = await a.inference.rpc(_store_cfg(b.get("store", "")), "StoresFind", pb.StoresFindOptions(
        Key=pb.StoresKey(Floats=[float(x) for x in b.get("key", [])]), TopK=int(b.get("topk", 0))))
    return {"keys": [list(k.Floats) for k in r.Keys], "values": [v.Bytes.decode(errors="replace") for v in r.Values],
            "similarities": list(r.Similarities)}


# ------------------------------------------------------------------------------------------------
# VAD / tokenize / metrics

@router.post("/vad")
@router.post("/v1/vad")
async def vad(request: Request):
    a = app_of(request)
    b = await request.json()
    name = b.get("model") or a.first_model_for(FLAG_VAD)
    cfg = a.configs.load_by_name(name)
    if not cfg.backend:
        cfg.backend = "silero-vad"
    r = await a.inference.vad(cfg, [float(x) for x in b.get("audio", [])])
    return {"segments": [{"start": s.start, "end": s.end} for s in r.segments]}


@router.post("/v1/tokenize")
async def tokenize(request: Request):
    a = app_of(request)
    b = await request.json()
    name = b.get("model") or a.first_model_for(FLAG_TOKENIZE)
    cfg = a.configs.load_by_name(name)
    toks = await a.inference.tokenize(cfg, b.get("content", ""))
    return {"tokens": toks}


@router.get("/v1/tokenMetrics")
async def token_metrics(request: Request):
    """get_token_metrics.go (not routed in the reference; routed here)."""
    a = app_of(request)
    name = request.query_params.get("model") or request.headers.get("model") or a.first_model_for(0)
    cfg = a.configs.load_by_name(name)
    m = await a.inference.metrics(cfg)
    return {"slot_id": m.slot_id, "prompt_json_for_slot": m.prompt_json_for_slot,
            "tokens_per_second": m.tokens_per_second, "tokens_generated": m.tokens_generated,
            "prompt_tokens_processed": m.prompt_tokens_processed}


# ------------------------------------------------------------------------------------------------
# backend monitor / shutdown / system

def _sample_process(pid: int) -> dict:
    import psutil
    p = psutil.Process(pid)
    mi = p.memory_info()
    return {"memory_info": {"rss": mi.rss, "vms": mi.vms}, "memory_percent": p.memory_percent(),
            "cpu_percent": p.cpu_percent(interval=0.1)}


@router.get("/backend/monitor")
@router.get("/v1/backend/monitor")
async def backend_monitor(request: Request):
    a = app_of(request)
    try:
        b = await request.json()
    except ValueError:
        b = {}
    name = b.get("model") or request.query_params.get("model", "")
    m = a.loader.get(name)
    if m is None:
        raise RequestError(f"model {name!r} is not loaded", 404)
    try:
        st = await m.apick().call("Status", pb.HealthMessage(), timeout=10)
        return {"state": int(st.state), "memory": {"total": st.memory.total, "breakdown": dict(st.memory.breakdown)}}
    except Exception:
        r = m.replicas[0]
        if r.proc is None:
            raise RequestError("backend has no local process to sample", 500)
        return _sample_process(r.proc.pid)


@router.post("/backend/shutdown")
@router.post("/v1/backend/shutdown")
async def backend_shutdown(request: Request):
    import asyncio
    a = app_of(request)
    b = await request.json()
    name = b.get("model", "")
    ok = await asyncio.get_running_loop().run_in_executor(None, a.loader.shutdown_model, name)
    if not ok:
        raise RequestError(f"model {name!r} is not loaded", 404)
    return Response(status_code=200)


@router.get("/system")
async def system(request: Request):
    from .. import workers as W
    a = app_of(request)
    loaded = [{"id": n} for n in a.loader.list_loaded()]
    import asyncio
    from .observability import gpu_metrics
    # AMD SMI (driver interface: utilisation, HBM use, power, temperature) — no HIP context in the gateway
    gpus = await asyncio.to_thread(gpu_metrics)
    return {"backends": sorted(W.WORKERS), "loaded_models": loaded, "gpus": gpus}


# ------------------------------------------------------------------------------------------------
# p2p (C3): token + node listing for federated / worker mode

@router.get("/api/p2p")
async def p2p_nodes(request: Request):
    a = app_of(request)
    p = a.p2p
    if p is None:
        return {"nodes": [], "federated_nodes": []}
    return {"nodes": p.nodes("worker"), "federated_nodes": p.nodes("federated")}


@router.post("/api/p2p/register")
async def p2p_register(request: Request):
    """Node announcement (replaces the libp2p ledger write of p2p.go nodeAnnounce)."""
    from .. import p2p as P
    a = app_of(request)
    if a.p2p is None:
        return JSONResponse({"error": "p2p is not enabled"}, status_code=404)
    if not a.p2p.registry.authorised(request.headers.get("authorization")):
        return JSONResponse({"error": "invalid token"}, status_code=401)
    d = await request.json()
    a.p2p.registry.add(P.NodeData(id=str(d["id"]), name=d.get("name", ""), address=d.get("address", ""),
                                  service=d.get("service", P.WORKER_ID)))
    return {"ok": True}


@router.get("/api/p2p/token")
async def p2p_token(request: Request):
    a = app_of(request)
    return Response(a.cfg.p2p_token or "", media_type="text/plain")
