"""OpenAI files + assistants API (behavioural parity: core/http/endpoints/openai/files.go:24-194,
assistant.go:77-522). Metadata persists as JSON under the upload/config dirs."""
from __future__ import annotations

import datetime
import os
import re
import time

from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse, PlainTextResponse, Response

from .multipart import read_form
from .openai import app_of

router = APIRouter()
MAX_FILE_IDS = 20


def _sanitize(name: str) -> str:
    name = os.path.basename(name.replace("\\", "/"))
    return re.sub(r"[^A-Za-z0-9._-]", "_", name) or "file"


def _next_id(items: list[dict], prefix: str) -> str:
    n = 0
    for it in items:
        m = re.match(rf"{prefix}-(\d+)$", str(it.get("id", "")))
        if m:
            n = max(n, int(m.group(1)))
    return f"{prefix}-{n + 1}"


def _bad(msg: str, code: int = 400):
    return PlainTextResponse(msg, status_code=code)


# ------------------------------------------------------------------------------------------------
# files

@router.post("/v1/files")
@router.post("/files")
async def upload_file(request: Request):
    a = app_of(request)
    form = await read_form(request)
    up = form.get("file")
    if up is None or not hasattr(up, "read"):
        return _bad("file is required")
    data = await up.read()
    if len(data) > a.cfg.upload_limit_mb * 1024 * 1024:
        return _bad(f"File size {len(data)} exceeds upload limit {a.cfg.upload_limit_mb}")
    purpose = form.get("purpose") or ""
    if not purpose:
        return _bad("Purpose is not defined")
    fname = _sanitize(up.filename or "file")
    path = os.path.join(a.cfg.upload_dir, fname)
    if os.path.exists(path):
        return _bad("File already exists")
    with open(path, "wb") as f:
        f.write(data)
    rec = {"id": _next_id(a.files.items, "file"), "object": "file", "bytes": len(data),
           "created_at": datetime.datetime.now(datetime.timezone.utc).isoformat(), "filename": fname,
           "purpose": purpose}
    a.files.items.append(rec)
    a.files.save()
    return rec


@router.get("/v1/files")
@router.get("/files")
async def list_files(request: Request):
    a = app_of(request)
    purpose = request.query_params.get("purpose", "")
    data = [f for f in a.files.items if not purpose or f.get("purpose") == purpose]
    return {"data": data, "object": "list"}


def _find_file(a, fid: str):
    return next((f for f in a.files.items if f.get("id") == fid), None)


@router.get("/v1/files/{file_id}")
@router.get("/files/{file_id}")
async def get_file(request: Request, file_id: str):
    f = _find_file(app_of(request), file_id)
    return f if f else _bad(f"unable to find file id {file_id}", 404)


@router.delete("/v1/files/{file_id}")
@router.delete("/files/{file_id}")
async def delete_file(request: Request, file_id: str):
    a = app_of(request)
    f = _find_file(a, file_id)
    if f is None:
        return _bad(f"unable to find file id {file_id}", 404)
    try:
        os.remove(os.path.join(a.cfg.upload_dir, f["filename"]))
    except FileNotFoundError:
        pass
    a.files.items = [x for x in a.files.items if x is not f]
    a.files.save()
    return {"id": file_id, "object": "file", "deleted": True}


@router.get("/v1/files/{file_id}/content")
@router.get("/files/{file_id}/content")
async def file_content(request: Request, file_id: str):
    a = app_of(request)
    f = _find_file(a, file_id)
    if f is None:
        return _bad(f"unable to find file id {file_id}", 404)
    with open(os.path.join(a.cfg.upload_dir, f["filename"]), "rb") as fh:
        return Response(fh.read(), media_type="application/octet-stream")


# ------------------------------------------------------------------------------------------------
# assistants

_FIELDS = ("model", "name", "description", "instructions", "tools", "file_ids", "metadata")


@router.post("/v1/assistants")
@router.post("/assistants")
async def create_assistant(request: Request):
    a = app_of(request)
    try:
        b = await request.json()
    except ValueError:
        return JSONResponse({"error": "Cannot parse JSON"}, status_code=400)
    if not a.model_exists(b.get("model", "")):
        return _bad(f"Model {b.get('model', '')!r} not found")
    asst = {"id": f"asst_{int(time.time() * 1e6)}", "object": "assistant", "created": int(time.time())}
    for k in _FIELDS:
        if k in b:
            asst[k] = b[k]
    a.assistants.items.append(asst)
    a.assistants.save()
    return asst


@router.get("/v1/assistants")
@router.get("/assistants")
async def list_assistants(request: Request):
    a = app_of(request)
    q = request.query_params
    try:
        limit = int(q.get("limit", "20"))
    except ValueError:
        return _bad(f"Invalid limit query value: {q.get('limit')}")
    items = sorted(a.assistants.items, key=lambda x: x.get("created", 0), reverse=q.get("order", "desc") != "asc")
    ids = [x["id"] for x in items]
    if q.get("after") in ids:
        items = items[ids.index(q["after"]) + 1:]
    if q.get("before") in ids:
        items = items[:ids.index(q["before"])]
    return items[:limit]


def _find_asst(a, aid):
    return next((x for x in a.assistants.items if x.get("id") == aid), None)


@router.get("/v1/assistants/{aid}")
@router.get("/assistants/{aid}")
async def get_assistant(request: Request, aid: str):
    x = _find_asst(app_of(request), aid)
    return x if x else _bad(f"Unable to find assistant with id: {aid}", 404)


@router.post("/v1/assistants/{aid}")
@router.post("/assistants/{aid}")
async def modify_assistant(request: Request, aid: str):
    a = app_of(request)
    x = _find_asst(a, aid)
    if x is None:
        return _bad(f"Unable to find assistant with id: {aid}", 404)
    b = await request.json()
    for k in _FIELDS:
        if k in b:
            x[k] = b[k]
    a.assistants.save()
    return x


@router.delete("/v1/assistants/{aid}")
@router.delete("/assistants/{aid}")
async def delete_assistant(request: Request, aid: str):
    a = app_of(request)
    x = _find_asst(a, aid)
    if x is None:
        return JSONResponse({"id": aid, "object": "assistant.deleted", "deleted": False}, status_code=404)
    a.assistants.items = [y for y in a.assistants.items if y is not x]
    a.assistants.save()
    return {"id": aid, "object": "assistant.deleted", "deleted": True}


@router.post("/v1/assistants/{aid}/files")
@router.post("/assistants/{aid}/files")
async def create_assistant_file(request: Request, aid: str):
    a = app_of(request)
    x = _find_asst(a, aid)
    if x is None:
        return _bad(f"Unable to find {aid!r}", 404)
    b = await request.json()
    fid = b.get("file_id", "")
    if len(x.get("file_ids", [])) >= MAX_FILE_IDS:
        return _bad(f"Max files {MAX_FILE_IDS} for assistant {x.get('name', '')} reached.")
    if _find_file(a, fid) is None:
        return _bad(f"Unable to find file_id: {fid}", 404)
    x.setdefault("file_ids", []).append(fid)
    rec = {"id": fid, "object": "assistant.file", "created_at": int(time.time()), "assistant_id": aid}
    a.assistant_files.items.append(rec)
    a.assistants.save()
    a.assistant_files.save()
    return rec


@router.get("/v1/assistants/{aid}/files")
@router.get("/assistants/{aid}/files")
async def list_assistant_files(request: Request, aid: str):
    a = app_of(request)
    q = request.query_params
    try:
        limit = int(q.get("limit", "20"))
    except ValueError:
        limit = 20
    if not 1 <= limit <= 100:
        limit = 20
    items = sorted((f for f in a.assistant_files.items if f.get("assistant_id") == aid),
                   key=lambda f: f.get("created_at", 0), reverse=q.get("order", "desc") != "asc")
    data = items[:limit]
    return {"object": "list", "data": data, "first_id": data[0]["id"] if data else "",
            "last_id": data[-1]["id"] if data else "", "has_more": len(items) > limit}


@router.get("/v1/assistants/{aid}/files/{fid}")
@router.get("/assistants/{aid}/files/{fid}")
async def get_assistant_file(request: Request, aid: str, fid: str):
    a = app_of(request)
    f = next((f for f in a.assistant_files.items if f.get("assistant_id") == aid and f.get("id") == fid), None)
    return f if f else _bad(f"Unable to find assistant file {fid}", 404)


@router.delete("/v1/assistants/{aid}/files/{fid}")
@router.delete("/assistants/{aid}/files/{fid}")
async def delete_assistant_file(request: Request, aid: str, fid: str):
    a = app_of(request)
    x = _find_asst(a, aid)
    f = next((f for f in a.assistant_files.items if f.get("assistant_id") == aid and f.get("id") == fid), None)
    if x is None or f is None:
        return JSONResponse({"id": fid, "object": "assistant.file.deleted", "deleted": False}, status_code=404)
    x["file_ids"] = [i for i in x.get("file_ids", []) if i != fid]
    a.assistant_files.items = [y for y in a.assistant_files.items if y is not f]
    a.assistants.save()
    a.assistant_files.save()
    return {"id": fid, "object": "assistant.file.deleted", "deleted": True}
