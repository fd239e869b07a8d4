"""ElevenLabs- and Jina-compatible endpoints (behavioural parity: core/http/routes/elevenlabs.go:12-29,
endpoints/elevenlabs/tts.go, soundgeneration.go; routes/jina.go:11-24, endpoints/jina/rerank.go:20)."""
from __future__ import annotations

import os
import uuid

from fastapi import APIRouter, Request
from fastapi.responses import FileResponse

from ..config.model_config import FLAG_RERANK, FLAG_SOUND_GENERATION, FLAG_TTS
from .media import run_tts
from .openai import app_of
from .request import RequestError

router = APIRouter()


@router.post("/v1/text-to-speech/{voice_id}")
async def elevenlabs_tts(request: Request, voice_id: str):
    a = app_of(request)
    b = await request.json()
    model = b.get("model_id") or a.first_model_for(FLAG_TTS)
    if not model:
        raise RequestError("model_id is required")
    path = await run_tts(a, {"input": b.get("text", ""), "voice": voice_id, "language": b.get("language_code", "")},
                         model)
    return FileResponse(path, filename=os.path.basename(path))


@router.post("/v1/sound-generation")
async def elevenlabs_sound(request: Request):
    a = app_of(request)
    b = await request.json()
    model = b.get("model_id") or a.first_model_for(FLAG_SOUND_GENERATION)
    if not model:
        raise RequestError("model_id is required")
    cfg = a.configs.load_by_name(model)
    adir = os.path.join(a.cfg.generated_content_dir, "audio")
    os.makedirs(adir, exist_ok=True)
    dst = os.path.join(adir, f"sound_{uuid.uuid4().hex}.wav")
    kw = dict(text=b.get("text", ""), model=cfg.parameters.model, dst=dst)
    if b.get("duration_seconds") is not None:
        kw["duration"] = float(b["duration_seconds"])
    if b.get("prompt_influence") is not None:
        kw["temperature"] = float(b["prompt_influence"])
    if b.get("do_sample") is not None:
        kw["sample"] = bool(b["do_sample"])
    await a.inference.sound(cfg, **kw)
    return FileResponse(dst, filename=os.path.basename(dst))


@router.post("/v1/rerank")
async def jina_rerank(request: Request):
    a = app_of(request)
    b = await request.json()
    model = b.get("model") or a.first_model_for(FLAG_RERANK)
    if not model:
        raise RequestError("model is required")
    cfg = a.configs.load_by_name(model)
    if b.get("backend"):
        cfg.backend = b["backend"]
    r = await a.inference.rerank(cfg, b.get("query", ""), list(b.get("documents", [])), int(b.get("top_n", 0)))
    return {"model": model, "usage": {"total_tokens": r.usage.total_tokens, "prompt_tokens": r.usage.prompt_tokens},
            "results": [{"index": d.index, "document": {"text": d.text}, "relevance_score": d.relevance_score}
                        for d in r.results]}
