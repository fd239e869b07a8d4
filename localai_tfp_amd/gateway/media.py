"""Media endpoints: images, audio transcription, speech, video, generated-content serving.

Behavioural parity: core/http/endpoints/openai/image.go:68-245, transcription.go:27,
localai/tts.go:25 (also served at /v1/audio/speech), localai/video.go:67, static dirs
core/http/app.go:168-170; backend side core/backend/image.go, transcript.go, tts.go, video.go."""
from __future__ import annotations

import asyncio
import base64
import os
import shutil
import tempfile
import time
import urllib.request
import uuid

from fastapi import APIRouter, Request
from fastapi.responses import FileResponse, JSONResponse

from ..config.model_config import FLAG_IMAGE, FLAG_TRANSCRIPT, FLAG_TTS, FLAG_VIDEO
from .multipart import read_form
from .openai import app_of, parse
from .request import RequestError

router = APIRouter()


def _safe_join(root: str, name: str) -> str:
    p = os.path.realpath(os.path.join(root, name))
    if not p.startswith(os.path.realpath(root) + os.sep):
        raise RequestError("invalid path", 404)
    return p


@router.get("/generated-images/{name}")
async def gen_image(request: Request, name: str):
    return FileResponse(_safe_join(os.path.join(app_of(request).cfg.generated_content_dir, "images"), name))


@router.get("/generated-audio/{name}")
async def gen_audio(request: Request, name: str):
    return FileResponse(_safe_join(os.path.join(app_of(request).cfg.generated_content_dir, "audio"), name))


@router.get("/generated-videos/{name}")
async def gen_video(request: Request, name: str):
    return FileResponse(_safe_join(os.path.join(app_of(request).cfg.generated_content_dir, "videos"), name))


def _materialize(a, data: str) -> str:
    """image.go: `file` is an http(s) URL or base64 -> temp file the backend can read."""
    if data.startswith(("http://", "https://")):
        with urllib.request.urlopen(data, timeout=60) as r:
            raw = r.read()
    else:
        raw = base64.b64decode(data.split(",", 1)[1] if data.startswith("data:") else data)
    fd, path = tempfile.mkstemp(prefix="b64", dir=a.cfg.generated_content_dir)
    with os.fdopen(fd, "wb") as f:
        f.write(raw)
    return path


@router.post("/v1/images/generations")
@router.post("/images/generations")
async def images(request: Request):
    a = app_of(request)
    req, cfg = await parse(request, FLAG_IMAGE)
    src = _materialize(a, req.file) if req.file else ""
    try:
        if cfg.backend in ("", "stablediffusion"):
            cfg.backend = "stablediffusion-ggml"
        size = req.size if "x" in (req.size or "") else "512x512"
        try:
            w, h = (int(x) for x in size.split("x"))
        except ValueError:
            raise RequestError("invalid value for 'size'")
        b64 = cfg.response_format == "b64_json"
        base_url = str(request.base_url).rstrip("/")
        jobs = []
        for prompt in cfg.prompt_strings:
            for _ in range(req.n or 1):
                pos, _, neg = prompt.partition("|")
                step = req.step or cfg.step or 15
                img_dir = os.path.join(a.cfg.generated_content_dir, "images")
                dst = os.path.join(img_dir if not b64 else a.cfg.generated_content_dir, f"b64{uuid.uuid4().hex}.png")
                jobs.append((dst, a.inference.image(
                    cfg, height=h, width=w, mode=req.mode, step=step, seed=cfg.resolved_seed(),
                    positive_prompt=pos, negative_prompt=neg, dst=dst, src=src,
                    EnableParameters=cfg.diffusers.enable_parameters, CLIPSkip=cfg.diffusers.clip_skip)))
        # the reference renders the N images one after another (image.go:158-226); here they are
        # issued together so data-parallel replicas (one per GPU) render them concurrently
        await asyncio.gather(*(j for _, j in jobs))
        out = []
        for dst, _ in jobs:
            if b64:
                with open(dst, "rb") as f:
                    out.append({"b64_json": base64.b64encode(f.read()).decode()})
                os.remove(dst)
            else:
                out.append({"url": f"{base_url}/generated-images/{os.path.basename(dst)}"})
        return {"id": str(uuid.uuid4()), "created": int(time.time()), "data": out,
                "usage": {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}}
    finally:
        if src:
            os.remove(src)


@router.post("/v1/audio/transcriptions")
async def transcription(request: Request):
    a = app_of(request)
    form = await read_form(request)
    up = form.get("file")
    if not hasattr(up, "read"):
        raise RequestError("file is required")
    model = form.get("model") or a.first_model_for(FLAG_TRANSCRIPT)
    cfg = a.configs.load_by_name(str(model))
    if not cfg.backend:
        cfg.backend = "whisper"
    d = tempfile.mkdtemp(prefix="whisper")
    try:
        dst = os.path.join(d, os.path.basename(up.filename or "audio"))
        with open(dst, "wb") as f:
            shutil.copyfileobj(up.file, f)
        r = await a.inference.transcribe(cfg, dst, str(form.get("language") or cfg.parameters.language or ""),
                                         bool(form.get("translate") or cfg.parameters.translate), cfg.threads or 0)
        return {"segments": [{"id": s.id, "start": s.start, "end": s.end, "text": s.text, "tokens": list(s.tokens)}
                             for s in r.segments], "text": r.text}
    finally:
        shutil.rmtree(d, ignore_errors=True)


async def run_tts(a, body: dict, model: str | None = None) -> str:
    name = model or body.get("model") or a.first_model_for(FLAG_TTS)
    if not name:
        raise RequestError("model is required")
    cfg = a.configs.load_by_name(name)
    if not cfg.backend:
        cfg.backend = body.get("backend") or "piper"
    voice = body.get("voice") or cfg.tts.voice
    lang = body.get("language") or ""
    audio_dir = os.path.join(a.cfg.generated_content_dir, "audio")
    os.makedirs(audio_dir, exist_ok=True)
    dst = os.path.join(audio_dir, f"tts_{uuid.uuid4().hex}.wav")
    await a.inference.tts(cfg, body.get("input") or body.get("text") or "", voice, dst, lang)
    fmt = body.get("response_format") or ""
    return audio_convert(dst, fmt)


def audio_convert(path: str, fmt: str) -> str:
    """utils.AudioConvert: wav passthrough; other formats need ffmpeg (not bundled here)."""
    if not fmt or fmt == "wav":
        return path
    ff = shutil.which("ffmpeg")
    if ff is None:
        return path
    import subprocess
    out = os.path.splitext(path)[0] + "." + fmt
    subprocess.run([ff, "-y", "-i", path, out], check=True, capture_output=True)
    return out


@router.post("/tts")
@router.post("/v1/audio/speech")
async def tts(request: Request):
    a = app_of(request)
    body = await request.json()
    path = await run_tts(a, body)
    return FileResponse(path, filename=os.path.basename(path))


@router.post("/video")
async def video(request: Request):
    a = app_of(request)
    body = await request.json()
    name = body.get("model") or a.first_model_for(FLAG_VIDEO)
    cfg = a.configs.load_by_name(name)
    vdir = os.path.join(a.cfg.generated_content_dir, "videos")
    os.makedirs(vdir, exist_ok=True)
    dst = os.path.join(vdir, f"video_{uuid.uuid4().hex}.mp4")
    srcs = []
    try:
        kw = dict(prompt=body.get("prompt", ""), width=int(body.get("width") or 512),
                  height=int(body.get("height") or 512), num_frames=int(body.get("num_frames") or 16),
                  fps=int(body.get("fps") or 8), seed=int(body.get("seed") or 0),
                  cfg_scale=float(body.get("cfg_scale") or 0.0), dst=dst)
        for k in ("start_image", "end_image"):
            if body.get(k):
                p = _materialize(a, body[k])
                srcs.append(p)
                kw[k] = p
        await a.inference.video(cfg, **kw)
    finally:
        for p in srcs:
            os.remove(p)
    base_url = str(request.base_url).rstrip("/")
    if body.get("response_format") == "b64_json":
        with open(dst, "rb") as f:
            return JSONResponse({"data": [{"b64_json": base64.b64encode(f.read()).decode()}]})
    return {"id": str(uuid.uuid4()), "created": int(time.time()),
            "data": [{"url": f"{base_url}/generated-videos/{os.path.basename(dst)}"}]}
