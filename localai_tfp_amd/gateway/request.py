"""Per-request model resolution and OpenAI-request -> model-config merge (behavioural parity:
core/http/middleware/request.go:28-442 — setModelNameFromRequest, SetModelAndConfig,
SetOpenAIRequest, mergeOpenAIRequestAndBackendConfig; multimodal placeholders
pkg/templates/multimodal.go:24-66; content fetch pkg/utils/base64.go:17)."""
from __future__ import annotations

import base64
import json
import logging
import re
import urllib.request

from ..functions import Function, functions_from_request
from ..templates import gotemplate

log = logging.getLogger("localai_tfp_amd.gateway")

DEFAULT_MULTIMODAL = ("{{ range .Audio }}[audio-{{.ID}}]{{end}}{{ range .Images }}[img-{{.ID}}]{{end}}"
                      "{{ range .Video }}[vid-{{.ID}}]{{end}}{{.Text}}")
_DATA_URI = re.compile(r"^data:[^;]+;base64,")


class RequestError(ValueError):
    def __init__(self, msg: str, status: int = 400):
        super().__init__(msg)
        self.status = status


def content_as_base64(url: str) -> str:
    """GetContentURIAsBase64: data URIs are stripped to their payload, http(s) URLs fetched."""
    if url.startswith("data:"):
        return _DATA_URI.sub("", url)
    if url.startswith(("http://", "https://")):
        with urllib.request.urlopen(url, timeout=30) as r:
            return base64.b64encode(r.read()).decode()
    raise ValueError("unsupported content URL")


def template_multimodal(tpl: str, total_images: int, total_videos: int, total_audios: int,
                        n_img: int, n_vid: int, n_aud: int, text: str) -> str:
    """TemplateMultiModal: IDs continue across messages (image N of the conversation)."""
    data = {
        "Text": text,
        "Images": [{"ID": i} for i in range(total_images - n_img, total_images)],
        "Video": [{"ID": i} for i in range(total_videos - n_vid, total_videos)],
        "Audio": [{"ID": i} for i in range(total_audios - n_aud, total_audios)],
    }
    return gotemplate.render(tpl or DEFAULT_MULTIMODAL, data)


class OpenAIRequest:
    """Parsed JSON body; unknown keys are kept in `.raw`."""

    def __init__(self, body: dict):
        self.raw = body
        g = body.get
        self.model: str = g("model") or ""
        self.stream: bool = bool(g("stream", False))
        self.messages: list[dict] = [dict(m) for m in (g("messages") or [])]
        self.functions: list[Function] = functions_from_request(g("functions"), g("tools"))
        self.tools: list = g("tools") or []
        self.tool_choice = g("tool_choice")
        self.function_call = g("function_call")
        self.n: int = int(g("n") or 0)
        self.prompt = g("prompt")
        self.input = g("input")
        self.instruction: str = g("instruction") or ""
        self.stop = g("stop")
        self.grammar: str = g("grammar") or ""
        self.grammar_json_functions = g("grammar_json_functions")
        self.response_format = g("response_format")
        self.size: str = g("size") or ""
        self.quality = g("quality") or ""
        self.step = int(g("step") or 0)
        self.mode = int(g("mode") or 0)
        self.file: str = g("file") or ""
        self.backend: str = g("backend") or ""
        self.stream_options = g("stream_options") or {}
        self.correlation_id = ""


def _set_if(d: dict, key: str, fn):
    v = d.get(key)
    if v is not None:
        fn(v)


def merge_request(cfg, req: OpenAIRequest):
    """mergeOpenAIRequestAndBackendConfig."""
    b = req.raw
    p = cfg.parameters
    if b.get("echo"):
        p.echo = True
    _set_if(b, "top_k", lambda v: setattr(p, "top_k", int(v)))
    _set_if(b, "top_p", lambda v: setattr(p, "top_p", float(v)))
    if req.backend:
        cfg.backend = req.backend
    if b.get("clip_skip"):
        cfg.diffusers.clip_skip = int(b["clip_skip"])
    if b.get("negative_prompt_scale"):
        p.negative_prompt_scale = float(b["negative_prompt_scale"])
    if b.get("negative_prompt"):
        p.negative_prompt = b["negative_prompt"]
    if b.get("rope_freq_base"):
        p.rope_freq_base = float(b["rope_freq_base"])
    if b.get("rope_freq_scale"):
        p.rope_freq_scale = float(b["rope_freq_scale"])
    if req.grammar:
        cfg.grammar = req.grammar
    _set_if(b, "temperature", lambda v: setattr(p, "temperature", float(v)))
    mt = b.get("max_tokens", b.get("max_completion_tokens"))
    if mt is not None:
        p.max_tokens = int(mt)
    rf = req.response_format
    if isinstance(rf, str):
        cfg.response_format = rf
    elif isinstance(rf, dict):
        cfg.response_format_map = rf
    stop = req.stop
    if isinstance(stop, str) and stop:
        cfg.stopwords = list(cfg.stopwords) + [stop]
    elif isinstance(stop, list):
        cfg.stopwords = list(cfg.stopwords) + [s for s in stop if isinstance(s, str)]
    if req.tool_choice is not None:
        tc = req.tool_choice
        if isinstance(tc, str):
            try:
                tc = json.loads(tc)
            except ValueError:
                tc = {}  # "auto" / "none" / "required"
        name = ((tc or {}).get("function") or {}).get("name", "") if isinstance(tc, dict) else ""
        req.function_call = {"name": name}
    # multimodal content -> text with placeholders + base64 media
    ni = nv = na = 0
    for m in req.messages:
        c = m.get("content")
        if isinstance(c, str):
            m["string_content"] = c
        elif isinstance(c, list):
            text = ""
            ci = cv = ca = 0
            imgs, vids, auds = [], [], []
            for part in c:
                if not isinstance(part, dict):
                    continue
                t = part.get("type", "")
                try:
                    if t == "text":
                        text += part.get("text", "")
                    elif t in ("image_url", "image"):
                        imgs.append(content_as_base64(_url(part, "image_url")))
                        ni += 1
                        ci += 1
                    elif t in ("video_url", "video"):
                        vids.append(content_as_base64(_url(part, "video_url")))
                        nv += 1
                        cv += 1
                    elif t in ("audio_url", "audio"):
                        auds.append(content_as_base64(_url(part, "audio_url")))
                        na += 1
                        ca += 1
                except Exception as ex:
                    log.error("failed encoding %s content: %s", t, ex)
            m["string_images"], m["string_videos"], m["string_audios"] = imgs, vids, auds
            m["string_content"] = template_multimodal(cfg.template.multimodal, ni, nv, na, ci, cv, ca, text)
        else:
            m["string_content"] = ""
    if b.get("repeat_penalty"):
        p.repeat_penalty = float(b["repeat_penalty"])
    if b.get("frequency_penalty"):
        p.frequency_penalty = float(b["frequency_penalty"])
    if b.get("presence_penalty"):
        p.presence_penalty = float(b["presence_penalty"])
    if b.get("n_keep"):
        p.n_keep = int(b["n_keep"])
    if b.get("batch"):
        p.batch = int(b["batch"])
    if b.get("ignore_eos"):
        p.ignore_eos = True
    _set_if(b, "seed", lambda v: setattr(p, "seed", int(v)))
    _set_if(b, "typical_p", lambda v: setattr(p, "typical_p", float(v)))
    if b.get("repeat_last_n"):
        p.repeat_last_n = int(b["repeat_last_n"])
    if b.get("mirostat") is not None:
        cfg.mirostat = int(b["mirostat"])
    if b.get("mirostat_tau") is not None:
        cfg.mirostat_tau = float(b["mirostat_tau"])
    if b.get("mirostat_eta") is not None:
        cfg.mirostat_eta = float(b["mirostat_eta"])
    inp = req.input
    if isinstance(inp, str):
        if inp:
            cfg.input_strings = list(cfg.input_strings) + [inp]
    elif isinstance(inp, list):
        for it in inp:
            if isinstance(it, str):
                cfg.input_strings.append(it)
            elif isinstance(it, list):
                cfg.input_tokens.append([int(x) for x in it])
            elif isinstance(it, int):
                # a flat token list is a single tokenized input
                cfg.input_tokens.append([int(x) for x in inp])
                break
    fc = req.function_call
    if isinstance(fc, str) and fc:
        cfg.function_call_string = fc
    elif isinstance(fc, dict):
        cfg.function_call_name = fc.get("name", "") or ""
    pr = req.prompt
    if isinstance(pr, str):
        cfg.prompt_strings = list(cfg.prompt_strings) + [pr]
    elif isinstance(pr, list):
        cfg.prompt_strings = list(cfg.prompt_strings) + [s for s in pr if isinstance(s, str)]
    if req.quality:
        try:
            cfg.step = int(req.quality)
        except ValueError:
            pass
    if not cfg.validate():
        raise RequestError("unable to validate configuration after merging")
    return cfg


def _url(part: dict, key: str) -> str:
    v = part.get(key)
    if isinstance(v, dict):
        return v.get("url", "")
    if isinstance(v, str):
        return v
    return part.get("url", "")
