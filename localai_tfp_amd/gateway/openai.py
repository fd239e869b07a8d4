"""OpenAI-compatible endpoints: chat, completions, edits, embeddings, models.

Behavioural parity: core/http/endpoints/openai/chat.go:30-490 (SSE chunks, tool calls,
handleQuestion), completion.go:30-208, edit.go:26, embeddings.go:24, list.go:15,
inference.go:11-65 (ComputeChoices), routes/openai.go:12-118.

SSE framing is the reference's: `data: <json>\\n\\n` per chunk, a final chunk carrying the
finish_reason and usage, then `data: [DONE]\\n\\n`."""
from __future__ import annotations

import json
import logging
import time
import uuid

from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse, Response

from .. import functions as F
from ..config.model_config import FLAG_CHAT, FLAG_COMPLETION, FLAG_EDIT, FLAG_EMBEDDINGS
from ..templates.evaluator import COMPLETION, EDIT
from .observability import StreamTimer
from .inference import LLMResponse, TokenUsage, finetune
from .request import OpenAIRequest, RequestError, merge_request

log = logging.getLogger("localai_tfp_amd.gateway.openai")
router = APIRouter()

_dumps = json.JSONEncoder(ensure_ascii=False, separators=(",", ":")).encode


def sse(obj) -> bytes:
    return b"data: " + _dumps(obj).encode() + b"\n\n"


SSE_DONE = b"data: [DONE]\n\n"
SSE_HEADERS = {"Cache-Control": "no-cache", "Connection": "keep-alive", "X-Accel-Buffering": "no"}


def app_of(request: Request):
    return request.app.state.localai


async def parse(request: Request, flag: int) -> tuple[OpenAIRequest, object]:
    """SetModelAndConfig + SetOpenAIRequest: body, model name fallbacks, config, merge."""
    a = app_of(request)
    try:
        body = await request.json()
    except ValueError:
        raise RequestError("failed parsing request body")
    if not isinstance(body, dict):
        raise RequestError("request body must be a JSON object")
    req = OpenAIRequest(body)
    name = req.model or request.path_params.get("model") or request.query_params.get("model") or ""
    if not name:
        auth = request.headers.get("authorization", "")
        bearer = auth[7:] if auth.lower().startswith("bearer ") else ""
        if bearer and a.model_exists(bearer):
            name = bearer
    if not name:
        name = a.first_model_for(flag)
    if not name:
        raise RequestError("no model specified and no model available for this use case")
    req.model = req.model or name
    cfg = a.configs.load_by_name(name)
    if not cfg.parameters.model:
        cfg.parameters.model = name
    req.correlation_id = request.headers.get("x-correlation-id") or str(uuid.uuid4())
    merge_request(cfg, req)
    return req, cfg


def _media(req: OpenAIRequest):
    imgs, vids, auds = [], [], []
    for m in req.messages:
        imgs += m.get("string_images", []) or []
        vids += m.get("string_videos", []) or []
        auds += m.get("string_audios", []) or []
    return imgs, vids, auds


async def compute_choices(a, req: OpenAIRequest, prompt: str, cfg, cb, on_token=None):
    """ComputeChoices: n predictions, usage summed, Finetune applied, `cb(text, choices)`."""
    n = req.n or 1
    choices: list = []
    usage = TokenUsage()
    imgs, vids, auds = _media(req)
    for _ in range(n):
        r: LLMResponse = await a.inference.predict(cfg, prompt, req.messages, imgs, vids, auds, on_token,
                                                   req.correlation_id)
        usage.add(r.usage)
        cb(finetune(cfg, prompt, r.response), choices)
    return choices, usage


# ------------------------------------------------------------------------------------------------
# chat

def _grammar_for_response_format(cfg):
    rf = cfg.response_format_map
    if not rf:
        return
    t = rf.get("type")
    if t == "json_object":
        cfg.grammar = F.JSON_BNF
    elif t == "json_schema":
        js = (rf.get("json_schema") or {}).get("schema") or {}
        try:
            cfg.grammar = F.schema_to_grammar({"anyOf": [js]}, F.grammar_options(cfg.function))
        except Exception as ex:
            log.warning("json_schema grammar failed: %s", ex)


@router.post("/v1/chat/completions")
@router.post("/chat/completions")
@router.post("/v1/engines/{model}/chat/completions")
async def chat(request: Request):
    a = app_of(request)
    req, cfg = await parse(request, FLAG_CHAT)
    cid = req.correlation_id
    created = int(time.time())
    extra_usage = bool(request.headers.get("extra-usage"))
    funcs = list(req.functions)
    should_use_fn = bool(funcs) and cfg.should_use_functions()
    strict = any(f.strict for f in funcs)
    no_action = cfg.function.no_action_function_name or "answer"
    no_action_desc = cfg.function.no_action_description_name or "use this action to answer without performing any action"
    _grammar_for_response_format(cfg)
    if (not cfg.function.grammar.no_grammar or strict) and should_use_fn:
        if not cfg.function.disable_no_action:
            funcs.append(F.Function(no_action, no_action_desc, False, {"properties": {"message": {
                "type": "string", "description": "The message to reply the user with"}}}))
        if cfg.function_to_call():
            funcs = F.select(funcs, cfg.function_to_call()) or funcs
        try:
            js = F.to_json_structure(funcs, cfg.function.function_name_key, cfg.function.function_name_key)
            cfg.grammar = F.schema_to_grammar(js, F.grammar_options(cfg.function))
        except Exception as ex:
            log.warning("tool grammar generation failed: %s", ex)
    elif req.grammar_json_functions:
        try:
            cfg.grammar = F.schema_to_grammar(req.grammar_json_functions, F.grammar_options(cfg.function))
        except Exception as ex:
            log.warning("grammar_json_functions failed: %s", ex)
    elif cfg.function_to_call():
        funcs = F.select(funcs, cfg.function_to_call()) or funcs

    prompt = ""
    if not cfg.template.use_tokenizer_template or should_use_fn:
        prompt = a.evaluator.template_messages(req.messages, cfg, funcs, should_use_fn)

    base = {"id": cid, "created": created, "model": req.model}

    if req.stream:
        include_usage = bool(req.stream_options.get("include_usage"))
        if not should_use_fn:
            return SSEResponse(_chat_stream(a, req, cfg, prompt, base, extra_usage, include_usage),
                               {"X-Correlation-ID": cid})
        return SSEResponse(_chat_stream_tools(a, req, cfg, prompt, base, no_action, extra_usage),
                           {"X-Correlation-ID": cid})

    text_to_return = [""]

    def cb(s: str, choices: list):
        if not should_use_fn:
            choices.append({"index": 0, "finish_reason": "stop",
                            "message": {"role": "assistant", "content": s}})
            return
        text_to_return[0] = F.parse_text_content(s, cfg.function)
        s2 = F.cleanup_llm_result(s, cfg.function)
        results = F.parse_function_call(s2, cfg.function)
        no_actions = (len(results) > 0 and results[0].name == no_action) or not results
        finish = "tool_calls" if req.tools else "stop"
        if no_actions:
            choices.append({"index": 0, "finish_reason": finish, "_question": (results, s2)})
            return
        if req.tools:
            choices.append({"index": 0, "finish_reason": finish, "message": {
                "role": "assistant", "content": text_to_return[0],
                "tool_calls": [{"index": i, "id": cid, "type": "function",
                                "function": {"name": r.name, "arguments": r.arguments}}
                               for i, r in enumerate(results)]}})
        else:
            for r in results:
                choices.append({"index": 0, "finish_reason": "function_call", "message": {
                    "role": "assistant", "content": text_to_return[0],
                    "function_call": {"name": r.name, "arguments": r.arguments}}})

    choices, usage = await compute_choices(a, req, prompt, cfg, cb)
    for ch in choices:
        q = ch.pop("_question", None)
        if q is not None:
            ans = await handle_question(a, cfg, req, q[0], q[1], prompt)
            ch["message"] = {"role": "assistant", "content": ans}
    return JSONResponse({**base, "object": "chat.completion", "choices": choices,
                         "usage": usage.openai(extra_usage)}, headers={"X-Correlation-ID": cid})


class SSEResponse(Response):
    """Raw ASGI text/event-stream response: one `send` per chunk, client disconnect cancels the
    producer (frees the backend sequence through the gRPC cancel). Starlette's StreamingResponse
    adds an anyio task group + checkpoints per chunk, which showed up in the gateway profile."""

    def __init__(self, gen, headers: dict | None = None):  # noqa: super().__init__ deliberately skipped
        self.gen = gen
        self.background = None
        self.status_code = 200
        self.raw_headers = [(b"content-type", b"text/event-stream"), (b"cache-control", b"no-cache"),
                        (b"connection", b"keep-alive"), (b"x-accel-buffering", b"no")]
        for k, v in (headers or {}).items():
            if k.lower() not in ("cache-control", "connection", "x-accel-buffering"):
                self.raw_headers.append((k.lower().encode(), str(v).encode()))

    async def __call__(self, scope, receive, send):
        import asyncio
        me = asyncio.current_task()
        gone = [False]

        async def watch():
            while True:
                msg = await receive()
                if msg["type"] == "http.disconnect":
                    gone[0] = True
                    me.cancel()
                    return
        watcher = asyncio.ensure_future(watch())
        try:
            await send({"type": "http.response.start", "status": 200, "headers": self.raw_headers})
            async for chunk in self.gen:
                await send({"type": "http.response.body", "body": chunk, "more_body": True})
            await send({"type": "http.response.body", "body": b"", "more_body": False})
        except asyncio.CancelledError:
            if not gone[0]:
                raise
        finally:
            watcher.cancel()
            await self.gen.aclose()


class _ChunkFmt:
    """Pre-serialised chat.completion.chunk envelope: per token only the content string (and the
    usage object when it changes) is JSON-encoded."""

    def __init__(self, base: dict, obj: str, extra_usage: bool):
        head = _dumps({**base, "object": obj})[:-1]
        self.pre = ("data: " + head + ',"choices":[{"index":0,"finish_reason":null,"delta":{"content":').encode()
        self.extra = extra_usage
        self._u = None
        self._ub = b""

    def usage(self, u: TokenUsage) -> bytes:
        key = (u.prompt, u.completion, u.timing_prompt_processing, u.timing_token_generation)
        if key != self._u:
            self._u = key
            self._ub = _dumps(u.openai(self.extra)).encode()
        return self._ub

    def content(self, text: str, u: TokenUsage) -> bytes:
        return self.pre + _dumps(text).encode() + b'}}],"usage":' + self.usage(u) + b"}\n\n"


async def _chat_stream(a, req, cfg, prompt, base, extra_usage, include_usage):
    fmt = _ChunkFmt(base, "chat.completion.chunk", extra_usage)
    usage = TokenUsage()
    yield sse({**base, "object": "chat.completion.chunk",
               "choices": [{"index": 0, "finish_reason": None, "delta": {"role": "assistant", "content": ""}}]})
    imgs, vids, auds = _media(req)
    timer = StreamTimer(getattr(cfg, "name", "") or req.model)
    ok = True
    try:
        for _ in range(req.n or 1):
            seen = 0
            async for text, u in a.inference.predict_stream(cfg, prompt, req.messages, imgs, vids, auds,
                                                            req.correlation_id):
                usage = u
                timer.chunk(max(1, u.completion - seen) if u.completion else 1)
                seen = u.completion or seen
                yield fmt.content(text, u)
    except Exception as ex:  # surface as an error event, then terminate the stream cleanly
        ok = False
        log.error("chat stream failed: %s", ex)
        yield sse({"error": {"message": str(ex), "type": "server_error"}})
    finally:
        timer.close(ok)
    yield sse({**base, "object": "chat.completion.chunk",
               "choices": [{"index": 0, "finish_reason": "stop", "delta": {"content": ""}}],
               "usage": usage.openai(extra_usage)})
    if include_usage:
        yield sse({**base, "object": "chat.completion.chunk", "choices": [], "usage": usage.openai(extra_usage)})
    yield SSE_DONE


async def _chat_stream_tools(a, req, cfg, prompt, base, no_action, extra_usage):
    """processTools: generate fully (grammar-constrained), then emit tool-call deltas."""
    result_parts = []

    def on_token(s, _u):
        result_parts.append(s)
    _, usage = await compute_choices(a, req, prompt, cfg, lambda s, c: None, on_token)
    result = "".join(result_parts)
    text = F.parse_text_content(result, cfg.function)
    result = F.cleanup_llm_result(result, cfg.function)
    results = F.parse_function_call(result, cfg.function)
    no_action_run = (len(results) > 0 and results[0].name == no_action) or not results
    tools_called = False
    if no_action_run:
        yield sse({**base, "object": "chat.completion.chunk",
                   "choices": [{"index": 0, "finish_reason": None, "delta": {"role": "assistant", "content": text}}]})
        ans = await handle_question(a, cfg, req, results, result, prompt)
        yield sse({**base, "object": "chat.completion.chunk",
                   "choices": [{"index": 0, "finish_reason": None, "delta": {"content": ans}}],
                   "usage": usage.openai(extra_usage)})
    else:
        tools_called = True
        for i, r in enumerate(results):
            yield sse({**base, "object": "chat.completion.chunk", "choices": [{"index": 0, "finish_reason": None,
                       "delta": {"role": "assistant", "tool_calls": [{"index": i, "id": base["id"], "type": "function",
                                                                      "function": {"name": r.name, "arguments": ""}}]}}]})
            yield sse({**base, "object": "chat.completion.chunk", "choices": [{"index": 0, "finish_reason": None,
                       "delta": {"role": "assistant", "content": text,
                                 "tool_calls": [{"index": i, "id": base["id"], "type": "function",
                                                 "function": {"arguments": r.arguments}}]}}]})
    finish = ("tool_calls" if req.tools else "function_call") if tools_called else "stop"
    yield sse({**base, "object": "chat.completion.chunk",
               "choices": [{"index": 0, "finish_reason": finish, "delta": {"content": text}}],
               "usage": usage.openai(extra_usage)})
    yield SSE_DONE


async def handle_question(a, cfg, req, results, result: str, prompt: str) -> str:
    """handleQuestion: reuse the no-action `message` argument, else re-ask without a grammar."""
    if not results and result:
        return result
    arg = results[0].arguments if results else ""
    try:
        args = json.loads(arg) if arg else {}
    except ValueError:
        args = {}
    msg = args.get("message") if isinstance(args, dict) else None
    if isinstance(msg, str) and msg:
        return finetune(cfg, prompt, msg)
    cfg.grammar = ""
    imgs, vids, auds = _media(req)
    r = await a.inference.predict(cfg, prompt, req.messages, imgs, vids, auds, None, req.correlation_id)
    return finetune(cfg, prompt, r.response)


# ------------------------------------------------------------------------------------------------
# completions / edits

@router.post("/v1/completions")
@router.post("/completions")
@router.post("/v1/engines/{model}/completions")
async def completion(request: Request):
    a = app_of(request)
    req, cfg = await parse(request, FLAG_COMPLETION)
    cid = req.correlation_id
    created = int(time.time())
    extra_usage = bool(request.headers.get("extra-usage"))
    _grammar_for_response_format(cfg)
    base = {"id": cid, "created": created, "model": req.model}
    prompts = cfg.prompt_strings or [""]
    tmpl = lambda p: a.evaluator.evaluate_for_prompt(COMPLETION, cfg, {  # noqa: E731
        "Input": p, "SystemPrompt": cfg.system_prompt})
    if req.stream:
        if len(prompts) > 1:
            raise RequestError("cannot handle more than 1 `PromptStrings` when Streaming")
        prompt = tmpl(prompts[0])
        return SSEResponse(_completion_stream(a, req, cfg, prompt, base, extra_usage), {"X-Correlation-ID": cid})
    all_choices = []
    total = TokenUsage()
    for k, p in enumerate(prompts):
        prompt = tmpl(p)

        def cb(s, choices, k=k):
            choices.append({"index": k, "finish_reason": "stop", "text": s})
        ch, u = await compute_choices(a, req, prompt, cfg, cb)
        total.add(u)
        all_choices += ch
    return JSONResponse({**base, "object": "text_completion", "choices": all_choices,
                         "usage": total.openai(extra_usage)}, headers={"X-Correlation-ID": cid})


async def _completion_stream(a, req, cfg, prompt, base, extra_usage):
    head = _dumps({**base, "object": "text_completion"})[:-1]
    pre = ("data: " + head + ',"choices":[{"index":0,"finish_reason":null,"text":').encode()
    fmt = _ChunkFmt(base, "text_completion", extra_usage)
    usage = TokenUsage()
    timer = StreamTimer(getattr(cfg, "name", "") or req.model)
    ok = True
    try:
        seen = 0
        async for text, u in a.inference.predict_stream(cfg, prompt, req.messages, (), (), (), req.correlation_id):
            usage = u
            timer.chunk(max(1, u.completion - seen) if u.completion else 1)
            seen = u.completion or seen
            yield pre + _dumps(text).encode() + b'}],"usage":' + fmt.usage(u) + b"}\n\n"
    except Exception as ex:
        ok = False
        log.error("completion stream failed: %s", ex)
        yield sse({"error": {"message": str(ex), "type": "server_error"}})
    finally:
        timer.close(ok)
    yield sse({**base, "object": "text_completion", "choices": [{"index": 0, "finish_reason": "stop"}],
               "usage": usage.openai(extra_usage)})
    yield SSE_DONE


@router.post("/v1/edits")
@router.post("/edits")
async def edit(request: Request):
    a = app_of(request)
    req, cfg = await parse(request, FLAG_EDIT)
    created = int(time.time())
    choices_all = []
    total = TokenUsage()
    for i in cfg.input_strings or [""]:
        prompt = a.evaluator.evaluate_for_prompt(EDIT, cfg, {"Input": i, "Instruction": req.instruction,
                                                             "SystemPrompt": cfg.system_prompt})
        ch, u = await compute_choices(a, req, prompt, cfg, lambda s, c: c.append({"index": 0, "text": s,
                                                                                  "finish_reason": "stop"}))
        total.add(u)
        choices_all += ch
    return {"id": req.correlation_id, "created": created, "model": req.model, "object": "edit",
            "choices": choices_all, "usage": total.openai()}


# ------------------------------------------------------------------------------------------------
# embeddings / models

@router.post("/v1/embeddings")
@router.post("/embeddings")
@router.post("/v1/engines/{model}/embeddings")
async def embeddings(request: Request):
    a = app_of(request)
    req, cfg = await parse(request, FLAG_EMBEDDINGS)
    data = []
    i = 0
    for toks in cfg.input_tokens:
        data.append({"embedding": await a.inference.embeddings(cfg, tokens=toks), "index": i, "object": "embedding"})
        i += 1
    for s in cfg.input_strings:
        data.append({"embedding": await a.inference.embeddings(cfg, text=s), "index": i, "object": "embedding"})
        i += 1
    return {"object": "list", "model": req.model, "data": data, "created": int(time.time()),
            "id": req.correlation_id, "usage": {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}}


@router.get("/v1/models")
@router.get("/models")
async def list_models(request: Request):
    from .state import ALWAYS_INCLUDE, SKIP_IF_CONFIGURED
    a = app_of(request)
    exclude_configured = request.query_params.get("excludeConfigured", "true").lower() != "false"
    policy = SKIP_IF_CONFIGURED if exclude_configured else ALWAYS_INCLUDE
    flt = request.query_params.get("filter", "")
    names = a.list_models(policy=policy)
    if flt:
        import re
        rx = re.compile(flt)
        names = [n for n in names if rx.search(n)]
    return {"object": "list", "data": [{"id": n, "object": "model"} for n in names]}
