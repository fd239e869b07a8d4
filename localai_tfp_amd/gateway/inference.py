"""Gateway-side calls into backend workers (behavioural parity: core/backend/*.go —
llm.go ModelInference/Finetune, embeddings.go, image.go, tts.go, transcript.go, rerank.go,
soundgeneration.go, stores.go, token_metrics.go, tokenize.go, vad.go).

All calls are async over grpc.aio so the event loop never parks a thread per streaming request."""
from __future__ import annotations

import asyncio
import codecs
import re
from dataclasses import dataclass, field

from ..grpc import pb
from ..serving.options import predict_options

_re_cache: dict[str, re.Pattern] = {}


def _re(p: str) -> re.Pattern:
    r = _re_cache.get(p)
    if r is None:
        r = _re_cache[p] = re.compile(p)
    return r


@dataclass
class TokenUsage:
    prompt: int = 0
    completion: int = 0
    timing_prompt_processing: float = 0.0
    timing_token_generation: float = 0.0

    def add(self, o: "TokenUsage"):
        self.prompt += o.prompt
        self.completion += o.completion
        self.timing_prompt_processing += o.timing_prompt_processing
        self.timing_token_generation += o.timing_token_generation

    def openai(self, extra: bool = False) -> dict:
        d = {"prompt_tokens": self.prompt, "completion_tokens": self.completion,
             "total_tokens": self.prompt + self.completion}
        if extra:
            if self.timing_prompt_processing:
                d["timing_prompt_processing"] = self.timing_prompt_processing
            if self.timing_token_generation:
                d["timing_token_generation"] = self.timing_token_generation
        return d


@dataclass
class LLMResponse:
    response: str = ""
    usage: TokenUsage = field(default_factory=TokenUsage)


def finetune(cfg, prompt: str, prediction: str) -> str:
    """backend.Finetune: echo, cutstrings, extract_regex, trimspace, trimsuffix."""
    if cfg.parameters.echo:
        prediction = prompt + prediction
    for c in cfg.cutstrings:
        prediction = _re(c).sub("", prediction)
    got = ""
    for r in cfg.extract_regex:
        m = _re(r).search(prediction)
        if m:
            got += m.group(0)
    if got:
        prediction = got
    for c in cfg.trimspace:
        prediction = prediction.removeprefix(c).strip()
    for c in cfg.trimsuffix:
        prediction = prediction.removesuffix(c).strip()
    return prediction


def _message_text(m: dict) -> str:
    c = m.get("content")
    if isinstance(c, str):
        return c
    if isinstance(c, list):
        return "".join(p.get("text", "") for p in c if isinstance(p, dict))
    return m.get("string_content", "") or ""


class Inference:
    """Bound to the gateway Application (loader + model path)."""

    def __init__(self, app):
        self.app = app

    async def model(self, cfg):
        loop = asyncio.get_running_loop()
        m = self.app.loader.get(cfg.name or cfg.parameters.model)
        if m is None:
            m = await loop.run_in_executor(None, self.app.loader.load, cfg)
        return m

    def _predict_opts(self, cfg, prompt: str, messages=None, images=(), videos=(), audios=()):
        o = predict_options(cfg, self.app.cfg.models_path)
        o.Prompt = prompt
        if cfg.template.use_tokenizer_template and not prompt and messages:
            for m in messages:
                o.Messages.append(pb.Message(role=m.get("role", ""), content=_message_text(m)))
        o.UseTokenizerTemplate = bool(cfg.template.use_tokenizer_template)
        o.Images.extend(images)
        o.Videos.extend(videos)
        o.Audios.extend(audios)
        return o

    async def predict(self, cfg, prompt: str, messages=None, images=(), videos=(), audios=(),
                      on_token=None, correlation_id: str = "") -> LLMResponse:
        """ModelInference: streaming when `on_token` is given (UTF-8 safe, rune by rune in the
        reference; here per decoded chunk with an incremental decoder), else unary Predict."""
        m = await self.model(cfg)
        opts = self._predict_opts(cfg, prompt, messages, images, videos, audios)
        opts.CorrelationId = correlation_id
        usage = TokenUsage()
        prefix = cfg.template.reply_prefix
        client = m.apick()
        if on_token is not None:
            if prefix:
                await _maybe_await(on_token(prefix, usage))
            dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
            parts = []
            async for r in client.stream("PredictStream", opts):
                text = dec.decode(r.message)
                if r.tokens or r.prompt_tokens:
                    usage.prompt = r.prompt_tokens
                    usage.completion = r.tokens
                    usage.timing_prompt_processing = r.timing_prompt_processing
                    usage.timing_token_generation = r.timing_token_generation
                if text:
                    parts.append(text)
                    await _maybe_await(on_token(text, usage))
            tail = dec.decode(b"", final=True)
            if tail:
                parts.append(tail)
                await _maybe_await(on_token(tail, usage))
            return LLMResponse("".join(parts), usage)
        r = await client.call("Predict", opts)
        usage = TokenUsage(r.prompt_tokens, r.tokens, r.timing_prompt_processing, r.timing_token_generation)
        text = r.message.decode("utf-8", errors="replace")
        return LLMResponse(prefix + text if prefix else text, usage)

    async def predict_stream(self, cfg, prompt: str, messages=None, images=(), videos=(), audios=(),
                             correlation_id: str = ""):
        """Async generator of (text, usage) pieces straight off the gRPC stream (no queue hop);
        `usage` is the same mutable TokenUsage updated as counts arrive."""
        m = await self.model(cfg)
        opts = self._predict_opts(cfg, prompt, messages, images, videos, audios)
        opts.CorrelationId = correlation_id
        usage = TokenUsage()
        if cfg.template.reply_prefix:
            yield cfg.template.reply_prefix, usage
        dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
        rep = m.pick_replica()
        mx = rep.mxclient()
        if mx is not None:  # batched token channel to our own workers (serving/mxstream.py)
            from ..serving.mxstream import F_ERROR
            async for flags, tok, ptok, tp, tg, data in mx.stream(opts):
                if flags & F_ERROR:
                    raise RuntimeError(data.decode("utf-8", "replace"))
                if tok or ptok:
                    usage.prompt, usage.completion = ptok, tok
                    usage.timing_prompt_processing, usage.timing_token_generation = tp, tg
                text = dec.decode(data) if data else ""
                if text:
                    yield text, usage
            tail = dec.decode(b"", final=True)
            if tail:
                yield tail, usage
            return
        async for r in rep.aclient().stream("PredictStream", opts):
            if r.tokens or r.prompt_tokens:
                usage.prompt, usage.completion = r.prompt_tokens, r.tokens
                usage.timing_prompt_processing = r.timing_prompt_processing
                usage.timing_token_generation = r.timing_token_generation
            text = dec.decode(r.message) if r.message else ""
            if text:
                yield text, usage
        tail = dec.decode(b"", final=True)
        if tail:
            yield tail, usage

    async def embeddings(self, cfg, text: str | None = None, tokens: list | None = None) -> list[float]:
        m = await self.model(cfg)
        o = predict_options(cfg, self.app.cfg.models_path)
        if tokens:
            o.EmbeddingTokens.extend(int(t) for t in tokens)
        else:
            o.Embeddings = text or ""
        r = await m.apick().call("Embedding", o)
        return list(r.embeddings)

    async def tokenize(self, cfg, text: str) -> list[int]:
        m = await self.model(cfg)
        o = predict_options(cfg, self.app.cfg.models_path)
        o.Prompt = text
        r = await m.apick().call("TokenizeString", o)
        return list(r.tokens)

    async def rerank(self, cfg, query: str, documents: list[str], top_n: int):
        m = await self.model(cfg)
        return await m.apick().call("Rerank", pb.RerankRequest(query=query, documents=documents, top_n=top_n))

    async def image(self, cfg, **kw):
        m = await self.model(cfg)
        r = await m.apick().call("GenerateImage", pb.GenerateImageRequest(**kw))
        if not r.success:
            raise RuntimeError(r.message or "image generation failed")
        return r

    async def video(self, cfg, **kw):
        m = await self.model(cfg)
        r = await m.apick().call("GenerateVideo", pb.GenerateVideoRequest(**kw))
        if not r.success:
            raise RuntimeError(r.message or "video generation failed")
        return r

    async def tts(self, cfg, text: str, voice: str, dst: str, language: str = ""):
        m = await self.model(cfg)
        req = pb.TTSRequest(text=text, model=cfg.parameters.model, dst=dst, voice=voice)
        if language:
            req.language = language
        r = await m.apick().call("TTS", req)
        if not r.success:
            raise RuntimeError(r.message or "tts failed")
        return r

    async def sound(self, cfg, **kw):
        m = await self.model(cfg)
        r = await m.apick().call("SoundGeneration", pb.SoundGenerationRequest(**kw))
        if not r.success:
            raise RuntimeError(r.message or "sound generation failed")
        return r

    async def transcribe(self, cfg, path: str, language: str = "", translate: bool = False, threads: int = 0):
        m = await self.model(cfg)
        return await m.apick().call("AudioTranscription", pb.TranscriptRequest(
            dst=path, language=language, translate=translate, threads=threads))

    async def vad(self, cfg, audio: list[float]):
        m = await self.model(cfg)
        return await m.apick().call("VAD", pb.VADRequest(audio=audio))

    async def metrics(self, cfg):
        m = await self.model(cfg)
        return await m.apick().call("GetMetrics", pb.MetricsRequest())

    async def rpc(self, cfg, name: str, req):
        m = await self.model(cfg)
        return await m.apick().call(name, req)


async def _maybe_await(x):
    if asyncio.iscoroutine(x):
        return await x
    return x
