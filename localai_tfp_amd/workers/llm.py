"""LLM worker: the backend.Backend gRPC service over :class:`engine.LLMEngine`.

Behavioural parity target: the reference's llama.cpp gRPC server
(backend/cpp/llama/grpc-server.cpp):
  * LoadModel  - ModelOptions -> engine/model settings (params_parse :2324-2455, LoadModel :2467-2487)
  * Predict / PredictStream - PredictOptions -> sampling request (parse_options :2164-2229), replies
    carrying message / tokens / prompt_tokens / timings (:2488-2576)
  * Embedding  - final-token pooled, L2-normalised hidden state (:2579-2601, send_embedding :1357-1414)
  * TokenizeString (:2603-2613), GetMetrics (:2615-2638); Status (not implemented there) reports
    engine state + HBM use here.

Differences by design: the engine is a paged-KV continuous-batching scheduler with hipGraph decode
(no per-slot context split, no `n_parallel`), `Messages` + `UseTokenizerTemplate` are honoured
(the reference ignores them), grammars are enforced by the native GBNF matcher
(csrc/runtime/grammar.cpp) with optional lazy trigger words (ModelOptions.GrammarTriggers).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time

import grpc

from ..engine.engine import EngineConfig, LLMEngine
from ..engine.sequence import Request
from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main
from ..ops.sampling import SamplingParams

log = logging.getLogger("localai_tfp_amd.workers.llm")


def parse_options(opts) -> dict:
    """ModelOptions.Options: ["key:value", "flag", ...] -> dict (grpc-server.cpp:2403-2430)."""
    out = {}
    for o in opts:
        k, _, v = o.partition(":")
        out[k.strip()] = v.strip() if v else True
    return out


def sampling_from_predict(r) -> SamplingParams:
    p = SamplingParams()
    p.temperature = float(r.Temperature)
    p.top_k = int(r.TopK) if r.TopK > 0 else 0
    p.top_p = float(r.TopP) if 0 < r.TopP <= 1 else 1.0
    p.typical_p = float(r.TypicalP) if 0 < r.TypicalP < 1 else 1.0
    p.min_p = 0.0
    p.repeat_penalty = float(r.Penalty) if r.Penalty > 0 else 1.0
    p.repeat_last_n = int(r.Repeat) if r.Repeat != 0 else 64
    p.presence_penalty = float(r.PresencePenalty)
    p.frequency_penalty = float(r.FrequencyPenalty)
    p.mirostat = int(r.Mirostat)
    if r.MirostatTAU:
        p.mirostat_tau = float(r.MirostatTAU)
    if r.MirostatETA:
        p.mirostat_eta = float(r.MirostatETA)
    p.seed = int(r.Seed) if r.Seed not in (0, -1) else -1
    p.ignore_eos = bool(r.IgnoreEOS)
    if r.LogitBias:
        try:
            lb = json.loads(r.LogitBias)
            p.logit_bias = {int(k): float(v) for k, v in lb.items()}
        except (ValueError, AttributeError):
            log.warning("ignoring malformed LogitBias %r", r.LogitBias[:80])
    return p


class LazyGrammar:
    """Grammar enforced only after a trigger word shows up in the output (lazy grammars,
    grpc-server.cpp:2437-2451). Before the trigger every token is allowed."""

    def __init__(self, make_matcher, triggers: list[str], token_bytes):
        self.make, self.triggers, self.tb = make_matcher, triggers, token_bytes
        self.m = None
        self.buf = b""
        self._dead = False

    def allowed_mask(self, V):
        if self.m is None:
            import numpy as np
            return np.full((V + 31) // 32, 0xFFFFFFFF, np.uint32)
        return self.m.allowed_mask(V)

    def accept(self, t: int) -> bool:
        if self.m is not None:
            return self.m.accept(t)
        self.buf += self.tb[t] if t < len(self.tb) else b""
        for w in self.triggers:
            i = self.buf.find(w.encode())
            if i >= 0:
                self.m = self.make()
                self._dead = not self.m.accept_bytes(self.buf[i:])
                return True
        return True

    def is_done(self) -> bool:
        return self.m is not None and (self._dead or self.m.is_done())


class _LoopChannel:
    def __init__(self, loop):
        self.loop = loop

    @staticmethod
    def _dispatch(items):
        for k, o in items:
            k.q.put_nowait(o)

    def deliver(self, items):
        self.loop.call_soon_threadsafe(self._dispatch, items)


class _QKey:
    __slots__ = ("channel", "q")

    def __init__(self, channel, q):
        self.channel, self.q = channel, q


def _is_musicgen(request) -> bool:
    if "musicgen" in (request.Type or "").lower():
        return True
    path = request.ModelFile or request.Model or ""
    if path.startswith("synthetic:musicgen"):
        return True
    if path and not os.path.isabs(path) and request.ModelPath:
        path = os.path.join(request.ModelPath, path)
    cfg = os.path.join(path, "config.json")
    if os.path.isfile(cfg):
        try:
            with open(cfg) as f:
                return json.load(f).get("model_type") == "musicgen"
        except (OSError, ValueError):
            return False
    return False


class LLMServicer(BackendServicer):
    def __init__(self, device: str | None = None, tp=None):
        super().__init__()
        self.tp = tp  # parallel.tp_engine.TPLink on the leader rank of a tensor-parallel worker
        self.engine: LLMEngine | None = None
        self.tok = None
        self.model_opts = None
        self.device = device
        self._vocab = None
        self._tb = None
        self._grammars: dict[str, object] = {}
        self._glock = threading.Lock()
        self.triggers: list[str] = []
        self._channels: dict = {}
        self.mxstream = None  # serving.mxstream.StreamServer once a model is loaded
        self.embeddings_enabled = False
        self.vision = None  # models.vision.ClipVision when ModelOptions.MMProj is set
        self.state = pb.STATE_UNINITIALIZED

    # ---------------------------------------------------------------- load
    def attach(self, engine: LLMEngine, tok):
        """Serve an engine built in-process (bench / embedding the worker in another program);
        subsequent LoadModel calls are acknowledged without reloading."""
        self.engine, self.tok = engine, tok
        self.preloaded = True
        self.state = pb.STATE_READY

    def _start_mxstream(self) -> str:
        """Batched token channel for this framework's gateway (serving/mxstream.py); the address
        is advertised in the LoadModel result as `mxstream=<path>`."""
        if os.environ.get("MX_STREAM", "1") == "0" or self.engine is None:
            return ""
        if self.mxstream is None:
            from ..serving.mxstream import StreamServer, socket_path_for
            addr = getattr(self, "bound_addr", "") or f"pid{os.getpid()}:0"
            try:
                self.mxstream = StreamServer(self, socket_path_for(addr))
            except OSError as ex:
                log.warning("mxstream disabled: %s", ex)
                return ""
        return self.mxstream.path

    def LoadModel(self, request, context):
        import torch
        from ..models.loader import load_llm
        if (request.Type or "").lower() == "outetts":
            # the transformers backend's OuteTTS type (backend/python/transformers/backend.py:205-243)
            from .outetts import OuteTTSServicer
            self._audio = OuteTTSServicer(self.device)
            return self._audio.LoadModel(request, context)
        if _is_musicgen(request):
            # the reference's transformers backend serves `type: MusicgenForConditionalGeneration` models
            # through SoundGeneration / TTS (backend/python/transformers/backend.py:452-507)
            from .musicgen import MusicgenServicer
            self._audio = MusicgenServicer(self.device)
            return self._audio.LoadModel(request, context)
        if getattr(self, "preloaded", False):
            mx = self._start_mxstream()
            return pb.Result(message="preloaded" + (f"; mxstream={mx}" if mx else ""), success=True)
        try:
            t0 = time.perf_counter()
            opts = parse_options(request.Options)
            path = request.ModelFile or request.Model
            if path and not path.startswith("synthetic:") and not os.path.isabs(path) and request.ModelPath:
                path = os.path.join(request.ModelPath, path)
            if self.device is None:
                if torch.cuda.is_available():
                    mg = request.MainGPU.strip()
                    self.device = f"cuda:{int(mg)}" if mg.isdigit() else "cuda:0"
                else:
                    self.device = "cpu"
            ov = {"rope_freq_base": request.RopeFreqBase, "rope_freq_scale": request.RopeFreqScale,
                  "rope_scaling": request.RopeScaling, "rms_norm_eps": request.RMSNormEps,
                  "lora": _lora_list(request, path), "lora_requant": opts.get("lora_requant", "runtime"),
                  # HF safetensors checkpoints (vllm / transformers backends): load-time block format
                  "hf_quant": opts.get("quant") or request.Quantization or "bf16"}
            ec = EngineConfig()
            if request.ContextSize > 0:
                ec.max_model_len = int(request.ContextSize)
            if request.NBatch > 0:
                ec.max_batched_tokens = max(int(request.NBatch), 64)
            par = int(os.environ.get("LLAMACPP_PARALLEL", "0") or 0) or int(opts.get("parallel", 0) or 0)
            if par > 0:
                ec.max_num_seqs = par
            if "gpu_memory_utilization" in opts or request.GPUMemoryUtilization > 0:
                ec.kv_mem_fraction = float(opts.get("gpu_memory_utilization", request.GPUMemoryUtilization))
            if opts.get("no_prefix_cache") or opts.get("cache_prompt") == "false":
                ec.enable_prefix_cache = False
            if request.EnforceEager or opts.get("enforce_eager"):
                ec.use_graphs = False
            ct = request.CacheTypeKey or request.CacheTypeValue or opts.get("kv_cache_dtype", "")
            if ct:  # one storage type for K and V (fp8 e4m3 for the 8-bit llama.cpp cache types)
                ec.kv_dtype = str(ct)
            if self.device == "cpu":
                ec.num_blocks = ec.num_blocks or 512
            if self.engine is not None:  # reload: stop the old engine (and the followers' replay)
                self.engine.shutdown()
                self.engine = None
            rpc = os.environ.get("LLAMACPP_GRPC_SERVERS", "") or str(opts.get("rpc_servers", ""))
            rpc_servers = [x.strip() for x in rpc.split(",") if x.strip()]
            if self.tp is not None:
                import dataclasses
                self.tp.send_control("load", (path, ov, dataclasses.asdict(ec)))
                with self.tp.quiet():  # followers load too: no heartbeats until they listen again
                    model, tok, mcfg, _ = load_llm(path, self.device, self.tp.rank, self.tp.world, None, ov)
            elif rpc_servers:
                # remote layer split (reference LLAMACPP_GRPC_SERVERS, grpc-server.cpp:139-161):
                # contiguous layer ranges on `local-ai worker llama-cpp-rpc` stages, tensor_split weights
                import re
                from ..parallel.pp_rpc import load_split
                ts = [float(x) for x in re.split(r"[,/]", request.TensorSplit) if x.strip()] or None
                if ts is not None and len(ts) != len(rpc_servers) + 1:
                    ts = None
                model, tok, mcfg, _ = load_split(path, rpc_servers, self.device, ts, ov)
            else:
                model, tok, mcfg, _ = load_llm(path, self.device, overrides=ov)
            self.vision = None
            if request.MMProj:
                from ..models.vision import load_mmproj
                mp = request.MMProj
                if not mp.startswith("synthetic:") and not os.path.isabs(mp) and request.ModelPath:
                    mp = os.path.join(request.ModelPath, mp)
                self.vision = load_mmproj(mp, self.device)
                if self.vision.proj_hidden != mcfg.hidden:
                    raise ValueError(f"mmproj projects to {self.vision.proj_hidden} but the LLM hidden size is "
                                     f"{mcfg.hidden}; make sure that you use the correct mmproj file")
            draft = None
            if request.DraftModel and self.tp is None:
                # speculative decoding (llama.cpp `-md` / reference `draft_model`): same tokenizer,
                # same GPU; k draft tokens per step from the `n_draft` option (default 4)
                dp = request.DraftModel
                if not dp.startswith("synthetic:") and not os.path.isabs(dp) and request.ModelPath:
                    dp = os.path.join(request.ModelPath, dp)
                draft, _dtok, dcfg, _ = load_llm(dp, self.device)
                if dcfg.vocab > mcfg.vocab:
                    raise ValueError(f"draft model vocab ({dcfg.vocab}) does not match the model's ({mcfg.vocab})")
                ec.n_draft = int(opts.get("n_draft", 4) or 4)
                ec.spec_max_batch = int(opts.get("spec_max_batch", ec.spec_max_batch))
            self.engine = LLMEngine(model, tok, ec, tp=self.tp, draft=draft)
            if not opts.get("lazy_graphs"):
                self.engine.precapture_graphs()
            self.engine.start()
            self.tok = tok
            self.model_opts = request
            self.embeddings_enabled = bool(request.Embeddings)
            self.triggers = [t.word for t in request.GrammarTriggers if t.word]
            self.state = pb.STATE_READY
            msg = f"loaded {path} in {time.perf_counter() - t0:.1f}s on {self.device}"
            mx = self._start_mxstream()
            if mx:
                msg += f"; mxstream={mx}"
            log.info(msg)
            return pb.Result(message=msg, success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            self.state = pb.STATE_ERROR
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    # ---------------------------------------------------------------- helpers
    def _need_engine(self, context):
        if self.engine is None:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "model not loaded")

    def _prompt_text(self, r) -> tuple[str, bool]:
        """-> (prompt text, whether BOS/special tokens still need adding)."""
        if r.UseTokenizerTemplate and len(r.Messages) and getattr(self.tok, "chat_template", None):
            from ..templates.chat import render_chat
            msgs = [{"role": m.role, "content": m.content} for m in r.Messages]
            return render_chat(msgs, self.tok, add_generation_prompt=True), False
        return r.Prompt, True

    def _prompt_ids(self, r) -> list[int]:
        if len(r.EmbeddingTokens) and not r.Prompt and not (r.UseTokenizerTemplate and len(r.Messages)):
            return list(r.EmbeddingTokens)
        text, special = self._prompt_text(r)
        return self.tok.encode(text, add_special=special)

    def _mm_prompt(self, r) -> tuple[list[int], list]:
        """Images (and, for a Qwen2-VL-family projector, videos as frame lists: vLLM's multi_modal_data["video"],
        backend/python/vllm/backend.py:238-252): encode with the vision tower + projector and splice the embeddings
        where the prompt has `[img-N]` / `[vid-N]` or the Qwen template's image / video pads (grpc-server.cpp:900-944;
        without markers the media precede the prompt, as the reference's input_suffix handling does). Placeholder
        rows use token id 0."""
        from ..models.vision import split_media
        text, special = self._prompt_text(r)
        imgs = list(r.Images)
        vids = list(r.Videos) if hasattr(self.vision, "embed_video") else []
        parts = split_media(text, len(imgs), len(vids))
        embs = {("img", i): e for i, e in enumerate(self.vision.embed_images(imgs))}
        for i, v in enumerate(vids):
            embs[("vid", i)] = self.vision.embed_video([v])
        ids: list[int] = []
        mm = []
        first = True
        for part in parts:
            if isinstance(part, tuple):
                e = embs[part]
                mm.append((len(ids), e))
                ids.extend([0] * e.shape[0])
            else:
                ids.extend(self.tok.encode(part, add_special=special and first) if (part or first) else [])
            first = False
        return ids, mm

    def _grammar(self, gbnf: str):
        from ..runtime_native import GrammarMatcher, NativeGrammar, NativeVocab
        with self._glock:
            if self._vocab is None:
                self._tb = self.tok.token_bytes()
                self._vocab = NativeVocab(self._tb)
            g = self._grammars.get(gbnf)
            if g is None:
                g = NativeGrammar(gbnf)
                if len(self._grammars) > 64:
                    self._grammars.clear()
                self._grammars[gbnf] = g
        eos = self.tok.eos_token_id if self.tok.eos_token_id is not None else -1
        vocab, tb = self._vocab, self._tb

        def make():
            return GrammarMatcher(g, vocab, tb, eos)
        if self.triggers:
            return lambda: LazyGrammar(make, self.triggers, tb)
        return make

    def _request(self, r) -> Request:
        mm = []
        if (len(r.Images) or (len(r.Videos) and hasattr(self.vision, "embed_video"))) and self.vision is not None:
            if self.tp is not None:
                raise ValueError("images with a tensor-parallel LLM worker are not supported")
            ids, mm = self._mm_prompt(r)
        else:
            ids = self._prompt_ids(r)
        mt = int(r.Tokens)
        max_tokens = mt if mt > 0 else self.engine.cfg.max_model_len
        req = Request(ids, sampling_from_predict(r), max_tokens, [s for s in r.StopPrompts if s])
        req.cache_prompt = not mm  # image placeholders must not enter the prefix cache (reference: same)
        req.n_draft = int(r.NDraft or 0)  # per-request cap on speculative draft length (0 = engine default)
        req.mm_embeds = mm
        req.n_keep = int(r.NKeep) if r.NKeep > 0 else 0
        if r.Grammar:
            req.grammar = self._grammar(r.Grammar)
        if (len(r.Images) and self.vision is None) or (len(r.Videos) and not hasattr(self.vision, "embed_video")) \
                or len(r.Audios):
            log.warning("ignoring %d images / %d videos / %d audios: this model has no projector for them",
                        len(r.Images) if self.vision is None else 0,
                        len(r.Videos) if not hasattr(self.vision, "embed_video") else 0, len(r.Audios))
        return req

    @staticmethod
    def _reply(o, text: bytes | str = b"") -> object:
        if isinstance(text, str):
            text = text.encode("utf-8")
        return pb.Reply(message=text, tokens=o.completion_tokens, prompt_tokens=o.prompt_tokens,
                        timing_prompt_processing=o.t_prompt_ms, timing_token_generation=o.t_gen_ms)

    # ---------------------------------------------------------------- RPCs
    def _submit_async(self, req):
        """Submit with an asyncio queue behind a per-loop channel: the engine delivers each step's
        outputs for all streams of this loop in one call_soon_threadsafe (engine.BatchedSink)."""
        import asyncio
        from ..engine.engine import BatchedSink
        loop = asyncio.get_running_loop()
        eng = self.engine
        if eng.batch_sink is None:
            eng.batch_sink = BatchedSink()
        ch = self._channels.get(id(loop))
        if ch is None:
            ch = self._channels[id(loop)] = _LoopChannel(loop)
        q: asyncio.Queue = asyncio.Queue()
        h = eng.submit(req, batch_key=_QKey(ch, q))
        return h, q

    async def Predict(self, request, context):
        if self.engine is None:
            await context.abort(grpc.StatusCode.FAILED_PRECONDITION, "model not loaded")
        req = self._request(request)
        h, q = self._submit_async(req)
        parts = []
        try:
            while True:
                o = await q.get()
                parts.append(o.text)
                if o.finished:
                    h.done = True
                    break
        finally:
            if not h.done:
                self.engine.abort(req.rid)
        if o.finish_reason and o.finish_reason.startswith("error"):
            await context.abort(grpc.StatusCode.INTERNAL, o.finish_reason)
        return self._reply(o, "".join(parts))

    async def PredictStream(self, request, context):
        """One Reply per engine output; when the client lags, queued outputs are coalesced into a
        single Reply (fewer messages under load, same byte stream)."""
        if self.engine is None:
            await context.abort(grpc.StatusCode.FAILED_PRECONDITION, "model not loaded")
        req = self._request(request)
        h, q = self._submit_async(req)
        try:
            while True:
                o = await q.get()
                text = o.text
                while not o.finished and not q.empty():
                    o = q.get_nowait()
                    text += o.text
                if o.finished:
                    h.done = True
                    if o.finish_reason and o.finish_reason.startswith("error"):
                        await context.abort(grpc.StatusCode.INTERNAL, o.finish_reason)
                    yield self._reply(o, text)
                    return
                if text:
                    yield pb.Reply(message=text.encode("utf-8"))
        finally:
            if not h.done:  # client went away: free the sequence's KV blocks now
                self.engine.abort(req.rid)

    def SoundGeneration(self, request, context):
        a = getattr(self, "_audio", None)
        if a is None:
            return self._no_audio(context, "SoundGeneration needs a MusicGen model (type: MusicgenForConditionalGeneration)")
        return a.SoundGeneration(request, context)

    def TTS(self, request, context):
        a = getattr(self, "_audio", None)
        if a is None:
            return self._no_audio(context, "TTS is not implemented by the LLM backend (MusicGen / OuteTTS models only)")
        return a.TTS(request, context)

    @staticmethod
    def _no_audio(context, msg):
        if context is not None:
            context.abort(grpc.StatusCode.UNIMPLEMENTED, msg)
        return pb.Result(message=msg, success=False)

    def Embedding(self, request, context):
        self._need_engine(context)
        if len(request.EmbeddingTokens):
            ids = list(request.EmbeddingTokens)
        else:
            ids = self.tok.encode(request.Embeddings or request.Prompt, add_special=True)
        req = Request(ids, SamplingParams(temperature=0.0), 1)
        req.embedding = True
        req.cache_prompt = False
        h = self.engine.submit(req)
        last = None
        for o in h:
            last = o
        if last is None or last.embedding is None:
            context.abort(grpc.StatusCode.INTERNAL, f"embedding failed: {last.finish_reason if last else '?'}")
        return pb.EmbeddingResult(embeddings=last.embedding)

    def TokenizeString(self, request, context):
        self._need_engine(context)
        ids = self.tok.encode(request.Prompt, add_special=False)
        return pb.TokenizationResponse(length=len(ids), tokens=ids)

    def GetMetrics(self, request, context):
        m = self.engine.last_metrics if self.engine else {}
        return pb.MetricsResponse(slot_id=0, prompt_json_for_slot="",
                                  tokens_per_second=float(m.get("tokens_per_second", 0.0)),
                                  tokens_generated=int(m.get("tokens_generated", 0)),
                                  prompt_tokens_processed=int(m.get("prompt_tokens_processed", 0)))

    def Status(self, request, context):
        st = super().Status(request, context)
        if self.engine is None:
            st.state = self.state
            return st
        e = self.engine
        busy = e.sched.has_work()
        st.state = pb.STATE_BUSY if busy else self.state
        try:
            import torch
            if e.device.type == "cuda":
                st.memory.breakdown["gpu_allocated"] = int(torch.cuda.memory_allocated(e.device))
                st.memory.breakdown["kv_cache"] = int(e.kv.k.numel() * e.kv.k.element_size() * 2)
                st.memory.breakdown["weights"] = int(e.model.weight_bytes())
        except Exception:
            pass
        for k in ("prompt_tokens_total", "gen_tokens_total", "cached_tokens_total", "preemptions", "steps",
                  "graph_steps", "finished"):
            st.memory.breakdown[k] = int(e.stats.get(k, 0))
        # engine state for the gateway's /metrics gauges (gateway/observability.py scrape_backends)
        st.memory.breakdown["busy_ms"] = int(e.stats.get("busy_s", 0.0) * 1e3)
        st.memory.breakdown["running_seqs"] = len(e.sched.running)
        st.memory.breakdown["waiting_seqs"] = len(e.sched.waiting)
        try:
            nb = int(e.kv.num_blocks)
            st.memory.breakdown["kv_blocks_total"] = nb
            st.memory.breakdown["kv_blocks_used"] = nb - int(e.sched.bm.num_free)
        except Exception:
            pass
        return st


def _lora_list(request, model_path: str) -> list:
    """LoraAdapter (+LoraScale, default 1.0; relative to the model file's directory, as
    grpc-server.cpp:2402-2410) and LoraAdapters (+LoraScales) -> [(path, scale)]."""
    base = os.path.dirname(model_path) if model_path and not model_path.startswith("synthetic:") \
        else (request.ModelPath or "")

    def full(p):
        return p if os.path.isabs(p) or not base else os.path.join(base, p)
    out = []
    if request.LoraAdapter:
        out.append((full(request.LoraAdapter), request.LoraScale or 1.0))
    sc = list(request.LoraScales)
    for i, p in enumerate(request.LoraAdapters):
        out.append((full(p), sc[i] if i < len(sc) else 1.0))
    return out


def main(argv=None):
    import sys
    # the engine thread and the gRPC event loop share the GIL: hand it over quickly so a decode
    # step never waits a full default 5 ms switch interval behind stream bookkeeping
    sys.setswitchinterval(0.0005)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # tensor-parallel worker under torch.distributed.run: rank 0 serves gRPC, others follow
        from ..parallel.tp_engine import follower_main, init_from_env
        link, dev = init_from_env()
        if link.rank != 0:
            follower_main(link, dev)
            return
        worker_main(lambda: LLMServicer(device=str(dev), tp=link), argv)
        link.send_control("stop")
        return
    worker_main(LLMServicer, argv)


if __name__ == "__main__":
    main()
