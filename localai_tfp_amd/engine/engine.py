"""LLM serving engine: the MI355X worker's replacement for the reference's llama.cpp slot server
(backend/cpp/llama/grpc-server.cpp). One engine drives one model replica (one GPU, or one TP group).

Loop (one iteration = one `step()`, cf. `llama_server_queue::start_loop` + `update_slots`,
utils.hpp:255, grpc-server.cpp:1639):
    schedule  -> paged continuous batch (decode rows first, then prefill chunks)
    forward   -> decode-only steps replay a captured hipGraph per batch-size bucket
    sample    -> fused on-GPU sampler (greedy rows: argmax kernel inside the graph)
    process   -> stop tokens / stop strings / length, incremental detokenisation, timings

Requests arrive from any thread through `submit()`; each gets a `RequestHandle` whose queue
receives `StepOutput`s (the reference's task/result queues, utils.hpp:192-409).
"""
from __future__ import annotations

import collections
import os
import logging
import queue
import threading
import time
from dataclasses import dataclass

import numpy as np
import torch

from ..utils import roctx
from ..utils.pinned import PinnedRing
from ..models.llama import ForwardBatch, LlamaModel, Workspace
from ..ops.sampling import SamplerBatch
from .kv_cache import KVCache, make_block_manager
from .scheduler import Scheduler, SchedulerOutput, needs_host_state
from .sequence import Request, Sequence, Status, StepOutput

log = logging.getLogger("localai_tfp_amd.engine")

# tensor-parallel decode graphs end in a vocab-parallel argmax (no per-step logits all-gather)
VOCAB_PARALLEL_ARGMAX = os.environ.get("MX_TP_VOCAB_ARGMAX", "1") != "0"

# ---- serving-loop GC policy ----------------------------------------------------------------------
# A full (generation-2) collection walks every live Python object — the model's parameter wrappers,
# tokenizer tables, request state — and stalls the engine thread for milliseconds while the GPU idles
# (profiles: 5-7 ms host bubbles). After load / graph capture everything alive is frozen into the
# permanent generation (never rescanned) and young collections are made rarer; pauses are counted.
GC_STATS = {"gc_s": 0.0, "gc_n": 0, "gc_max_ms": 0.0}
_gc_t0 = [0.0]


def _gc_cb(phase, info):
    if phase == "start":
        _gc_t0[0] = time.perf_counter()
    else:
        dt = time.perf_counter() - _gc_t0[0]
        GC_STATS["gc_s"] += dt
        GC_STATS["gc_n"] += 1
        GC_STATS["gc_max_ms"] = max(GC_STATS["gc_max_ms"], dt * 1e3)
        k = f"gen{info.get('generation', 0)}_max_ms"  # which generation the long pauses come from
        GC_STATS[k] = max(GC_STATS.get(k, 0.0), dt * 1e3)


def gc_tune():
    """Called at engine start-up and after graph capture: collect + freeze what is alive, then count only
    the collections that happen while serving (the start-up collection itself walks every object created
    by model loading and is not a serving pause)."""
    import gc
    import os
    if os.environ.get("MX_GC_TUNE", "1") != "0":
        gc.collect()
        gc.freeze()
        # young collections every ~10k net container allocations: each pause scans at most that many objects
        # (round 3's 50k threshold gave rare but 10+ ms pauses, host_gc.gc_max_ms)
        gc.set_threshold(10_000, 5, 1000)
    for k in [k for k in GC_STATS if k.startswith("gen")]:
        del GC_STATS[k]
    GC_STATS.update(gc_s=0.0, gc_n=0, gc_max_ms=0.0)
    if _gc_cb not in gc.callbacks:
        gc.callbacks.append(_gc_cb)


@dataclass
class EngineConfig:
    max_num_seqs: int = 256
    # tokens per step (llama.cpp's n_batch; a model's `batch:` overrides it). 416 = a full c128 decode batch plus a
    # 288-token prompt chunk: the measured best step composition on MI355X (profiles/r5_step_composition.md; 512
    # packs two prompts' chunks into 512-row steps that the GEMM tiles cover less evenly)
    max_batched_tokens: int = 416
    prefill_chunk: int | None = None  # prompt tokens per sequence per step (None: the whole step budget)
    max_model_len: int = 8192
    block_size: int = 16
    num_blocks: int | None = None  # None -> size from free HBM
    kv_mem_fraction: float = 0.85
    enable_prefix_cache: bool = True
    use_graphs: bool = True
    graph_buckets: tuple = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 224, 256)
    # mixed steps (decode rows + prompt chunks) replay graphs too: prefill-token buckets, max prompt
    # sequences per graphed step, and a cap on captured graphs (captured lazily, first use of a shape)
    mixed_graph_tokens: tuple = tuple(int(x) for x in (__import__("os").environ.get("MX_MIXED_TOKENS") or
                                                       "64,128,192,256,288,320,352,384,448,512,768,1024").split(",")
                              if x.strip())
    mixed_graph_seqs: int = 4
    max_graphs: int = 64
    attn_part_size: int = 256  # must match ops.core.attn_decode's default
    # dense 16-bit copy of the layer projections for hipBLASLt (ops/linear.py DENSE_MIN_M_*). Off: the K-quant
    # MFMA kernels (qmm2 / qmm3) run every M > 4 GEMM on the quantised weights; MX_DENSE_CACHE=1 restores the copy
    # (A/B only; it costs 2 B/param of HBM)
    prefill_bf16_cache: bool = __import__("os").environ.get("MX_DENSE_CACHE", "0") == "1"
    kv_dtype: str = "bf16"  # paged KV cache element type: bf16 | fp8 (OCP e4m3, half the bytes per token)
    # overlap the host with the GPU: launch step N, then read step N-1's sampled tokens (async
    # device->host copy) and schedule N+1 while N runs; decode inputs come from the device
    overlap: bool = True
    # launched-but-unread steps kept in flight (2: the host post-processes step N-2 while N-1 runs and N
    # is queued, so a slow host step no longer idles the GPU). Default 1: at c128 the step is GPU-bound
    # and depth 2 measured the same throughput with a worse TTFT (profiles/r2_verify_depth_{1,2}.json:
    # 13618 vs 13590 tok/s, p50 TTFT 18.8 vs 30.2 ms)
    overlap_depth: int = int(__import__("os").environ.get("MX_OVERLAP_DEPTH", "1"))
    # time every GEMM shape of the model over the compiled tile / split candidates at load (ops/autotune.py)
    gemm_autotune: bool = __import__("os").environ.get("MX_GEMM_TUNE", "1") != "0"
    n_draft: int = 0  # speculative decoding: draft tokens per step (needs a draft model; 0 = off)
    spec_max_batch: int = 32  # speculate only on decode batches up to this size (latency-bound regime)


def kv_torch_dtype(name: str) -> torch.dtype:
    """KV cache type names (engine `kv_dtype`, reference `cache_type_k` / `cache_type_v`: f16 / q8_0 / ...) -> storage
    dtype: 16-bit types bf16, fp8 e4m3 (the gfx950-native 8-bit float), and the llama.cpp block formats q8_0 / q4_0 /
    q4_1 / q5_0 / q5_1 / iq4_nl as uint8 rows of real blocks (kv_format, ops/kvq.py)."""
    n = (name or "bf16").lower()
    if n in ("fp8", "f8", "e4m3", "fp8_e4m3"):
        return torch.float8_e4m3fn
    if n in ("q8", "q8_0", "q4_0", "q4_1", "q5_0", "q5_1", "iq4_nl"):
        return torch.uint8
    if n in ("bf16", "f16", "fp16", "f32", "auto", ""):
        return torch.bfloat16
    raise ValueError(f"unknown KV cache type {name!r}")


def kv_format_id(name: str) -> int:
    """ops/kvq.py format id of a KV cache type name (0 bf16, 1 fp8, 2.. llama.cpp block formats)."""
    from ..ops.kvq import FORMATS
    n = (name or "bf16").lower()
    n = "q8_0" if n == "q8" else n
    if n in FORMATS:
        return FORMATS[n]
    return 1 if kv_torch_dtype(n) == torch.float8_e4m3fn else 0


class RequestHandle:
    """Per-request output channel. By default a thread-safe queue; `sink` (e.g. an asyncio
    loop.call_soon_threadsafe bound to an asyncio.Queue) receives outputs instead."""

    def __init__(self, rid: int, sink=None):
        self.rid = rid
        self.q: queue.Queue[StepOutput] = queue.Queue()
        self.sink = sink
        self.done = False

    def put(self, o: StepOutput):
        if self.sink is not None:
            self.sink(o)
        else:
            self.q.put(o)

    def __iter__(self):
        while True:
            o = self.q.get()
            yield o
            if o.finished:
                return


class BatchedSink:
    """Collects the outputs of one engine step for handles submitted with a `batch_key` and hands
    them over per consumer channel in ONE call (`key.channel.deliver([(key, output), ...])`, from the
    engine thread): one loop.call_soon_threadsafe per step for the gRPC event loop, one sendall per
    step per mxstream connection — instead of one cross-thread wakeup per token."""

    def __init__(self, deliver=None):
        self.buf: list = []

    def flush(self):
        items, self.buf = self.buf, []
        by: dict = {}
        for k, o in items:
            by.setdefault(k.channel, []).append((k, o))
        for ch, its in by.items():
            ch.deliver(its)


class StepGraph:
    """hipGraph of one engine step for a shape bucket (forward + greedy argmax).

    Bucket (B, P, PS): B decode rows (padded: slot -1, length 1) followed by room for P prefill
    tokens in up to PS prefill sequences (padded sequences have q_len 0; padded attention tiles carry
    sequence -1 and exit). P = 0 is the decode-only graph. Mixed continuous-batching steps (decode rows
    plus an arriving prompt chunk) replay a graph too, so no step pays the ~7 ms of per-kernel Python
    launches of the eager forward.

    Every input lives in ONE static int32 device buffer (views below); the host writes the padded
    image into a pinned ring buffer and refreshes all inputs with ONE async H2D copy per step.
    """

    def __init__(self, engine: "LLMEngine", B: int, P: int = 0, PS: int = 0, L: int = 0):
        e = engine
        dev = e.device
        self.B, self.P, self.PS = B, P, PS
        # L > 0: decode-only graph for contexts of <= L keys (small batches): the decode attention is captured
        # with ONE partition per sequence — a single pass with no partition-merge launch (models/llama.py)
        self.L = L
        self.maxb = mb = e.max_blocks_per_seq
        self.rows = e.model.prefill_rows() if P else 1
        self.NT = (P // self.rows + PS) if P else 0  # prefill attention tile capacity
        T = B + P
        self.S = min(B + PS, e.ws.max_seqs)  # logits rows
        Bp = max(B, 1)
        # tokens has one dummy row past T: the in-graph fix-up of decode inputs sampled by the previous
        # (still unread) step scatters into it for the rows that need no fix
        lay = [("tokens", (T + 1,)), ("positions", (T,)), ("slots", (T,)), ("lidx", (self.S,)),
               ("dec_bt", (Bp, mb)), ("dec_lens", (Bp,)), ("fix_dst", (Bp,)), ("fix_src", (Bp,)), ("argmax_on", (1,))]
        if P:
            lay += [("pf_bt", (PS, mb)), ("pf_cu", (PS + 1,)), ("pf_ctx", (PS,)), ("pf_tseq", (self.NT,)),
                    ("pf_tq0", (self.NT,))]
        self.off, o = {}, 0
        for k, sh in lay:
            self.off[k] = (o, sh)
            o += int(np.prod(sh))
        self.n = o
        img = np.zeros(o, np.int32)
        self._default = img
        for k, v in (("slots", -1), ("dec_lens", 1), ("pf_tseq", -1), ("fix_dst", T), ("argmax_on", 1)):
            if k in self.off:
                self.view(img, k)[...] = v
        self.buf = torch.from_numpy(img.copy()).to(dev)
        # pinned staging ring: a slot is rewritten only after the H2D copy that read it has run
        self._pin = PinnedRing(e.pin_ring, 4 * o, dev) if dev.type == "cuda" else None
        v = {k: self.view(self.buf, k) for k in self.off}
        self.v = v
        self.prev = torch.zeros(e.ws.max_seqs, dtype=torch.int32, device=dev)  # previous step's samples
        self.argmax = torch.zeros(self.S, dtype=torch.int32, device=dev)
        self.fb = ForwardBatch(v["tokens"][:T], v["positions"], v["slots"], v["lidx"], n_decode=B,
                               dec_block_tables=v["dec_bt"][:B], dec_seq_lens=v["dec_lens"][:B],
                               dec_max_len=L or e.cfg.max_model_len)
        if P:
            self.fb.pf_block_tables, self.fb.pf_cu_q, self.fb.pf_ctx_lens = v["pf_bt"], v["pf_cu"], v["pf_ctx"]
            self.fb.pf_tiles = (v["pf_tseq"], v["pf_tq0"])
        self.graph = None
        self.logits = None
        self.replay_s = 0.0  # host time inside hipGraphLaunch (profiling)

    def view(self, flat, k):
        o, sh = self.off[k]
        return flat[o:o + int(np.prod(sh))].reshape(sh)

    def fits(self, plan: dict) -> bool:
        nd = plan["nd"]
        if nd > self.B:
            return False
        if "pf_cu" not in plan:
            return True
        cu = plan["pf_cu"]
        return (self.P and len(cu) - 1 <= self.PS and int(cu[-1]) <= self.P
                and len(plan["pf_tseq"]) <= self.NT and len(plan["lidx"]) <= self.S)

    def capture(self, engine: "LLMEngine", pool=None):
        from .. import _native as N
        s = torch.cuda.Stream(device=engine.device)
        s.wait_stream(torch.cuda.current_stream(engine.device))
        # tensor parallel: the graph ends at the vocabulary shards + a vocab-parallel argmax; sampled steps
        # gather the full logits after the replay (plan["gather"], every rank)
        self.vp = engine.model.tp_size > 1 and VOCAB_PARALLEL_ARGMAX
        self.fb.tp_local_logits = self.vp

        def head(lg):
            if self.vp:
                engine.model.vocab_argmax(lg, engine.ws, self.argmax)
            else:
                N.kcall("mxk_argmax_gated", lg.data_ptr(), lg.stride(0), self.S, lg.shape[1], self.argmax.data_ptr(),
                        self.v["argmax_on"].data_ptr(), N.stream_ptr())

        with torch.cuda.stream(s):
            for _ in range(2):  # warm-up (allocations, lazy init) outside capture
                self._fix()
                head(engine.model.forward(self.fb, engine.kv, engine.ws))
        torch.cuda.current_stream(engine.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool, stream=s):
            self._fix()
            self.logits = engine.model.forward(self.fb, engine.kv, engine.ws)
            head(self.logits)
        self.graph = g

    def _fix(self):
        v = self.v
        if v["tokens"].is_cuda:
            from .. import _native as N
            N.kcall("mxk_fix_tokens", v["tokens"].data_ptr(), v["fix_dst"].data_ptr(), v["fix_src"].data_ptr(),
                    self.prev.data_ptr(), v["fix_dst"].numel(), N.stream_ptr())
        else:
            v["tokens"].index_copy_(0, v["fix_dst"].long(), self.prev.index_select(0, v["fix_src"].long()))

    def image(self, plan: dict) -> np.ndarray:
        """Padded host image of the step's inputs in this bucket's layout."""
        img = self._default.copy()
        nd, B = plan["nd"], self.B
        tok, pos, sl = plan["tokens"], plan["positions"], plan["slots"]
        npf = len(tok) - nd
        for k, a in (("tokens", tok), ("positions", pos), ("slots", sl)):
            d = self.view(img, k)
            d[:nd] = a[:nd]
            d[B:B + npf] = a[nd:]
        lidx = plan["lidx"]
        d = self.view(img, "lidx")
        d[:len(lidx)] = lidx
        d[nd:len(lidx)] += B - nd  # prefill rows sit after the padded decode block
        if nd:
            bt = plan["dec_bt"]
            self.view(img, "dec_bt")[:nd, :bt.shape[1]] = bt
            self.view(img, "dec_lens")[:nd] = plan["dec_lens"]
        if "pf_cu" in plan:
            bt, cu = plan["pf_bt"], plan["pf_cu"]
            ns = len(cu) - 1
            self.view(img, "pf_bt")[:ns, :bt.shape[1]] = bt
            c = self.view(img, "pf_cu")
            c[:ns + 1] = cu
            c[ns + 1:] = cu[-1]  # padded sequences: q_len 0
            self.view(img, "pf_ctx")[:ns] = plan["pf_ctx"]
            ts = plan["pf_tseq"]
            self.view(img, "pf_tseq")[:len(ts)] = ts
            self.view(img, "pf_tq0")[:len(ts)] = plan["pf_tq0"]
        if "fix" in plan:
            dst, src = plan["fix"]
            self.view(img, "fix_dst")[:len(dst)] = dst
            self.view(img, "fix_src")[:len(src)] = src
        if not plan.get("argmax_on", True):
            self.view(img, "argmax_on")[0] = 0
        return img

    def run(self, plan: dict, prev=None):
        """prev: device int32 tokens of the previous (unread) step when the plan has a "fix" entry."""
        if "fix" in plan:
            self.prev[:prev.numel()].copy_(prev, non_blocking=True)
        img = self.image(plan)
        if self._pin is not None:
            self._pin.stage(img, self.buf)
        else:
            self.buf.copy_(torch.from_numpy(img))
        t0 = time.perf_counter()
        self.graph.replay()
        self.replay_s += time.perf_counter() - t0
        S = len(plan["lidx"])
        return self.logits[:S], self.argmax[:S]


class LLMEngine:
    def __init__(self, model: LlamaModel, tokenizer, cfg: EngineConfig | None = None, tp=None,
                 draft: LlamaModel | None = None):
        self.tp = tp  # parallel.tp_engine.TPLink (leader or follower side) when tensor parallel
        self.model = model
        self.tok = tokenizer
        self.cfg = cfg or EngineConfig()
        self.device = model.device
        mc = model.cfg
        c = self.cfg
        c.max_model_len = min(c.max_model_len, max(mc.ctx_train, 256)) if c.max_model_len else mc.ctx_train
        self.recurrent = bool(getattr(model, "recurrent", False))
        if self.recurrent:
            # state-space models (models/mamba.py): one cache "block" per sequence holding its
            # recurrent state, so the block id is the state slot; no prefix sharing, no drafts, no TP
            if tp is not None:
                raise ValueError("tensor parallelism is not supported for recurrent models")
            c.block_size = c.max_model_len
            c.enable_prefix_cache = False
            draft = None
        self.max_blocks_per_seq = (c.max_model_len + c.block_size - 1) // c.block_size
        use_spec = draft is not None and c.n_draft > 0 and tp is None
        frac = c.kv_mem_fraction
        self.kv_dtype = kv_torch_dtype(c.kv_dtype)
        self.kvf = kv_format_id(c.kv_dtype)
        eb = self.kv_dtype.itemsize
        if self.kvf >= 2:  # block-quantised rows: llama.cpp's bytes per element (e.g. q4_0 18 / 32)
            from ..ops.kvq import row_bytes
            eb = row_bytes(self.kvf, mc.head_dim) / mc.head_dim
        if use_spec:  # the draft's cache shares the block ids: split the pool bytes between the two
            per_t = KVCache.bytes_per_block(mc.n_layers, model.n_kv, c.block_size, mc.head_dim, eb)
            per_d = KVCache.bytes_per_block(draft.cfg.n_layers, draft.n_kv, c.block_size, draft.cfg.head_dim, eb)
            frac *= per_t / (per_t + per_d)
        if self.recurrent:
            nb = c.max_num_seqs + 1
            self.kv = model.make_state_cache(nb, c.block_size)
        else:
            nl = getattr(model, "kv_layers", mc.n_layers)
            nb = c.num_blocks or KVCache.auto_num_blocks(max(1, nl), model.n_kv, c.block_size, mc.head_dim,
                                                         self.device, frac, dtype_bytes=eb)
            if self.tp is not None:  # every rank must hold the same block ids
                nb = self.tp.allreduce_min(nb)
            if getattr(model, "remote", None) is not None:  # remote layer ranges: same block ids everywhere
                nb = model.remote.setup_kv(nb, c.block_size, c.kv_dtype, max(c.max_batched_tokens, c.max_num_seqs),
                                           c.max_num_seqs, max(1, -(-c.max_model_len // c.attn_part_size)))
                self.cfg.use_graphs = False  # a network hop cannot live inside a hipGraph
            self.kv = KVCache(nl, nb, model.n_kv, c.block_size, mc.head_dim, self.device, self.kv_dtype, kvf=self.kvf)
        self.bm = make_block_manager(nb, c.block_size, c.enable_prefix_cache)
        # scheduler + step planner: native (csrc/runtime/scheduler.cpp) on the native block manager; the Python
        # Scheduler is the reference implementation (MX_PY_SCHED=1, or no libmxrt)
        from . import native_scheduler as NS
        self.native_sched = (os.environ.get("MX_PY_SCHED", "0") != "1" and hasattr(self.bm, "_h") and NS.available())
        sched_cls = NS.NativeScheduler if self.native_sched else Scheduler
        self.sched = sched_cls(self.bm, c.block_size, c.max_num_seqs, c.max_batched_tokens, c.max_model_len,
                               prefill_chunk=c.prefill_chunk)
        max_parts = max(1, -(-c.max_model_len // c.attn_part_size))
        if self.recurrent:
            self.ws = model.make_workspace(max(c.max_batched_tokens, c.max_num_seqs), c.max_num_seqs)
        else:
            # rows: a mixed step's graph bucket pads its decode rows to the decode bucket (<= max_num_seqs) and its
            # prompt tokens to the next mixed-graph token bucket, so the workspace holds both paddings at once
            p_max = next((x for x in c.mixed_graph_tokens if x >= c.max_batched_tokens), c.max_batched_tokens)
            self.ws = Workspace(mc, max(c.max_batched_tokens, c.max_num_seqs + p_max), c.max_num_seqs, self.device,
                                model.tp_size, max_parts)
        self.sampler = SamplerBatch(self.device)
        self.handles: dict[int, RequestHandle] = {}
        self.seqs: dict[int, Sequence] = {}
        self._inbox: queue.Queue = queue.Queue()
        self._cv = threading.Condition()
        self._thread: threading.Thread | None = None
        self._stop = False
        self.graphs: dict[tuple, StepGraph] = {}
        self._graph_pool = None
        self.use_graphs = c.use_graphs and self.device.type == "cuda"
        self.eos_ids = set(getattr(tokenizer, "eos_token_ids", []) or [])
        self.stats = dict(steps=0, decode_tokens=0, prefill_tokens=0, graph_steps=0, preemptions=0,
                          busy_s=0.0, prompt_tokens_total=0, gen_tokens_total=0, cached_tokens_total=0,
                          out_tokens=0, finished=0, sched_s=0.0, plan_s=0.0, fwd_s=0.0, fwd_graph_s=0.0, wait_s=0.0,
                          process_s=0.0)
        self.last_metrics = {}
        # per-step host timeline (t0, scheduled, launched, sampler launched, committed, wait s, done, graph, nd,
        # prefill tokens, sampled rows) when MX_STEP_TRACE is set
        self.trace = [] if os.environ.get("MX_STEP_TRACE") else None
        self.trace_events = []  # (before launch, after sampler) device events per traced step
        self._trace_wait = 0.0
        self.on_step = None  # optional hook called with the step index before each loop step (bench)
        self.batch_sink: BatchedSink | None = None
        if c.prefill_bf16_cache and self.device.type == "cuda" and hasattr(model, "enable_prefill_bf16_cache"):
            model.enable_prefill_bf16_cache()
        if c.gemm_autotune and self.device.type == "cuda" and hasattr(model, "gemm_specs"):
            # per-shape GEMM plans timed on this GPU before any graph is captured (ops/autotune.py)
            from ..ops.autotune import tune_gemms
            self.stats_tune_s = tune_gemms(model.gemm_specs())
        # overlap mode state: the launched-but-unread step, the device tokens it samples, and pinned
        # host staging (ring of 3: a buffer is rewritten only after the step that used it was read)
        # tensor parallel: the leader ships each plan before launching it and broadcasts the sampled
        # tokens on the device (RCCL), so followers gather decode inputs exactly like the leader
        self.overlap = bool(c.overlap and not use_spec and not self.recurrent
                            and getattr(model, "remote", None) is None
                            and os.environ.get("MX_TP_OVERLAP", "1") != "0" if tp is not None else
                            c.overlap and not use_spec and not self.recurrent and getattr(model, "remote", None) is None)
        # rows whose next sample needs host state advanced by their in-flight token (a grammar mask, mirostat-2's
        # mu): by default they stay in every step — the step's forward is launched first and the previous step is
        # read while it runs, before the sampler (see _step_overlap). MX_OVERLAP_HOLD=1: such a row sits out
        # every other step instead (round-3 behaviour, kept for A/B)
        self.sched.hold_host_state = self.overlap and os.environ.get("MX_OVERLAP_HOLD", "0") == "1"
        self._inflight = collections.deque()  # launched-but-unread steps, oldest first
        self._prev_dev = None  # (device int32 tokens of the last launched step, {rid: row})
        self._pin_tok = self._pin_lp = self._pin_in = None
        self._pin_i = 0
        # pinned rings: one buffer per step that can be launched-but-unread (+1 being written)
        self.pin_ring = max(3, c.overlap_depth + 1)
        if self.overlap:
            n = max(c.max_num_seqs, 1)
            pin = self.device.type == "cuda"
            self._pin_tok = [torch.empty(n, dtype=torch.int32, pin_memory=pin) for _ in range(self.pin_ring)]
            self._pin_lp = [torch.empty(n, dtype=torch.float32, pin_memory=pin) for _ in range(self.pin_ring)]
        self.spec = None
        if use_spec:
            from .speculative import SpeculativeDecoder
            self.spec = SpeculativeDecoder(self, draft, c.n_draft, c.spec_max_batch)

    # ------------------------------------------------------------------ request API
    def submit(self, req: Request, sink=None, batch_key=None) -> RequestHandle:
        """`sink`: per-output callback; `batch_key` (with `self.batch_sink` set): outputs are
        gathered per step and delivered together as (batch_key, output) pairs."""
        h = RequestHandle(req.rid, sink)
        h.batch_key = batch_key
        self.handles[req.rid] = h
        self._inbox.put(("add", req))
        with self._cv:
            self._cv.notify()
        return h

    def abort(self, rid: int):
        self._inbox.put(("abort", rid))
        with self._cv:
            self._cv.notify()

    def _drain_inbox(self):
        while True:
            try:
                kind, x = self._inbox.get_nowait()
            except queue.Empty:
                return
            if kind == "add":
                req: Request = x
                max_prompt = self.cfg.max_model_len - 1
                if len(req.prompt_ids) > max_prompt:
                    # reference truncation rule (grpc-server.cpp:1793-1814): keep the head (n_keep)
                    # and the back half of what remains
                    ids = req.prompt_ids
                    n_keep = min(getattr(req, "n_keep", 0) or 0, max_prompt // 2)
                    erased = len(ids) - max_prompt
                    req.prompt_ids = ids[:n_keep] + ids[n_keep + erased:]
                if not req.prompt_ids:
                    req.prompt_ids = [getattr(self.tok, "bos_token_id", 0) or 0]
                s = self.sched.new_sequence(req, self.tok) if self.native_sched else Sequence(req, self.tok)
                self.seqs[req.rid] = s
                self.sched.add(s)
            else:
                s = self.sched.abort(x)
                if s is not None:
                    self._finish(s, "abort")

    # ------------------------------------------------------------------ loop
    def precapture_graphs(self):
        """Capture every decode bucket up front (vLLM-style) so no capture lands mid-serving."""
        if not self.use_graphs:
            return 0
        if self.tp is not None and self.tp.is_leader:
            self.tp.send_plan("capture")  # followers capture the same buckets in the same order
        n = 0
        c = self.cfg
        for b in c.graph_buckets:
            if b <= c.max_num_seqs and self._graph_for(b) is not None:  # decode-only buckets
                n += 1
        # the full-batch steps of a saturated server: the single-partition decode form and every mixed (decode + prompt
        # chunk) bucket the step budget allows, so no capture (~10-50 ms) stalls serving or lands in a timed window
        top = max((b for b in c.graph_buckets if b <= c.max_num_seqs), default=0)
        # (single-rank engines only: tensor-parallel ranks keep to the decode buckets they have always shared)
        if top and self.tp is None and not self.recurrent and hasattr(self.model, "prefill_rows") and \
                os.environ.get("MX_PRECAPTURE_MIXED", "1") == "1":
            keys = [(top, 0, 0, self.SINGLE_PART_CTX)] if top >= self.SINGLE_PART_B else []
            for p in c.mixed_graph_tokens:
                if p > c.max_batched_tokens or top + p > self.ws.max_tokens:
                    continue
                keys.append((top, p, c.mixed_graph_seqs, 0))
                if top >= self.SINGLE_PART_B:
                    keys.append((top, p, c.mixed_graph_seqs, self.SINGLE_PART_CTX))
            for k in keys:
                if len(self.graphs) >= c.max_graphs:
                    break
                if self._graph_get(k) is not None:
                    n += 1
        gc_tune()
        return n

    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
            self._thread.start()

    def shutdown(self):
        self._stop = True
        with self._cv:
            self._cv.notify_all()
        if self._thread:
            self._thread.join(timeout=10)
        if self.tp is not None and self.tp.is_leader and not getattr(self, "_tp_stopped", False):
            self._tp_stopped = True
            self.tp.send_plan(None)  # followers leave follow()

    def flush_outputs(self):
        bs = self.batch_sink
        if bs is not None and bs.buf:
            bs.flush()

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        gc_tune()
        while not self._stop:
            self._drain_inbox()
            self.flush_outputs()
            if not self.sched.has_work():
                if self._inflight:
                    self._drain_inflight()
                    self.flush_outputs()
                    continue
                with self._cv:
                    self._cv.wait(timeout=0.05)
                continue
            try:
                if self.on_step is not None:
                    self.on_step(self.stats["steps"])
                self.step()
            except Exception as ex:  # fail every in-flight request loudly, keep the worker alive
                log.exception("engine step failed")
                self._fail_step(ex)
            self.flush_outputs()

    def _fail_step(self, ex: Exception):
        """A step raised: drop the in-flight steps, finish every live request with the error, free all blocks."""
        self._inflight, self._prev_dev = collections.deque(), None
        if self.native_sched:
            self.sched.clear_prev()
        for s in list(self.sched.running) + list(self.sched.waiting):
            s.n_pending = 0
            self.sched.abort(s.rid)
            self._finish(s, f"error:{type(ex).__name__}: {ex}")
        # finished / aborted sequences still waiting on the dropped in-flight samples: nothing will read those
        # back now, so free their KV blocks (and native slots) here
        for s in list(self.sched.deferred):
            s.n_pending = 0
        if self.sched.deferred:
            self.sched.release_deferred()

    def run_until_done(self, max_steps: int = 1 << 30):
        """Synchronous driver (tests / bench): step until every submitted request finished."""
        self._drain_inbox()
        n = 0
        while (self.sched.has_work() or self._inflight) and n < max_steps:
            if self.sched.has_work():
                self.step()
            else:
                self._drain_inflight()
            self._drain_inbox()
            n += 1
        return n

    # ------------------------------------------------------------------ one iteration
    def step(self):
        if roctx.ENABLED:
            with roctx.range(f"engine.step {self.stats['steps']}"):
                return self._step()
        return self._step()

    def _step(self):
        t0 = time.perf_counter()
        if roctx.ENABLED:
            with roctx.range("schedule"):
                so = self.sched.schedule()
        else:
            so = self.sched.schedule()
        for s in so.preempted:
            if s.status == Status.FINISHED:
                self._finish(s, s.finish_reason or "error")
            else:
                self.stats["preemptions"] += 1
        if so.empty:
            if self._inflight:
                self._drain_inflight()
            return
        if self.overlap and self._overlap_ok(so):
            if self._inflight and not self._pending_on_device(so):
                so = self._drain_and_filter(so)  # a pending token lives in an older step's buffer
                if so is None:
                    return
            self.stats["overlap_steps"] = self.stats.get("overlap_steps", 0) + 1
            return self._step_overlap(so, t0)
        if self.overlap:
            self.stats["sync_steps"] = self.stats.get("sync_steps", 0) + 1
        if self._inflight:  # this step needs host-known tokens: read the in-flight ones first
            so = self._drain_and_filter(so)
            if so is None:
                return
        if self.spec is not None:
            for s in so.preempted:
                self.spec.forget(s.rid)
            if self.spec.eligible(so) and self.spec.step(so):
                st = self.stats
                st["steps"] += 1
                st["decode_tokens"] += len(so.decode)
                st["busy_s"] += time.perf_counter() - t0
                return
        t1 = time.perf_counter()
        if roctx.ENABLED:
            roctx.mark(f"decode={len(so.decode)} prefill={sum(p.n for p in so.prefill)}")
        toks, lps = self._forward_and_sample(so)
        t2 = time.perf_counter()
        self.sched.commit(so)
        self._process(so, toks, lps)
        t3 = time.perf_counter()
        dt = t3 - t0
        st = self.stats
        st["sched_s"] += t1 - t0
        st["fwd_s"] += t2 - t1
        st["process_s"] += t3 - t2
        st["steps"] += 1
        st["decode_tokens"] += len(so.decode)
        st["prefill_tokens"] += sum(p.n for p in so.prefill)
        st["busy_s"] += dt

    # ------------------------------------------------------------------ overlap mode
    @staticmethod
    def _simple_params(p) -> bool:
        """Sampling that needs no host-side token history or per-token host state."""
        return (p.mirostat != 2 and p.repeat_penalty == 1.0 and not p.presence_penalty and not p.frequency_penalty)

    @staticmethod
    def _argmax_only(items) -> bool:
        """True when every row's token is the plain argmax of its logits (greedy, no logit bias, no
        penalties, no grammar). The ONE predicate behind both decisions that must agree: whether tensor
        parallel ranks gather the full logits (plan["gather"] = not this) and whether the step takes the
        vocab-parallel argmax instead of the sampler (a sampler on an ungathered shard samples this rank's
        vocabulary slice only)."""
        return all(it.seq.params.greedy and not it.seq.params.logit_bias and it.seq.params.repeat_penalty == 1.0
                   and not it.seq.params.presence_penalty and not it.seq.params.frequency_penalty
                   and it.seq.grammar is None for it in items)

    def _overlap_params(self, p) -> bool:
        """Sampling the overlap pipeline can launch before the previous step's tokens reach the host: the
        simple chain, and repeat / presence / frequency penalties while at most one token per row is in
        flight (overlap_depth 1: the kernel counts that pending token, ops/sampling.py pack). Mirostat v2
        rows are launched only with their previous token processed (scheduler hold_host_state)."""
        if p.mirostat == 2:
            return True  # held by the scheduler, or its mu advanced by the late read in _step_overlap
        return self._simple_params(p) or self.cfg.overlap_depth <= 1

    def _overlap_row_ok(self, it) -> bool:
        s = it.seq
        ok = s.overlap_static
        if ok is None:  # the request's own part of the decision, fixed for its lifetime
            ok = s.overlap_static = not s.req.embedding and self._overlap_params(s.params)
        if not ok:
            return False
        # grammar rows: held by the scheduler while a token is in flight, or masked after the late read of that
        # token (_step_overlap), so their mask is current when they are sampled
        return s.grammar is None or not self.sched.hold_host_state or not s.n_pending

    def _overlap_ok(self, so: SchedulerOutput) -> bool:
        if not all(self._overlap_row_ok(it) for it in so.decode):
            return False
        return all(self._overlap_row_ok(it) for it in so.prefill if it.sample)

    def _overlap_sample_args(self, items):
        """(histories, pend_tok, pend) for the overlap sampler: full histories only for penalty rows, and the
        index of each row's in-flight previous token in the last launched step's token tensor."""
        params = [it.seq.params for it in items]
        if all(self._simple_params(p) for p in params):
            return [[] for _ in items], None, None
        if self._prev_dev is None:  # nothing in flight: the host histories are complete
            return [[] if self._simple_params(p) else it.seq.all_ids for it, p in zip(items, params)], None, None
        prev_tok, prev_map = self._prev_dev
        hist, pend = [], []
        for it, p in zip(items, params):
            if self._simple_params(p):
                hist.append([])
                pend.append(-1)
                continue
            hist.append(it.seq.all_ids)
            # n_pending counts this step's sample already (_step_overlap): > 1 = the previous token is in flight
            r = prev_map.get(it.seq.rid, -1) if (prev_map is not None and it.seq.n_pending > 1) else -1
            pend.append(r)
        return hist, prev_tok, pend

    def _step_overlap(self, so: SchedulerOutput, t0: float):
        """Launch this step without waiting for it; then read the previous step's tokens (its async
        copy has landed or lands while this step runs) and post-process them."""
        t1 = time.perf_counter()
        if roctx.ENABLED:
            roctx.push("plan")
        plan = self._plan(so)
        if roctx.ENABLED:
            roctx.pop()
        self.stats["plan_s"] += time.perf_counter() - t1
        items = list(so.decode) + [it for it in so.prefill if it.sample]
        # the graph's greedy argmax head runs only when this step takes its tokens from it
        plan["argmax_on"] = bool(items) and self._argmax_only(items)
        if self.tp is not None:
            plan["ns"] = len(items)
            plan["gather"] = bool(items) and not self._argmax_only(items)
            self.tp.send_plan(plan)
        if roctx.ENABLED:
            roctx.push("launch graph" if plan["graph"] else "launch eager")
        if self.trace is not None and self.device.type == "cuda":
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        logits, am = self._execute(plan)
        t_exec = time.perf_counter()
        tok_dev, lp_dev = None, None
        steps = [it.seq.n_generated for it in items]  # sampler step index (seed advance) of each row's sample
        # this step's samples are in flight from here on (their KV blocks must stay)
        nslots = None
        if self.native_sched:
            nslots = self.sched.item_slots(so, items)
            self.sched.add_pending(nslots, 1)
        else:
            for it in items:
                it.seq.n_pending += 1
        if items and not self.sched.hold_host_state and any(
                needs_host_state(it.seq) and it.seq.n_pending > 1 for it in items):
            # a grammar mask / mirostat mu needs the previous step's token: read that step now, while this
            # step's forward (already queued) keeps the GPU busy, then launch the sampler with current state
            self._drain_inflight()
        if items:
            if am is not None and self._argmax_only(items):
                tok_dev = am
            elif not logits.is_cuda:  # CPU reference sampler (host lists)
                hist, ptok, pend = self._overlap_sample_args(items)
                mask = self._grammar_mask(items, logits.shape[1]) if any(it.seq.grammar for it in items) else None
                t, l = self.sampler.sample(logits, [it.seq.params for it in items], hist, steps, mask, None, ptok,
                                           pend)
                tok_dev = torch.as_tensor(t, dtype=torch.int32)
                lp_dev = torch.as_tensor(l, dtype=torch.float32) if l is not None else None
            else:
                hist, ptok, pend = self._overlap_sample_args(items)
                mask = self._grammar_mask(items, logits.shape[1]) if any(it.seq.grammar for it in items) else None
                mus = ([it.seq.mirostat_mu for it in items] if any(it.seq.params.mirostat == 2 for it in items)
                       else None)
                tok_dev, lp_dev = self.sampler.sample(logits, [it.seq.params for it in items], hist, steps, mask,
                                                      mus, ptok, pend)
            if self.tp is not None:
                tok_dev = self._tp_bcast_tokens(tok_dev, len(items))
            k = self._pin_i
            self._pin_i = (k + 1) % self.pin_ring
            S = len(items)
            self._pin_tok[k][:S].copy_(tok_dev[:S], non_blocking=True)
            if lp_dev is not None:
                self._pin_lp[k][:S].copy_(lp_dev[:S], non_blocking=True)
            self._snapshot_collectives()
            ev = None
            if self.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
            new = (ev, k, items, lp_dev is not None, nslots)
        else:
            new = None
        if roctx.ENABLED:
            roctx.pop()
        t_samp = t2 = time.perf_counter()
        if self.trace is not None and self.device.type == "cuda":
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self.trace_events.append((ev0, ev1))
        self.sched.commit(so)
        if new is not None:
            self._inflight.append(new)
        self._prev_dev = (tok_dev, {it.seq.rid: r for r, it in enumerate(items)}) if items else None
        if self.native_sched:
            self.sched.set_prev(items, nslots) if items else self.sched.clear_prev()
        # read back the oldest launched steps, keeping `overlap_depth - 1` of them (plus this one) in
        # flight; a step without samples is a sync point (the next plan cannot gather from it)
        keep = max(0, self.cfg.overlap_depth - 1) if items else 0
        while len(self._inflight) > keep + (1 if new is not None else 0):
            prev = self._inflight.popleft()
            if roctx.ENABLED:
                with roctx.range("process_prev"):
                    self._process_inflight(prev)
            else:
                self._process_inflight(prev)
        t3 = time.perf_counter()
        if self.trace is not None:  # host timeline of this step (MX_STEP_TRACE; tools: bench.py dumps it)
            self.trace.append((t0, t1, t_exec, t_samp, t2, self._trace_wait, t3, bool(plan["graph"]), len(so.decode),
                               sum(p.n for p in so.prefill), len(items)))
            self._trace_wait = 0.0
        st = self.stats
        st["sched_s"] += t1 - t0
        st["fwd_s"] += t2 - t1
        if plan["graph"]:
            st["fwd_graph_s"] += t2 - t1
        st["process_s"] += t3 - t2
        st["steps"] += 1
        st["decode_tokens"] += len(so.decode)
        st["prefill_tokens"] += sum(p.n for p in so.prefill)
        st["busy_s"] += t3 - t0

    def _process_inflight(self, inf):
        ev, k, items, has_lp, nslots = inf
        t0 = time.perf_counter()
        if ev is not None:
            if roctx.ENABLED:
                with roctx.range("wait"):
                    ev.synchronize()
            else:
                ev.synchronize()
        self.stats["wait_s"] += time.perf_counter() - t0
        if self.trace is not None:
            self._trace_wait += time.perf_counter() - t0
        self._check_collectives()
        S = len(items)
        toks = self._pin_tok[k][:S].tolist()
        lps = self._pin_lp[k][:S].tolist() if has_lp else None
        now = time.perf_counter()
        if nslots is not None:
            self.sched.add_pending(nslots, -1)
        for j, it in enumerate(items):
            s = it.seq
            if nslots is None:
                s.n_pending -= 1
            if s.status == Status.FINISHED:
                continue  # finished on an earlier token (or aborted): this sample is discarded
            if s.t_first_token is None:
                s.t_first_token = now
            self._accept_tokens(s, [int(toks[j])], [lps[j]] if lps is not None else None)
        if self.sched.deferred:
            self.sched.release_deferred()

    def _pending_on_device(self, so: SchedulerOutput) -> bool:
        """Every decode row whose input token is still in flight can gather it from the latest step."""
        if self.native_sched:
            return self.sched.pending_on_device(so)
        rows = self._prev_dev[1] if self._prev_dev is not None else {}
        return all(it.seq.rid in rows for it in so.decode if it.seq.n_pending)

    def _drain_and_filter(self, so: SchedulerOutput) -> SchedulerOutput | None:
        """Read every in-flight step; drop sequences that finished on those tokens from the plan."""
        self._drain_inflight()
        if any(it.seq.status == Status.FINISHED for it in so.decode + so.prefill):
            self.sched.drop_finished()
            so = SchedulerOutput([it for it in so.decode if it.seq.status != Status.FINISHED],
                                 [it for it in so.prefill if it.seq.status != Status.FINISHED])
        return None if so.empty else so

    def _drain_inflight(self):
        q, self._inflight = self._inflight, collections.deque()
        self._prev_dev = None
        if self.native_sched:
            self.sched.clear_prev()
        while q:
            self._process_inflight(q.popleft())

    # decode-only graphs of fewer than SHORT_CTX_B rows get a second, short-context form (contexts <= SHORT_CTX
    # keys: one 512-key partition per sequence, no partition-merge launch)
    SHORT_CTX, SHORT_CTX_B = 512, 8
    # large decode-only batches with contexts <= 1024 keys: a graph whose attention is one partition per sequence
    # (models/llama.py SINGLE_PART_*: no partition-merge launch per layer)
    SINGLE_PART_CTX, SINGLE_PART_B = 1024, int(os.environ.get("MX_SINGLE_PART_MIN_B", "64"))

    def _graph_for(self, n: int) -> StepGraph | None:
        """Decode-only graph of the bucket holding n rows."""
        b = self._dec_bucket(n)
        return self._graph_get((b, 0, 0, 0)) if b else None

    def _dec_bucket(self, n: int) -> int | None:
        return next((x for x in self.cfg.graph_buckets if x >= n and x <= self.cfg.max_num_seqs), None)

    def _graph_key(self, plan: dict):
        """Shape bucket (B, P, PS) whose graph can run this plan, or None (eager)."""
        c = self.cfg
        if not self.use_graphs or "mm" in plan or plan["keep_hidden"]:
            return None
        nd = plan["nd"]
        B = self._dec_bucket(nd) if nd else 0
        if B is None:
            return None
        if "pf_cu" not in plan:
            if not nd:
                return None
            ml = int(plan["dec_lens"].max())
            if B < self.SHORT_CTX_B and ml <= self.SHORT_CTX:
                return (B, 0, 0, self.SHORT_CTX)
            if B >= self.SINGLE_PART_B and ml <= self.SINGLE_PART_CTX:
                return (B, 0, 0, self.SINGLE_PART_CTX)
            return (B, 0, 0, 0)
        if self.recurrent or not hasattr(self.model, "prefill_rows") or len(plan["pf_cu"]) - 1 > c.mixed_graph_seqs:
            return None
        npf = int(plan["pf_cu"][-1])
        P = next((x for x in c.mixed_graph_tokens if x >= npf), None)
        if P is None or B + P > self.ws.max_tokens:
            return None
        # the decode rows of a mixed step: one attention partition per sequence too (no partition-merge launch)
        if nd and B >= self.SINGLE_PART_B and int(plan["dec_lens"].max()) <= self.SINGLE_PART_CTX and \
                os.environ.get("MX_MIXED_SINGLE_PART", "1") == "1":
            return (B, P, c.mixed_graph_seqs, self.SINGLE_PART_CTX)
        return (B, P, c.mixed_graph_seqs, 0)

    def _graph_get(self, key, create: bool = True) -> StepGraph | None:
        if not self.use_graphs:
            return None
        key = tuple(int(x) for x in key)
        g = self.graphs.get(key)
        if g is None:
            if not create or len(self.graphs) >= self.cfg.max_graphs:
                return None
            if self._graph_pool is None:
                self._graph_pool = torch.cuda.graph_pool_handle()
            g = StepGraph(self, *key)
            try:
                g.capture(self, self._graph_pool)
            except Exception:
                log.exception("hipGraph capture failed for bucket %s; running eager", key)
                self.use_graphs = False
                return None
            self.graphs[key] = g
        return g

    # ------------------------------------------------------------------ step plan / execution
    def _plan(self, so: SchedulerOutput) -> dict:
        """Host-side description of one forward step (plain numpy; broadcast verbatim to tensor-
        parallel followers, which replay it with engine.follow())."""
        bs = self.cfg.block_size
        dec, pf = so.decode, so.prefill
        nd = len(dec)
        if self.native_sched:
            plan = self.sched.plan_arrays(so)
            plan["nd"], plan["keep_hidden"] = nd, False
            return self._plan_finish(so, plan)
        T = so.num_tokens
        tokens = np.empty(T, np.int32)
        positions = np.empty(T, np.int32)
        slots = np.empty(T, np.int32)
        i = 0
        fix_dst, fix_src = [], []
        prev_rows = self._prev_dev[1] if self._prev_dev is not None else {}
        for it in dec:
            s = it.seq
            p = s.num_computed
            if s.n_pending:  # input token sampled by the previous, still unread step: take it on device
                tokens[i] = 0
                fix_dst.append(i)
                fix_src.append(prev_rows[s.rid])
            else:
                tokens[i] = s.output_ids[-1] if s.output_ids else s.prompt_ids[-1]
            positions[i] = p
            slots[i] = s.blocks[p // bs] * bs + p % bs
            i += 1
        for it in pf:
            s = it.seq
            ids = s.all_ids
            r = np.arange(it.start, it.start + it.n)
            tokens[i:i + it.n] = ids[it.start:it.start + it.n]
            positions[i:i + it.n] = r
            blk = np.asarray(s.blocks, np.int32)
            slots[i:i + it.n] = blk[r // bs] * bs + r % bs
            i += it.n
        # rows whose logits are needed: decode rows + last row of finishing prefills
        lidx = list(range(nd))
        off = nd
        for it in pf:
            if it.sample:
                lidx.append(off + it.n - 1)
            off += it.n
        plan = {"nd": nd, "tokens": tokens, "positions": positions, "slots": slots,
                "lidx": np.asarray(lidx, np.int32), "keep_hidden": False}
        if fix_dst:
            plan["fix"] = (np.asarray(fix_dst, np.int64), np.asarray(fix_src, np.int64))
        if nd:
            maxb = max(len(it.seq.blocks) for it in dec)
            bt = np.zeros((nd, maxb), np.int32)
            lens = np.empty(nd, np.int32)
            for k, it in enumerate(dec):
                bt[k, :len(it.seq.blocks)] = it.seq.blocks
                lens[k] = it.seq.num_computed + 1
            plan["dec_bt"], plan["dec_lens"] = bt, lens
        if pf:
            maxb = max(len(it.seq.blocks) for it in pf)
            bt = np.zeros((len(pf), maxb), np.int32)
            cu = np.zeros(len(pf) + 1, np.int32)
            ctx = np.empty(len(pf), np.int32)
            for k, it in enumerate(pf):
                bt[k, :len(it.seq.blocks)] = it.seq.blocks
                cu[k + 1] = cu[k] + it.n
                ctx[k] = it.start + it.n
            plan["pf_bt"], plan["pf_cu"], plan["pf_ctx"] = bt, cu, ctx
        return self._plan_finish(so, plan)

    def _plan_finish(self, so: SchedulerOutput, plan: dict) -> dict:
        """The Python-side rest of a plan: multimodal spans, embedding rows, prefill attention tiles, graph bucket."""
        pf = so.prefill
        nd = plan["nd"]
        mm = []
        row = nd
        for it in pf:  # multimodal spans intersecting this chunk -> (row in T, embedding rows)
            for p0, emb in it.seq.req.mm_embeds:
                lo, hi = max(p0, it.start), min(p0 + emb.shape[0], it.start + it.n)
                if lo < hi:
                    mm.append((row + lo - it.start, emb[lo - p0:hi - p0]))
            row += it.n
        if mm:
            plan["mm"] = mm
        if pf:
            plan["keep_hidden"] = any(it.seq.req.embedding for it in pf if it.sample)
        if pf and self.device.type == "cuda" and hasattr(self.model, "prefill_rows"):
            from ..ops.core import prefill_tiles
            ts, tq = prefill_tiles([it.n for it in pf], self.model.prefill_rows())
            plan["pf_tseq"], plan["pf_tq0"] = np.asarray(ts, np.int32), np.asarray(tq, np.int32)
        key = self._graph_key(plan)
        # tensor parallel: a capture runs collectives, so only graphs every rank captured up front
        # (precapture_graphs: decode buckets) are used; single-rank engines capture on first use
        g = self._graph_get(key, create=self.tp is None) if key is not None else None
        if g is None and key is not None and key[3]:
            # a short-context form that is not captured (tensor parallel replays precaptured buckets only): the
            # bucket's full-context graph runs the same step
            key = (key[0], key[1], key[2], 0)
            g = self._graph_get(key, create=self.tp is None)
        plan["graph"] = key if g is not None and g.fits(plan) else False
        return plan

    def _execute(self, plan: dict):
        """Run the step's forward on this rank. Returns (logits, argmax-or-None)."""
        nd = plan["nd"]
        if plan["graph"]:
            g = self._graph_get(plan["graph"])
            logits, am = g.run(plan, self._prev_dev[0] if "fix" in plan else None)
            self.stats["graph_steps"] += 1
            if getattr(g, "vp", False) and plan.get("gather"):
                logits = self.model.finish_logits(logits, self.ws)
            return logits, am
        t = self._stage_plan(plan, ("tokens", "positions", "slots", "lidx", "dec_bt", "dec_lens", "pf_bt", "pf_cu",
                                    "pf_ctx", "pf_tseq", "pf_tq0"))
        fb = self._build_fb(plan, t)
        if "fix_dst" in t and fb.tokens.is_cuda:
            # one kernel (no int64 casts + index_select + index_copy launches)
            from .. import _native as N
            prev = self._prev_dev[0]
            if prev.dtype != torch.int32 or not prev.is_contiguous():
                prev = prev.to(torch.int32).contiguous()
            N.kcall("mxk_fix_tokens", fb.tokens.data_ptr(), t["fix_dst"].data_ptr(), t["fix_src"].data_ptr(),
                    prev.data_ptr(), t["fix_dst"].numel(), N.stream_ptr())
        elif (fix := self._fix_tensors(t)) is not None:
            dst, src, prev = fix
            fb.tokens.index_copy_(0, dst, prev.index_select(0, src))
        logits = self.model.forward(fb, self.kv, self.ws)
        self._hidden = self.model.last_hidden if fb.keep_hidden else None
        return logits, None

    def _stage_plan(self, plan: dict, keys) -> dict:
        """Every int32 array of the step (and the overlap-mode fix-up indices) in ONE pinned H2D copy.
        Never torch.from_numpy(...).to(dev): a copy from pageable memory makes the host wait for the
        stream to drain, i.e. the GPU idles while the rest of the step is launched."""
        arrays = [(k, plan[k]) for k in keys if k in plan]
        if "fix" in plan:
            arrays += [("fix_dst", plan["fix"][0]), ("fix_src", plan["fix"][1])]
        parts, spec, off = [], [], 0
        for k, a in arrays:
            a = np.asarray(a)
            parts.append(a.reshape(-1).astype(np.int32, copy=False))
            spec.append((k, off, a.shape))
            off += a.size
        d = self._stage_h2d(np.concatenate(parts) if parts else np.zeros(1, np.int32))
        return {k: d[o:o + int(np.prod(sh))].view(sh) for k, o, sh in spec}

    def _stage_h2d(self, flat: np.ndarray) -> torch.Tensor:
        """int32 host array -> device through the pinned ring (utils/pinned.py: a slot is reused only
        after the async copy that sourced it has run); a fresh pinned allocation per step costs ~ms."""
        if self.device.type != "cuda":
            return torch.from_numpy(np.array(flat, dtype=np.int32))
        if self._pin_in is None:
            c = self.cfg
            cap = 4 * (4 * c.max_batched_tokens + c.max_num_seqs * (6 + 2 * self.max_blocks_per_seq) + 1024)
            self._pin_in = PinnedRing(self.pin_ring, cap, self.device)
        return self._pin_in.stage(np.ascontiguousarray(flat, dtype=np.int32))

    def _fix_tensors(self, t: dict):
        if "fix_dst" not in t:
            return None
        return t["fix_dst"].long(), t["fix_src"].long(), self._prev_dev[0]

    def _forward_and_sample(self, so: SchedulerOutput):
        t0 = time.perf_counter()
        plan = self._plan(so)
        self.stats["plan_s"] += time.perf_counter() - t0
        sample_items = [it for it in so.decode] + [it for it in so.prefill if it.sample]
        greedy_only = self._argmax_only(sample_items)
        if self.tp is not None:
            plan["gather"] = bool(sample_items) and not greedy_only
            self.tp.send_plan(plan)
        logits, am = self._execute(plan)
        self._snapshot_collectives()
        if not sample_items:
            return [], None
        if am is not None and greedy_only:
            t0 = time.perf_counter()
            out = am.cpu().tolist()
            self.stats["wait_s"] += time.perf_counter() - t0
            self._check_collectives()
            return out, None
        out = self._sample(logits, sample_items)
        self._check_collectives()
        return out

    def _snapshot_collectives(self):
        """After a step's launches: queue the one-shot all-reduce error flag's async read-back (checked later,
        without blocking, by _check_collectives)."""
        if self.tp is None:
            return
        ar = getattr(self.model, "custom_ar", None)
        if ar is not None:
            ar.snapshot()

    def _check_collectives(self, every: int = 1):
        """Tensor parallel: the one-shot all-reduce kernel flags a peer that never delivered (bounded
        spin) instead of hanging; the flag is read from retired async snapshots (OneShotAllReduce.check never
        synchronises the stream), and a set flag fails the rank loudly (exit non-zero through TPLink)
        rather than serving wrong logits."""
        if self.tp is None:
            return
        ar = getattr(self.model, "custom_ar", None)
        if ar is None:
            return
        self._ar_checks = getattr(self, "_ar_checks", 0) + 1
        if self._ar_checks % every:
            return
        try:
            ar.check()
        except RuntimeError as ex:
            self.tp._fail("one-shot all-reduce", ex)

    def _build_fb(self, plan: dict, t: dict | None = None) -> ForwardBatch:
        nd = plan["nd"]
        if t is None:
            t = self._stage_plan(plan, ("tokens", "positions", "slots", "lidx", "dec_bt", "dec_lens", "pf_bt",
                                        "pf_cu", "pf_ctx"))
        fb = ForwardBatch(t["tokens"], t["positions"], t["slots"], t["lidx"], n_decode=nd)
        if nd:
            fb.dec_block_tables, fb.dec_seq_lens = t["dec_bt"], t["dec_lens"]
            fb.dec_max_len = int(plan["dec_lens"].max())
        if "pf_cu" in plan:
            fb.pf_block_tables, fb.pf_cu_q, fb.pf_ctx_lens = t["pf_bt"], t["pf_cu"], t["pf_ctx"]
            if "pf_tseq" in t:
                fb.pf_tiles = (t["pf_tseq"], t["pf_tq0"])
            cu = plan["pf_cu"]
            fb.pf_q_lens_host = [int(cu[k + 1] - cu[k]) for k in range(len(cu) - 1)]
            fb.pf_ctx_lens_host = [int(x) for x in plan["pf_ctx"]]
        fb.keep_hidden = bool(plan.get("keep_hidden"))
        fb.plan = plan  # host copy (remote pipeline stages replay it)
        fb.embed_rows = plan.get("mm")
        return fb

    # ------------------------------------------------------------------ tensor-parallel follower
    def follow(self):
        """Follower-rank loop: replay the leader's step plans (forward only; the leader samples).
        Returns when the leader sends a stop message."""
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            msg = self.tp.recv_plan()
            if msg is None:
                return
            if msg == "capture":
                self.precapture_graphs()
                continue
            self._execute(msg)
            ns = int(msg.get("ns", 0))
            if ns:  # overlap mode: the leader's sampled tokens, for the next plan's device-side fix-up
                self._prev_dev = (self._tp_bcast_tokens(None, ns), None)
            self._snapshot_collectives()
            self._check_collectives()

    def _tp_bcast_tokens(self, tok_dev, n: int):
        """Leader: broadcast its n sampled token ids (device int32) to the TP group on the compute stream;
        follower: receive them into a persistent device buffer (stream order makes one buffer enough: the
        next plan's fix-up reads it before the next broadcast rewrites it)."""
        import torch.distributed as dist
        buf = getattr(self, "_tp_tok", None)
        if buf is None or buf.numel() < n:
            buf = self._tp_tok = torch.zeros(max(n, self.cfg.max_num_seqs), dtype=torch.int32, device=self.device)
        v = buf[:n]
        if tok_dev is not None:
            v.copy_(tok_dev[:n].to(torch.int32))
        dist.broadcast(v, src=self.tp.src, group=self.tp.gpu_group)
        return v

    def _sample(self, logits, items):
        params = [it.seq.params for it in items]
        hist = [it.seq.all_ids for it in items]
        steps = [len(it.seq.output_ids) for it in items]
        mask = None
        if any(it.seq.grammar for it in items):
            mask = self._grammar_mask(items, logits.shape[1])
        mus = [it.seq.mirostat_mu for it in items] if any(p.mirostat == 2 for p in params) else None
        tok, lp = self.sampler.sample(logits, params, hist, steps, mask, mus)
        return tok.cpu().tolist(), (lp.cpu().tolist() if lp is not None else None)

    def _grammar_mask(self, items, V):
        words = (V + 31) // 32
        m = np.full((len(items), words), 0xFFFFFFFF, np.uint32)
        from ..runtime_native import GrammarMatcher
        batch, rows = [], []
        for k, it in enumerate(items):
            g = it.seq.grammar
            if g is None:
                continue
            nm = g if isinstance(g, GrammarMatcher) else getattr(g, "m", None)  # LazyGrammar: after its trigger
            if isinstance(nm, GrammarMatcher) and (not batch or (nm.v is batch[0].v and nm.eos == batch[0].eos)):
                batch.append(nm)
                rows.append(k)
            else:
                m[k] = g.allowed_mask(V)
        # the native rows together, on several threads (a new grammar state walks the whole vocabulary trie)
        GrammarMatcher.masks_into(batch, m, rows)
        t = torch.from_numpy(m.view(np.int32))
        if self.device.type != "cuda":
            return t
        # through a pinned ring (a pageable H2D copy would make the host wait for the queued forward)
        ring = getattr(self, "_pin_mask", None)
        if ring is None:
            ring = self._pin_mask = PinnedRing(self.pin_ring, m.nbytes, self.device)
        return ring.stage(m.view(np.int32)).view(len(items), words)

    # ------------------------------------------------------------------ post-processing
    def _process(self, so: SchedulerOutput, toks, lps):
        now = time.perf_counter()
        items = [it for it in so.decode] + [it for it in so.prefill if it.sample]
        for k, it in enumerate(items):
            s = it.seq
            if s.status == Status.FINISHED:
                continue
            if s.t_first_token is None:
                s.t_first_token = now
            if s.req.embedding:
                # last-token pooling over the final-normed hidden state, L2-normalised
                # (grpc-server.cpp:1357-1414 send_embedding with pooling != NONE)
                v = self._hidden[k]
                v = (v / v.norm().clamp_min(1e-12)).cpu().tolist()
                self.sched.finish(s, "stop")
                h = self.handles.get(s.rid)
                o = StepOutput(s.rid, finished=True, finish_reason="stop", embedding=v)
                self._fill_usage(s, o, metrics=False)
                self.handles.pop(s.rid, None)
                self.seqs.pop(s.rid, None)
                if h is not None:
                    if h.batch_key is not None and self.batch_sink is not None:
                        self.batch_sink.buf.append((h.batch_key, o))
                    else:
                        h.put(o)
                continue
            self._accept_tokens(s, [int(toks[k])], [lps[k]] if lps is not None else None)

    def _accept_tokens(self, s: Sequence, toks: list, lps: list | None):
        """Append sampled tokens to a sequence (one per plain step, several per speculative step),
        stopping at the first stop condition; flush text and emit. Returns (tokens appended, reason)."""
        reason = None
        n = 0
        for j, t in enumerate(toks):
            lp = lps[j] if lps is not None else None
            if s.grammar is not None:
                s.grammar.accept(t)
            if s.params.mirostat == 2 and lp is not None:
                # mu <- mu - eta * (surprise - tau)  (surprise in bits)
                s.mirostat_mu -= s.params.mirostat_eta * (-lp / 0.6931471805599453 - s.params.mirostat_tau)
            s.append_token(t, lp)
            n += 1
            self.stats["out_tokens"] += 1
            if (t in self.eos_ids or t in s.req.stop_token_ids) and not s.params.ignore_eos:
                reason = "stop"
                s.pop_output()  # EOS is not part of the visible output
            elif len(s.output_ids) >= s.req.max_tokens:
                reason = "length"
            elif s.known_len >= self.cfg.max_model_len:
                reason = "length"
            elif s.grammar is not None and s.grammar.is_done():
                reason = "stop"
            if reason:
                break
        text, hit = s.flush_text(final=reason is not None)
        if hit:
            reason = "stop"
        if reason:
            self.sched.finish(s, reason)
        self._emit(s, text, reason)
        return n, reason

    def _emit(self, s: Sequence, text: str, reason: str | None):
        h = self.handles.get(s.rid)
        ids, lp = s.take_pending()
        o = StepOutput(s.rid, text, ids, lp, reason is not None, reason)
        if reason is not None:
            self._fill_usage(s, o)
            if self.spec is not None:
                self.spec.forget(s.rid)
            self.handles.pop(s.rid, None)
            self.seqs.pop(s.rid, None)
            st = self.stats
            st["finished"] += 1
            st["prompt_tokens_total"] += len(s.prompt_ids)
            st["gen_tokens_total"] += len(s.output_ids)
            st["cached_tokens_total"] += s.num_cached
        if h is not None:
            if h.batch_key is not None and self.batch_sink is not None:
                self.batch_sink.buf.append((h.batch_key, o))
            else:
                h.put(o)

    def _fill_usage(self, s: Sequence, o: StepOutput, metrics: bool = True):
        o.prompt_tokens = len(s.prompt_ids)
        o.completion_tokens = len(s.output_ids)
        o.cached_tokens = s.num_cached
        t_first = s.t_first_token or time.perf_counter()
        o.ttft_ms = (t_first - s.t_arrival) * 1e3
        o.t_prompt_ms = (t_first - (s.t_first_sched or s.t_arrival)) * 1e3
        o.t_gen_ms = ((s.t_finish or time.perf_counter()) - t_first) * 1e3
        if metrics:
            self.last_metrics = dict(tokens_per_second=(o.completion_tokens / max(o.t_gen_ms, 1e-3) * 1e3),
                                     tokens_generated=o.completion_tokens,
                                     prompt_tokens_processed=o.prompt_tokens)

    def _finish(self, s: Sequence, reason: str):
        if s.status != Status.FINISHED:
            self.sched.finish(s, reason)
        s.finish_reason = reason
        self._emit(s, "", reason)

    # ------------------------------------------------------------------ convenience
    def generate(self, prompt_ids, params=None, max_tokens=32, stop=None) -> StepOutput:
        from ..ops.sampling import SamplingParams
        req = Request(list(prompt_ids), params or SamplingParams(temperature=0.0), max_tokens, stop or [])
        h = self.submit(req)
        if self._thread is None:
            self.run_until_done()
        text, ids = "", []
        last = None
        for o in h:
            text += o.text
            ids += o.token_ids
            last = o
        last.text, last.token_ids = text, ids
        return last
