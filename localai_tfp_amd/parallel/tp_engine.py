"""Tensor-parallel serving: one process per GPU, rank 0 leads.

The leader owns the scheduler, sampler, gRPC server and block manager; every engine step it sends
the step plan (engine._plan: token ids, positions, KV slots, block tables) to the followers, and all
ranks run the same forward (16-bit RCCL all-reduces over xGMI inside the model, parallel/tp.py;
vocab-parallel LM head gathered to every rank). Only the leader samples. Control messages (model
load / unload) travel on the same channel, so ranks stay in lock-step by construction.

Channel: a gloo (CPU/TCP) process group next to the RCCL one — plans are host data the followers
need on the host anyway, and a CPU broadcast never queues behind GPU work on the RCCL stream.
Wire format: a fixed 4 x int32 header {magic, kind, body length, sequence} and, for plans, ONE flat
int32 body (encode_plan: every array of the plan with its rank and shape) — no pickling on the hot
path; only control payloads and multimodal plans (float embeddings) fall back to a pickled object.

Failure detection: the gloo group has a finite timeout (MX_TP_TIMEOUT_S, default 600 s); the leader
sends a heartbeat whenever the channel has been idle for MX_TP_HEARTBEAT_S (5 s), so a follower that
hears nothing for a whole timeout knows the leader is gone, and the leader's next send fails as soon as
a follower's socket closes. Either side then logs and exits non-zero (os._exit: never waits on a
collective that cannot complete), so the process supervisor (serving/model_loader.py watchdog)
restarts the whole group instead of leaving it hung.
Behavioural parity: the reference's only TP is inside vLLM (backend/python/vllm/backend.py:106-107).
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
import time

import numpy as np
import torch

log = logging.getLogger("localai_tfp_amd.tp")

MAGIC = 0x4D585450  # "MXTP"
K_PLAN, K_STOP, K_CAPTURE, K_PICKLE, K_HEARTBEAT, K_PART = 1, 2, 3, 4, 5, 6
PLAN_ARRAYS = ("tokens", "positions", "slots", "lidx", "dec_bt", "dec_lens", "pf_bt", "pf_cu", "pf_ctx",
               "pf_tseq", "pf_tq0", "fix_dst", "fix_src")
EXIT_TP_FAILURE = 75

STOP = None


# ------------------------------------------------------------------ plan codec (int32, no pickles)
def encode_plan(plan: dict) -> np.ndarray:
    """Flat int32 image of a step plan: [nd, flags, graph bucket (B, P, PS, L), ns (rows the leader samples and
    broadcasts on the device: overlap mode), then per PLAN_ARRAYS entry: ndim, *shape, *data]."""
    g = plan.get("graph")
    flags = int(bool(g)) | (int(bool(plan.get("keep_hidden"))) << 1) | (int(bool(plan.get("gather"))) << 2) | \
        (int(not plan.get("argmax_on", True)) << 3)
    gk = (tuple(g) + (0, 0, 0, 0))[:4] if g else (0, 0, 0, 0)  # (B, P, PS[, L]) padded to 4
    parts = [np.array([plan["nd"], flags, *gk, int(plan.get("ns", 0))], np.int32)]
    arrays = dict(plan)
    if "fix" in plan:
        arrays["fix_dst"], arrays["fix_src"] = plan["fix"]
    for k in PLAN_ARRAYS:
        a = arrays.get(k)
        if a is None:
            parts.append(np.zeros(1, np.int32))
            continue
        a = np.asarray(a)
        parts.append(np.array([a.ndim, *a.shape], np.int32))
        parts.append(a.astype(np.int32, copy=False).reshape(-1))
    return np.concatenate(parts)


def decode_plan(buf: np.ndarray) -> dict:
    nd, flags = int(buf[0]), int(buf[1])
    plan = {"nd": nd, "graph": tuple(int(x) for x in buf[2:6]) if flags & 1 else False,
            "keep_hidden": bool(flags & 2), "gather": bool(flags & 4), "ns": int(buf[6]), "argmax_on": not flags & 8}
    i = 7
    for k in PLAN_ARRAYS:
        ndim = int(buf[i])
        i += 1
        if ndim == 0:
            continue
        shape = tuple(int(x) for x in buf[i:i + ndim])
        i += ndim
        n = int(np.prod(shape))
        plan[k] = buf[i:i + n].reshape(shape).copy()
        i += n
    if "fix_dst" in plan:
        plan["fix"] = (plan.pop("fix_dst").astype(np.int64), plan.pop("fix_src").astype(np.int64))
    return plan


class TPLink:
    """Leader -> follower channel of one tensor-parallel group.

    cpu_group carries only leader broadcasts (plans, control, heartbeats); sync_group (default: the same
    group, single-threaded users) carries the rare all-rank collectives, so a heartbeat can never be
    matched against a follower's all-reduce."""

    def __init__(self, rank: int, world: int, cpu_group, gpu_group=None, src: int = 0, heartbeat_s: float | None = None,
                 sync_group=None, shm: bool | None = None):
        self.rank, self.world = rank, world
        self.cpu_group, self.gpu_group = cpu_group, gpu_group
        self.sync_group = sync_group if sync_group is not None else cpu_group
        self.src = src  # global rank of the leader inside cpu_group
        self.is_leader = rank == 0
        self._lock = threading.Lock()
        self._sync_lock = threading.Lock() if sync_group is not None else self._lock
        self._quiet = 0
        self._seq = 0
        self._last_send = time.monotonic()
        self._hb = None
        hb = float(os.environ.get("MX_TP_HEARTBEAT_S", "5")) if heartbeat_s is None else heartbeat_s
        self.shm = None
        if shm is None:
            shm = os.environ.get("MX_TP_SHM", "1") != "0"
        if shm and world > 1:
            self.shm = self._open_shm(max(hb, 0.5))
        if self.is_leader and world > 1 and hb > 0 and self.shm is None:
            self._hb_stop = threading.Event()
            self._hb = threading.Thread(target=self._heartbeat, args=(hb,), daemon=True, name="tp-heartbeat")
            self._hb.start()

    def _open_shm(self, heartbeat: float):
        """Plans over a /dev/shm ring (parallel/shm_channel.py): all ranks of a group are on one node. The
        leader draws a random name and broadcasts it (16 raw bytes over the gloo group, no pickles)."""
        import torch.distributed as dist
        from .shm_channel import ChannelDead, ShmChannel, channel_name
        tok = torch.from_numpy(np.frombuffer(os.urandom(16), np.uint8).copy()) if self.is_leader else \
            torch.empty(16, dtype=torch.uint8)
        dist.broadcast(tok, src=self.src, group=self.cpu_group)
        name = channel_name(bytes(tok.numpy()).hex()[:20])
        to = tp_timeout().total_seconds()
        try:
            ch = ShmChannel(name, self.rank, self.world, create=self.is_leader, timeout=to, heartbeat=heartbeat)
        except (ChannelDead, OSError) as ex:
            self._fail("shared-memory channel setup", ex)
        dist.barrier(group=self.cpu_group)  # every follower attached before the leader may publish
        return ch

    # -------------------------------------------------------------- failure handling
    def _fail(self, what: str, ex: BaseException):
        log.critical("tensor-parallel rank %d: %s failed (%s: %s); exiting so the supervisor restarts the "
                     "group", self.rank, what, type(ex).__name__, ex)
        logging.shutdown()
        os._exit(EXIT_TP_FAILURE)

    def _heartbeat(self, period: float):
        while not self._hb_stop.wait(period / 2):
            if not self._quiet and time.monotonic() - self._last_send >= period:
                self._send(K_HEARTBEAT)

    class _Quiet:
        def __init__(self, link):
            self.link = link

        def __enter__(self):
            self.link._quiet += 1

        def __exit__(self, *a):
            self.link._quiet -= 1
            self.link._last_send = time.monotonic()

    def quiet(self):
        """No heartbeats while the followers are busy outside the channel (model load): a broadcast
        waits for its receivers, and a heartbeat queued behind a long load would hit the timeout."""
        return TPLink._Quiet(self)

    def close(self):
        if self._hb is not None:
            self._hb_stop.set()
        if self.shm is not None:
            self.shm.close()

    # -------------------------------------------------------------- raw channel
    def _send(self, kind: int, body: np.ndarray | None = None, obj=None):
        import torch.distributed as dist
        if self.shm is not None:
            from .shm_channel import ChannelDead
            with self._lock:
                try:
                    b = None if body is None else np.ascontiguousarray(body, np.int32)
                    if b is not None and b.nbytes > self.shm.max_body():
                        # oversized plan (long prompts, many sequences): raw int32 pieces through the same ring,
                        # the last one carrying the message kind — no pickling
                        per = self.shm.max_body() // 4
                        for o in range(0, b.size - per, per):
                            self.shm.send(K_PART, b[o:o + per])
                        self.shm.send(kind, b[(b.size - 1) // per * per:])
                    else:
                        self.shm.send(kind, b)
                        if kind == K_PICKLE:
                            dist.broadcast_object_list([obj], src=self.src, group=self.cpu_group)
                    self._last_send = time.monotonic()
                except (ChannelDead, RuntimeError) as ex:
                    self._fail("send", ex)
            return
        with self._lock:
            try:
                self._seq += 1
                n = 0 if body is None else int(body.size)
                hdr = torch.tensor([MAGIC, kind, n, self._seq], dtype=torch.int32)
                dist.broadcast(hdr, src=self.src, group=self.cpu_group)
                if n:
                    dist.broadcast(torch.from_numpy(np.ascontiguousarray(body, np.int32)), src=self.src,
                                   group=self.cpu_group)
                if kind == K_PICKLE:
                    dist.broadcast_object_list([obj], src=self.src, group=self.cpu_group)
                self._last_send = time.monotonic()
            except Exception as ex:  # a follower died or the group timed out
                self._fail("send", ex)

    def _recv(self):
        import torch.distributed as dist
        if self.shm is not None:
            from .shm_channel import ChannelDead
            try:
                kind, raw = self.shm.recv()
                parts = []
                while kind == K_PART:  # pieces of an oversized message (see _send)
                    parts.append(np.frombuffer(raw, np.int32))
                    kind, raw = self.shm.recv()
                if parts:
                    parts.append(np.frombuffer(raw, np.int32))
                    body = np.concatenate(parts)
                else:
                    body = np.frombuffer(raw, np.int32).copy() if raw else None
                obj = None
                if kind == K_PICKLE:
                    buf = [None]
                    dist.broadcast_object_list(buf, src=self.src, group=self.cpu_group)
                    obj = buf[0]
                    if isinstance(obj, dict):
                        kind = K_PLAN
                        body = encode_plan(obj) if "mm" not in obj else None
                        if body is None:
                            kind = K_PICKLE
                return kind, body, obj
            except (ChannelDead, RuntimeError) as ex:
                self._fail("receive", ex)
        while True:
            try:
                hdr = torch.empty(4, dtype=torch.int32)
                dist.broadcast(hdr, src=self.src, group=self.cpu_group)
                magic, kind, n, _seq = (int(x) for x in hdr)
                if magic != MAGIC:
                    raise RuntimeError(f"bad tensor-parallel header {hdr.tolist()}")
                body = None
                if n:
                    t = torch.empty(n, dtype=torch.int32)
                    dist.broadcast(t, src=self.src, group=self.cpu_group)
                    body = t.numpy()
                obj = None
                if kind == K_PICKLE:
                    buf = [None]
                    dist.broadcast_object_list(buf, src=self.src, group=self.cpu_group)
                    obj = buf[0]
            except Exception as ex:  # leader gone (no heartbeat within the group timeout)
                self._fail("receive", ex)
            if kind != K_HEARTBEAT:
                return kind, body, obj

    # -------------------------------------------------------------- messages (leader -> followers)
    def send_plan(self, plan):
        assert self.is_leader
        if plan is None:
            self._send(K_STOP)
        elif isinstance(plan, str) and plan == "capture":
            self._send(K_CAPTURE)
        elif "mm" in plan:  # multimodal embedding rows (float): rare, pickled
            self._send(K_PICKLE, obj=plan)
        else:
            self._send(K_PLAN, encode_plan(plan))

    def recv_plan(self):
        kind, body, obj = self._recv()
        if kind == K_STOP:
            return None
        if kind == K_CAPTURE:
            return "capture"
        if kind == K_PLAN:
            return decode_plan(body)
        return obj

    def send_control(self, kind: str, payload=None):
        self._send(K_PICKLE, obj=("ctl", kind, payload))

    def recv_control(self):
        _, _, msg = self._recv()
        if not (isinstance(msg, tuple) and msg and msg[0] == "ctl"):
            raise RuntimeError(f"tensor-parallel follower expected a control message, got {type(msg)}")
        return msg[1], msg[2]

    # -------------------------------------------------------------- collectives on host ints
    def allreduce_min(self, x: int) -> int:
        import torch.distributed as dist
        with self._sync_lock:
            t = torch.tensor([int(x)], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.sync_group)
            return int(t.item())


def tp_timeout() -> datetime.timedelta:
    return datetime.timedelta(seconds=float(os.environ.get("MX_TP_TIMEOUT_S", "600")))


def init_from_env():
    """torch.distributed.run environment -> (TPLink, local device). RCCL for the model's
    all-reduces, gloo (finite timeout + leader heartbeat, see module doc) for plans."""
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, timeout=tp_timeout())
    cpu = dist.new_group(backend="gloo", timeout=tp_timeout())
    sync = dist.new_group(backend="gloo", timeout=tp_timeout())
    return TPLink(rank, world, cpu, None, sync_group=sync), dev


def follower_main(link: TPLink, device):
    """Non-leader ranks: wait for control messages; on `load` build the same model shard + engine
    and replay plans until the leader unloads / stops."""
    from ..engine.engine import EngineConfig, LLMEngine
    from ..models.loader import load_llm
    while True:
        kind, payload = link.recv_control()
        if kind == "stop":
            return
        if kind != "load":
            continue
        path, overrides, ecfg_dict = payload
        model, tok, _, _ = load_llm(path, device, link.rank, link.world, link.gpu_group, overrides)
        ec = EngineConfig(**ecfg_dict)
        eng = LLMEngine(model, tok, ec, tp=link)
        log.info("rank %d: model shard loaded, following", link.rank)
        eng.follow()
        del eng, model
        torch.cuda.empty_cache()


def tp_selfcheck(cfg, src, device, rank: int, size: int, group, prompt_len: int = 37) -> float | None:
    """Logits of one prefill step of `cfg` sharded over the TP group vs the same weights unsharded on
    the leader (every rank must call). Returns max |dlogit| / max |logit| on the leader, None elsewhere.
    Used by bench.py --tp so a multi-GPU run validates what it measures."""
    from ..models.llama import ForwardBatch, LlamaModel, Workspace
    from ..engine.kv_cache import KVCache
    dev = torch.device(device)

    def run(model, tp):
        bs = 16
        kv = KVCache(cfg.n_layers, 8, model.n_kv, bs, cfg.head_dim, dev)
        ws = Workspace(cfg, 64, 4, dev, tp_size=tp)
        toks = torch.arange(prompt_len, dtype=torch.int32) * 7 % cfg.vocab
        P = prompt_len
        pos = torch.arange(P, dtype=torch.int32)
        blocks = list(range(1, (P + bs - 1) // bs + 1))
        slots = torch.tensor([blocks[p // bs] * bs + p % bs for p in range(P)], dtype=torch.int32)
        fb = ForwardBatch(toks.to(dev), pos.to(dev), slots.to(dev), torch.tensor([P - 1], dtype=torch.int32, device=dev),
                          n_decode=0, pf_block_tables=torch.tensor([blocks], dtype=torch.int32, device=dev),
                          pf_cu_q=torch.tensor([0, P], dtype=torch.int32, device=dev),
                          pf_ctx_lens=torch.tensor([P], dtype=torch.int32, device=dev), pf_q_lens_host=[P],
                          pf_ctx_lens_host=[P])
        return model.forward(fb, kv, ws).float().cpu().clone()

    m_tp = LlamaModel.load(cfg, src, dev, rank, size, group)
    out_tp = run(m_tp, size)
    del m_tp
    if rank != 0:
        return None
    m1 = LlamaModel.load(cfg, src, dev)
    ref = run(m1, 1)
    del m1
    return float((out_tp - ref).abs().max() / ref.abs().max().clamp_min(1e-6))
