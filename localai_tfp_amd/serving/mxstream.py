"""mxstream: a batched token channel between this framework's gateway and its LLM workers.

The backend.proto contract (PredictStream: one gRPC stream and one message per generated token) is
kept for compatibility — any gateway speaking the reference's protocol can drive the workers — but
at serving rates (10k+ tokens/s per GPU) the per-message cost of Python gRPC in both processes was
the largest overhead on the /v1/chat/completions path (the worker's gRPC event loop and the engine
thread share a GIL). mxstream carries the same information in bulk:

  gateway -> worker   SUBMIT(rid, PredictOptions bytes) | ABORT(rid)
  worker  -> gateway  BATCH: every output the engine produced for this connection in one step

over a Unix-domain socket (TCP loopback as a fallback). The worker's engine thread writes each
step's batch with a single sendall — no per-token Python object crosses a thread or an event loop in
the worker. The gateway demultiplexes batches into per-request asyncio queues.

Frames: u32 little-endian length (of what follows), u8 type, payload.
  SUBMIT  1: u64 rid | PredictOptions
  ABORT   2: u64 rid
  BATCH   3: u32 n | n x (u64 rid, u8 flags, u32 tokens, u32 prompt_tokens, f32 t_prompt_ms,
                        f32 t_gen_ms, u32 len, bytes)   flags: 1 finished, 2 error (bytes = message)
"""
from __future__ import annotations

import asyncio
import logging
import os
import socket
import struct
import threading

log = logging.getLogger("localai_tfp_amd.mxstream")

T_SUBMIT, T_ABORT, T_BATCH = 1, 2, 3
F_FINISHED, F_ERROR = 1, 2
_HDR = struct.Struct("<IB")
_ITEM = struct.Struct("<QBIIffI")
_U64 = struct.Struct("<Q")
_U32 = struct.Struct("<I")


def socket_path_for(addr: str) -> str:
    port = addr.rsplit(":", 1)[-1]
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"localai-mx-{os.getpid()}-{port}.sock")


def pack_batch(items) -> bytes:
    """items: iterable of (rid, flags, tokens, prompt_tokens, t_prompt_ms, t_gen_ms, data bytes)"""
    parts = []
    n = 0
    for rid, flags, tok, ptok, tp, tg, data in items:
        parts.append(_ITEM.pack(rid, flags, tok, ptok, tp, tg, len(data)))
        parts.append(data)
        n += 1
    body = _U32.pack(n) + b"".join(parts)
    return _HDR.pack(len(body) + 1, T_BATCH) + body


def unpack_batch(body: memoryview):
    (n,) = _U32.unpack_from(body, 0)
    off = 4
    out = []
    for _ in range(n):
        rid, flags, tok, ptok, tp, tg, ln = _ITEM.unpack_from(body, off)
        off += _ITEM.size
        out.append((rid, flags, tok, ptok, tp, tg, bytes(body[off:off + ln])))
        off += ln
    return out


def _recv_exact(sock: socket.socket, n: int) -> bytes | None:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            return None
        got += k
    return bytes(buf)


# ------------------------------------------------------------------------------------------------
# worker side

class _Conn:
    """One gateway connection: the engine's BatchedSink channel for outputs keyed by (conn, rid)."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.lock = threading.Lock()
        self.engine_rid: dict[int, int] = {}
        self.alive = True

    def deliver(self, items):
        """Called from the engine thread with [(key, StepOutput)]; one sendall per step."""
        recs = []
        for key, o in items:
            flags = F_FINISHED if o.finished else 0
            data = o.text.encode("utf-8") if o.text else b""
            if o.finished and o.finish_reason and o.finish_reason.startswith("error"):
                flags |= F_ERROR
                data = o.finish_reason.encode("utf-8", "replace")
            recs.append((key.rid, flags, o.completion_tokens, o.prompt_tokens, o.t_prompt_ms, o.t_gen_ms, data))
            if o.finished:
                self.engine_rid.pop(key.rid, None)
        if not recs or not self.alive:
            return
        frame = pack_batch(recs)
        try:
            with self.lock:
                self.sock.sendall(frame)
        except OSError:
            self.alive = False


class _Key:
    __slots__ = ("channel", "rid")

    def __init__(self, channel, rid):
        self.channel, self.rid = channel, rid


class StreamServer:
    """Accepts gateway connections for an LLMServicer (workers/llm.py) and feeds its engine."""

    def __init__(self, servicer, path: str):
        self.svc = servicer
        self.path = path
        if os.path.exists(path):
            os.unlink(path)
        self.lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.lsock.bind(path)
        self.lsock.listen(64)
        self._stop = False
        threading.Thread(target=self._accept, daemon=True, name="mxstream-accept").start()

    def close(self):
        self._stop = True
        try:
            self.lsock.close()
            os.unlink(self.path)
        except OSError:
            pass

    def _accept(self):
        while not self._stop:
            try:
                s, _ = self.lsock.accept()
            except OSError:
                return
            s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
            threading.Thread(target=self._serve, args=(s,), daemon=True, name="mxstream-conn").start()

    def _serve(self, s: socket.socket):
        from ..grpc import pb
        conn = _Conn(s)
        svc = self.svc
        try:
            while True:
                hdr = _recv_exact(s, _HDR.size)
                if hdr is None:
                    break
                ln, typ = _HDR.unpack(hdr)
                body = _recv_exact(s, ln - 1) if ln > 1 else b""
                if body is None:
                    break
                if typ == T_SUBMIT:
                    (rid,) = _U64.unpack_from(body, 0)
                    opts = pb.PredictOptions.FromString(body[8:])
                    try:
                        req = svc._request(opts)
                    except Exception as ex:  # bad request: report as an error output
                        conn.deliver([(_Key(conn, rid), _ErrOut(str(ex)))])
                        continue
                    conn.engine_rid[rid] = req.rid
                    self._ensure_sink()
                    svc.engine.submit(req, batch_key=_Key(conn, rid))
                elif typ == T_ABORT:
                    (rid,) = _U64.unpack_from(body, 0)
                    erid = conn.engine_rid.pop(rid, None)
                    if erid is not None:
                        svc.engine.abort(erid)
        except OSError:
            pass
        finally:
            conn.alive = False
            for erid in list(conn.engine_rid.values()):
                svc.engine.abort(erid)
            try:
                s.close()
            except OSError:
                pass

    def _ensure_sink(self):
        from ..engine.engine import BatchedSink
        eng = self.svc.engine
        if eng.batch_sink is None:
            eng.batch_sink = BatchedSink(None)
        eng.batch_sink.routed = True


class _ErrOut:
    finished = True
    completion_tokens = prompt_tokens = 0
    t_prompt_ms = t_gen_ms = 0.0
    text = ""

    def __init__(self, msg):
        self.finish_reason = "error:" + msg


# ------------------------------------------------------------------------------------------------
# gateway side

class StreamClient:
    """asyncio client bound to one event loop; many concurrent requests share the connection."""

    def __init__(self, path: str):
        self.path = path
        self.reader = self.writer = None
        self.queues: dict[int, asyncio.Queue] = {}
        self._rid = 0
        self._task = None
        self._lock = None

    async def _connect(self):
        if self.writer is not None:
            return
        if self._lock is None:
            self._lock = asyncio.Lock()
        async with self._lock:
            if self.writer is not None:
                return
            self.reader, self.writer = await asyncio.open_unix_connection(self.path, limit=1 << 24)
            self._task = asyncio.ensure_future(self._read_loop())

    async def _read_loop(self):
        r = self.reader
        try:
            while True:
                hdr = await r.readexactly(_HDR.size)
                ln, typ = _HDR.unpack(hdr)
                body = await r.readexactly(ln - 1)
                if typ != T_BATCH:
                    continue
                for rec in unpack_batch(memoryview(body)):
                    q = self.queues.get(rec[0])
                    if q is not None:
                        q.put_nowait(rec)
        except (asyncio.IncompleteReadError, ConnectionError, OSError):
            pass
        finally:
            self.writer = None
            for q in list(self.queues.values()):
                q.put_nowait((0, F_FINISHED | F_ERROR, 0, 0, 0.0, 0.0, b"worker connection lost"))

    async def stream(self, opts):
        """Async generator of (flags, tokens, prompt_tokens, t_prompt_ms, t_gen_ms, data)."""
        await self._connect()
        self._rid += 1
        rid = self._rid
        q: asyncio.Queue = asyncio.Queue()
        self.queues[rid] = q
        payload = opts.SerializeToString()
        self.writer.write(_HDR.pack(len(payload) + 9, T_SUBMIT) + _U64.pack(rid) + payload)
        done = False
        try:
            while True:
                rec = await q.get()
                _, flags, tok, ptok, tp, tg, data = rec
                if flags & F_FINISHED:
                    done = True
                yield flags, tok, ptok, tp, tg, data
                if done:
                    return
        finally:
            self.queues.pop(rid, None)
            if not done and self.writer is not None:
                try:
                    self.writer.write(_HDR.pack(9, T_ABORT) + _U64.pack(rid))
                except Exception:
                    pass

    async def close(self):
        if self.writer is not None:
            self.writer.close()
        if self._task is not None:
            self._task.cancel()
