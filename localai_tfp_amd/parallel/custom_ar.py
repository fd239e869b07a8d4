"""One-shot all-reduce over hipIpc-mapped peer buffers (csrc/kernels/allreduce.hip) for the small
tensor-parallel messages of decode steps; RCCL (torch.distributed "nccl") above ``max_bytes``.

Set-up is collective over the TP group: every rank allocates an uncached receive buffer
(2 parities x world slots x max_bytes/4 granules of 8 bytes), exports its hipIpc handle as 64 raw bytes,
all-gathers the handles as a uint8 tensor (no pickles) and opens its peers' buffers. Works for ranks on
different GPUs of one node (xGMI) and for several processes sharing one GPU (the CPU-launched test).

    ar = OneShotAllReduce(group, device, max_bytes=1 << 20)
    ar(t)          # in place, t: 16-bit CUDA tensor; falls back to dist.all_reduce when too large
    ar.snapshot()  # after a step's launches: async copy of the error flag into a pinned ring + an event
    ar.check()     # raises if a completed snapshot saw a peer that never arrived (bounded spin in the kernel);
                   # never blocks on queued work (block=True waits for every snapshot: shutdown / tests)
"""
from __future__ import annotations

import ctypes as C
import os
from collections import deque

import torch

from .. import _native as N

_SIGS = {
    "mxk_ar_alloc": [C.c_size_t, C.POINTER(C.c_void_p)],
    "mxk_ar_free": [C.c_void_p],
    "mxk_ar_ipc_handle": [C.c_void_p, C.c_void_p],
    "mxk_ar_ipc_open": [C.c_void_p, C.POINTER(C.c_void_p)],
    "mxk_ar_ipc_close": [C.c_void_p],
    "mxk_ar_handle_size": [],
    "mxk_allreduce_1shot": [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_long,
                            C.c_void_p, C.c_void_p, C.c_void_p],
    "mxk_allreduce_1shot_add": [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_long,
                                C.c_void_p, C.c_void_p, C.c_void_p],
}


def _lib():
    lib = N.kernels()
    for n, a in _SIGS.items():
        f = getattr(lib, n)
        f.argtypes = a
        f.restype = C.c_int
    return lib


def _ok(rc, what):
    if rc != 0:
        raise N.NativeError(f"{what} failed: {N.HIP_ERRORS.get(rc, rc)} ({rc})")


class OneShotAllReduce:
    MAX_WORLD = 8

    def __init__(self, group, device, max_bytes: int = 1 << 20, rank: int | None = None, world: int | None = None):
        """group None with world 1: a single-rank instance (no process group, no handle exchange) — the same
        kernel over its own slot only, which the one-GPU tensor-parallel rehearsal runs where the real group's
        all-reduce + residual add would be (bench.py --tp-rehearsal)."""
        import torch.distributed as dist
        solo = group is None and world == 1
        self.group = group
        self.rank = 0 if solo else dist.get_rank(group) if rank is None else rank
        self.world = 1 if solo else dist.get_world_size(group) if world is None else world
        if self.world > self.MAX_WORLD:
            raise ValueError(f"one-shot all-reduce supports up to {self.MAX_WORLD} ranks")
        self.device = torch.device(device)
        self.max_bytes = int(max_bytes)
        self.slot = self.max_bytes // 4  # granules (2 x 16-bit elements each) per source slot
        lib = _lib()
        self.lib = lib
        with torch.cuda.device(self.device):
            self.buf = C.c_void_p()
            _ok(lib.mxk_ar_alloc(2 * self.world * self.slot * 8, C.byref(self.buf)), "mxk_ar_alloc")
            self.ptrs = (C.c_void_p * self.world)()
            self._opened = []
            if not solo:
                hs = lib.mxk_ar_handle_size()
                h = (C.c_ubyte * hs)()
                _ok(lib.mxk_ar_ipc_handle(self.buf, h), "hipIpcGetMemHandle")
                mine = torch.tensor(bytearray(h), dtype=torch.uint8)
                # the handle exchange runs on the group's backend: CPU tensors for gloo, device tensors for RCCL
                on_dev = dist.get_backend(group) == "nccl"
                src = mine.to(self.device) if on_dev else mine
                allh = [torch.empty_like(src) for _ in range(self.world)]
                dist.all_gather(allh, src, group=group)
            for p in range(self.world):
                if p == self.rank:
                    self.ptrs[p] = self.buf
                    continue
                hb = bytes(allh[p].cpu().numpy().tobytes())
                ptr = C.c_void_p()
                _ok(lib.mxk_ar_ipc_open(hb, C.byref(ptr)), "hipIpcOpenMemHandle")
                self.ptrs[p] = ptr
                self._opened.append(ptr)
            self.epoch = torch.zeros(2, dtype=torch.int32, device=self.device)  # {epoch, last-workgroup ticket}
            self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # error-flag snapshots: pinned host slots filled by async copies, each with the event that retires it
        self._err_host = torch.zeros(self.SNAP_RING, dtype=torch.int32, pin_memory=self.device.type == "cuda")
        self._snaps: deque = deque()
        self._snap_i = 0
        if not solo:
            dist.barrier(group=group)

    def __call__(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        out = t if out is None else out
        n = t.numel()
        if (t.dtype not in (torch.float16, torch.bfloat16) or n * 2 > self.max_bytes or n % 2
                or not t.is_contiguous() or not out.is_contiguous()):
            if out is not t:
                out.copy_(t)
            if self.world > 1:
                import torch.distributed as dist
                dist.all_reduce(out, group=self.group)
            return out
        N.ensure_act(t.dtype)
        _ok(self.lib.mxk_allreduce_1shot(t.data_ptr(), out.data_ptr(), n, self.rank, self.world, self.ptrs,
                                         self.slot, self.epoch.data_ptr(), self.err.data_ptr(),
                                         N.stream_ptr(self.device)), "mxk_allreduce_1shot")
        return out

    def fits(self, t: torch.Tensor) -> bool:
        return (t.dtype in (torch.float16, torch.bfloat16) and t.numel() * 2 <= self.max_bytes and t.numel() % 2 == 0
                and t.is_contiguous())

    def add_into(self, t: torch.Tensor, res: torch.Tensor):
        """res (fp32, same shape) += all-reduce(t) in one kernel (the row-parallel projection's all-reduce
        fused with the residual add); falls back to RCCL + add for large or unsupported tensors."""
        if not self.fits(t) or res.dtype != torch.float32 or not res.is_contiguous() or res.numel() != t.numel():
            self(t)
            res.add_(t)
            return res
        N.ensure_act(t.dtype)
        _ok(self.lib.mxk_allreduce_1shot_add(t.data_ptr(), res.data_ptr(), t.numel(), self.rank, self.world, self.ptrs,
                                             self.slot, self.epoch.data_ptr(), self.err.data_ptr(),
                                             N.stream_ptr(self.device)), "mxk_allreduce_1shot_add")
        return res

    SNAP_RING = 16

    def snapshot(self):
        """Queue an async copy of the error flag (behind the work launched so far) into the next pinned slot
        and record its event. Cheap enough for every step; check() reads only retired snapshots."""
        if len(self._snaps) >= self.SNAP_RING:  # ring full: retire the oldest (long retired in practice)
            self._retire(self._snaps.popleft(), block=True)
        k = self._snap_i
        self._snap_i = (k + 1) % self.SNAP_RING
        self._err_host[k:k + 1].copy_(self.err, non_blocking=True)
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        self._snaps.append((ev, k))

    def _retire(self, snap, block: bool):
        ev, k = snap
        if ev is not None:
            if block:
                ev.synchronize()
            elif not ev.query():
                return False
        if int(self._err_host[k]):
            raise RuntimeError("one-shot all-reduce: a peer never delivered its data (rank dead or desynchronised)")
        return True

    def check(self, block: bool = False):
        """Raise if any retired snapshot saw the error flag. Non-blocking by default: a snapshot whose copy is
        still queued behind running work is left for a later check (no device->host sync on the stream, so a
        check between two launched steps never serialises the overlap pipeline). block=True: snapshot now
        and wait for everything."""
        if block:
            self.snapshot()
        while self._snaps:
            if not self._retire(self._snaps[0], block):
                return
            self._snaps.popleft()

    def close(self):
        for p in self._opened:
            self.lib.mxk_ar_ipc_close(p)
        self._opened = []
        if self.buf:
            self.lib.mxk_ar_free(self.buf)
            self.buf = C.c_void_p()

    def __del__(self):
        try:
            if os.environ.get("MX_AR_NO_FREE") is None:
                self.close()
        except Exception:
            pass
