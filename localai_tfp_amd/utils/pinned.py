"""Pinned host staging ring whose slots are recycled only after the device has consumed them.

Every host->device input of an engine step (plan arrays, graph input images, sampler parameters)
goes through one async copy from a page-locked buffer. A slot of the ring may be rewritten only
when the copy that last sourced it has executed on the stream: each `stage()` records an event
after its copy and the next use of that slot waits for that event (normally long signalled, so
the wait is free). Tying reuse to "the step was read back" is not enough: steps that sample no
rows (prefill-only chunks, tensor-parallel followers) are never read back, and a long prompt
queued as several chunks would otherwise overwrite a slot before its copy ran.
"""
from __future__ import annotations

import numpy as np
import torch


class PinnedRing:
    def __init__(self, n_slots: int, nbytes: int, device):
        self.device = torch.device(device)
        self.n = max(2, int(n_slots))
        self.cap = 0
        self._buf: list[torch.Tensor] = []
        self._ev: list = []
        self._k = 0
        self._grow(int(nbytes))

    def _grow(self, nbytes: int):
        if self._buf:
            # the old buffers may still source in-flight copies
            for e in self._ev:
                if e is not None:
                    e.synchronize()
        self.cap = max(nbytes, 1)
        pin = self.device.type == "cuda"
        self._buf = [torch.empty(self.cap, dtype=torch.uint8, pin_memory=pin) for _ in range(self.n)]
        self._ev = [None] * self.n
        self._k = 0

    def acquire(self, nbytes: int) -> tuple[int, torch.Tensor]:
        """Next slot (waiting for the copy that last read it), as a uint8 host tensor of nbytes."""
        if nbytes > self.cap:
            self._grow(max(nbytes, 2 * self.cap))
        k = self._k
        self._k = (k + 1) % self.n
        e = self._ev[k]
        if e is not None:
            e.synchronize()
            self._ev[k] = None
        return k, self._buf[k][:nbytes]

    def release(self, k: int):
        """Mark slot k as read by the copies just enqueued on the current stream."""
        if self.device.type == "cuda":
            e = torch.cuda.Event()
            e.record()
            self._ev[k] = e

    def stage(self, flat: np.ndarray, dst: torch.Tensor | None = None) -> torch.Tensor:
        """Copy a host array to the device through one slot; returns the device tensor (a view of
        `dst` when given, else a fresh allocation of the same dtype)."""
        flat = np.ascontiguousarray(flat)
        raw = flat.view(np.uint8).reshape(-1)
        k, hb = self.acquire(raw.size)
        hb.numpy()[:] = raw
        src = hb.view(torch.from_numpy(flat[:0]).dtype) if flat.dtype != np.uint8 else hb
        if dst is None:
            out = src.to(self.device, non_blocking=True) if self.device.type == "cuda" else src.clone()
        else:
            dst.copy_(src, non_blocking=True)
            out = dst
        self.release(k)
        return out
