"""Single-node leader -> followers message ring in POSIX shared memory (/dev/shm) for tensor-parallel
step plans.

All ranks of a TP group live on one MI355X node, so a step plan (a few KB of int32: tokens, positions,
KV slots, block tables) does not need a socket: the leader writes it into a slot of a ring in shared
memory and bumps the slot's sequence number; every follower spins on the sequence of the next slot it
expects, copies the body out and publishes its read position. x86-64 stores are seen in program order
(TSO), so a follower that observes the new sequence also observes the body written before it.

    [header 4 KB: magic, nslot, slot_bytes, world, leader heartbeat (ns), ack[rank] (last seq read)]
    [slot i: seq u64 | kind i32 | nbytes i32 | body ...] x nslot

Back-pressure: the leader reuses slot s only when every follower's ack >= seq - nslot. Liveness: the
leader stamps a heartbeat every period from a thread; a follower that has waited `timeout` with a stale
heartbeat declares the leader dead, and the leader declares a follower dead when the ring stays full
for `timeout`. Either side raises ChannelDead (TPLink turns it into a non-zero exit).

Replaces the per-step gloo TCP broadcast of round 2 (parallel/tp_engine.py), whose two collectives per
plan cost ~0.1-0.3 ms of host time on every rank every step.
"""
from __future__ import annotations

import os
import threading
import time
from multiprocessing import shared_memory

import numpy as np

MAGIC = 0x4D58534852494E47  # "MXSHRING"
HDR = 4096
_U64 = np.dtype("<u8")


class ChannelDead(RuntimeError):
    pass


class ShmChannel:
    def __init__(self, name: str, rank: int, world: int, create: bool, nslot: int = 16, slot_bytes: int = 1 << 20,
                 timeout: float = 600.0, heartbeat: float = 1.0):
        self.name, self.rank, self.world = name, rank, world
        self.timeout, self.heartbeat = float(timeout), float(heartbeat)
        size = HDR + nslot * slot_bytes
        if create:
            try:  # a stale segment of a crashed run with the same name
                old = shared_memory.SharedMemory(name=name)
                old.close()
                old.unlink()
            except FileNotFoundError:
                pass
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=size)
            hdr = np.ndarray(8, _U64, self.shm.buf, 0)
            hdr[1], hdr[2], hdr[3] = nslot, slot_bytes, world
            hdr[4] = time.monotonic_ns()
            hdr[5] = os.getpid()
            np.ndarray(64, _U64, self.shm.buf, 64)[:] = 0
            hdr[0] = MAGIC
        else:
            t0 = time.monotonic()
            while True:
                try:
                    self.shm = shared_memory.SharedMemory(name=name)
                    if int(np.ndarray(1, _U64, self.shm.buf, 0)[0]) == MAGIC:
                        break
                    self.shm.close()
                except FileNotFoundError:
                    pass
                if time.monotonic() - t0 > timeout:
                    raise ChannelDead(f"shared-memory channel {name} never appeared")
                time.sleep(0.01)
            try:  # the leader owns the segment's lifetime; followers must not unlink it at exit
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, "shared_memory")  # noqa: SLF001
            except Exception:
                pass
        self.hdr = np.ndarray(8, _U64, self.shm.buf, 0)
        self.nslot, self.slot_bytes = int(self.hdr[1]), int(self.hdr[2])
        self.acks = np.ndarray(64, _U64, self.shm.buf, 64)  # [0, 32): read positions, [32, 64): pids
        if not create:
            self.acks[32 + rank] = os.getpid()
        self._seq = 0  # leader: last written; follower: last read
        self._hb = None
        self.is_leader = create
        if create and heartbeat > 0:
            self._hb_stop = threading.Event()
            self._hb = threading.Thread(target=self._beat, daemon=True, name="shm-heartbeat")
            self._hb.start()

    # ---------------------------------------------------------------- leader
    def _beat(self):
        while not self._hb_stop.wait(self.heartbeat):
            self.hdr[4] = time.monotonic_ns()

    def _slot(self, seq: int):
        off = HDR + (seq % self.nslot) * self.slot_bytes
        return np.ndarray(2, _U64, self.shm.buf, off), off + 16

    def max_body(self) -> int:
        return self.slot_bytes - 16

    def send(self, kind: int, body: np.ndarray | bytes | None = None):
        raw = b"" if body is None else (body.tobytes() if isinstance(body, np.ndarray) else bytes(body))
        if len(raw) > self.max_body():
            raise ValueError(f"message of {len(raw)} B exceeds the slot size {self.max_body()} B")
        seq = self._seq + 1
        # back-pressure: the slot's previous message (seq - nslot) must have been read by every follower
        need = seq - self.nslot
        if need > 0:
            t0 = time.monotonic()
            spins = 0
            while min(int(self.acks[r]) for r in range(1, self.world)) < need:
                spins += 1
                if spins > 200:
                    time.sleep(20e-6)
                    if spins % 5000 == 0:
                        for r in range(1, self.world):
                            if int(self.acks[r]) < need and not _alive(int(self.acks[32 + r])):
                                raise ChannelDead(f"tensor-parallel follower rank {r} exited")
                    if time.monotonic() - t0 > self.timeout:
                        raise ChannelDead("a tensor-parallel follower stopped reading plans")
        meta, boff = self._slot(seq)
        self.shm.buf[boff:boff + len(raw)] = raw
        meta[1] = (len(raw) << 32) | (kind & 0xFFFFFFFF)
        meta[0] = seq  # publish last (x86-64 TSO: the body is visible first)
        self.hdr[4] = time.monotonic_ns()
        self._seq = seq

    # ---------------------------------------------------------------- follower
    def recv(self) -> tuple[int, bytes]:
        seq = self._seq + 1
        meta, boff = self._slot(seq)
        spins = 0
        t_wait = None
        while int(meta[0]) != seq:
            spins += 1
            if spins > 2000:  # ~a few hundred us of hot spinning, then yield the core in short naps
                time.sleep(20e-6 if spins < 20000 else 200e-6)
                now = time.monotonic()
                if spins % 2000 == 0 and not _alive(int(self.hdr[5])):
                    raise ChannelDead("tensor-parallel leader exited")
                if t_wait is None:
                    t_wait = now
                elif now - t_wait > self.timeout:
                    stale = (time.monotonic_ns() - int(self.hdr[4])) / 1e9
                    if stale > self.timeout:
                        raise ChannelDead(f"tensor-parallel leader silent for {stale:.0f} s")
                    t_wait = now
        info = int(meta[1])
        kind, n = info & 0xFFFFFFFF, info >> 32
        body = bytes(self.shm.buf[boff:boff + n])
        self.acks[self.rank] = seq
        self._seq = seq
        return kind, body

    def close(self, unlink: bool | None = None):
        if self._hb is not None:
            self._hb_stop.set()
        for a in ("hdr", "acks"):
            setattr(self, a, None)
        try:
            self.shm.close()
            if self.is_leader if unlink is None else unlink:
                self.shm.unlink()
        except Exception:
            pass


def _alive(pid: int) -> bool:
    if pid <= 0:
        return True  # not registered yet
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:  # a zombie (exited, not yet reaped) counts as dead
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except OSError:
        return True


def channel_name(tag: str) -> str:
    return f"mx_tp_{os.getuid()}_{tag}"
