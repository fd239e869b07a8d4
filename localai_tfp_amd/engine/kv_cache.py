"""Paged KV cache + block manager with automatic prefix caching.

Replaces the reference's static per-slot context split (`n_ctx_slot = n_ctx / n_parallel`,
grpc-server.cpp:572) and its per-slot `cache_prompt` prefix reuse (`common_part`,
grpc-server.cpp:1826-1870) with a shared pool of fixed-size blocks:

* storage: one bf16 tensor per layer for K and for V, shape [num_blocks, Hkv, block_size, D],
  sized from free HBM (288 GB per MI355X -> millions of cached tokens for an 8B model);
* allocation: free list + per-block refcounts; a sequence owns a block table;
* prefix cache: every FULL block is keyed by hash(parent_hash, its tokens); a new request walks its
  prompt block by block and re-uses any cached block (refcount++), so shared system prompts /
  multi-turn chats skip their prefill. Unreferenced cached blocks are evicted LRU on demand.

The bookkeeping is in the native runtime (csrc/runtime/block_manager.cpp via libmxrt) when it is
built, with an identical pure-Python fallback used by CPU-only environments.
"""
from __future__ import annotations

import collections
import hashlib
import struct

import torch


class KVCache:
    """Paged K / V caches [n_layers, num_blocks, n_kv, block_size, head_dim] in bf16 / fp8, or, for the llama.cpp
    block formats (kvf >= 2, ops/kvq.py), uint8 rows [.., block_size, row_bytes] of the quantised head vectors."""

    def __init__(self, n_layers: int, num_blocks: int, n_kv: int, block_size: int, head_dim: int, device,
                 dtype=torch.bfloat16, kvf: int = 0):
        self.n_layers, self.num_blocks, self.block_size = n_layers, num_blocks, block_size
        self.n_kv, self.head_dim = n_kv, head_dim
        self.kvf = kvf
        if kvf >= 2:
            from ..ops.kvq import row_bytes
            shape = (n_layers, num_blocks, n_kv, block_size, row_bytes(kvf, head_dim))
            dtype = torch.uint8
        else:
            shape = (n_layers, num_blocks, n_kv, block_size, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)

    def layer(self, i: int):
        k, v = self.k[i], self.v[i]
        if self.kvf >= 2:
            k.kvf = v.kvf = self.kvf
        return k, v

    @staticmethod
    def bytes_per_block(n_layers, n_kv, block_size, head_dim, dtype_bytes=2):
        return int(2 * n_layers * n_kv * block_size * head_dim * dtype_bytes)

    @classmethod
    def auto_num_blocks(cls, n_layers, n_kv, block_size, head_dim, device, fraction: float = 0.85,
                        reserve_bytes: int = 4 << 30, cap: int | None = None, dtype_bytes: int = 2):
        dev = torch.device(device)
        per = cls.bytes_per_block(n_layers, n_kv, block_size, head_dim, dtype_bytes)
        if dev.type != "cuda":
            n = 4096
        else:
            free, _total = torch.cuda.mem_get_info(dev)
            n = int(max(0, free * fraction - reserve_bytes) // per)
        if cap:
            n = min(n, cap)
        return max(n, 16)


def _block_hash(parent: bytes, tokens) -> bytes:
    h = hashlib.blake2b(parent, digest_size=16)
    h.update(struct.pack(f"<{len(tokens)}i", *tokens))
    return h.digest()


class PyBlockManager:
    """Pure-Python block manager (same semantics as the native one)."""

    def __init__(self, num_blocks: int, block_size: int, enable_prefix_cache: bool = True):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.enable_prefix_cache = enable_prefix_cache
        # block 0 is reserved as the dummy target of padded rows (graph padding / masked reads)
        self.free = collections.deque(range(1, num_blocks))
        self.ref = [0] * num_blocks
        self.hash_of: dict[int, bytes] = {}
        self.cached: dict[bytes, int] = {}
        self.evictable: collections.OrderedDict[int, None] = collections.OrderedDict()
        self.hits = 0
        self.queries = 0

    @property
    def num_free(self) -> int:
        return len(self.free) + len(self.evictable)

    def _take(self) -> int:
        if self.free:
            return self.free.popleft()
        if self.evictable:
            b, _ = self.evictable.popitem(last=False)
            h = self.hash_of.pop(b, None)
            if h is not None and self.cached.get(h) == b:
                del self.cached[h]
            return b
        raise MemoryError("KV cache exhausted")

    def allocate(self, n: int) -> list[int]:
        if n > self.num_free:
            raise MemoryError("KV cache exhausted")
        out = []
        for _ in range(n):
            b = self._take()
            self.ref[b] = 1
            out.append(b)
        return out

    def release(self, blocks) -> None:
        for b in blocks:
            self.ref[b] -= 1
            if self.ref[b] == 0:
                if b in self.hash_of and self.enable_prefix_cache:
                    self.evictable[b] = None
                else:
                    self.hash_of.pop(b, None)
                    self.free.append(b)

    def match_prefix(self, tokens) -> tuple[list[int], list[bytes]]:
        """Longest run of cached full blocks for `tokens` (never the whole prompt: at least one
        token is left to compute so the step produces logits). Returns (blocks, their hashes)."""
        self.queries += 1
        out: list[int] = []
        hashes: list[bytes] = []
        parent = b""
        if not self.enable_prefix_cache or not len(tokens):
            return out, hashes
        bs = self.block_size
        nfull = (len(tokens) - 1) // bs
        for i in range(nfull):
            h = _block_hash(parent, tokens[i * bs:(i + 1) * bs])
            b = self.cached.get(h)
            if b is None:
                break
            if self.ref[b] == 0:
                self.evictable.pop(b, None)
            self.ref[b] += 1
            out.append(b)
            hashes.append(h)
            parent = h
        if out:
            self.hits += 1
        return out, hashes

    def commit_full_block(self, block: int, parent: bytes, tokens) -> bytes:
        h = _block_hash(parent, tokens)
        if self.enable_prefix_cache and h not in self.cached:
            self.cached[h] = block
            self.hash_of[block] = h
        return h

    def usage(self) -> float:
        return 1.0 - self.num_free / max(1, self.num_blocks - 1)


def make_block_manager(num_blocks: int, block_size: int, enable_prefix_cache: bool = True):
    try:
        from ..runtime_native import NativeBlockManager
        return NativeBlockManager(num_blocks, block_size, enable_prefix_cache)
    except Exception:
        return PyBlockManager(num_blocks, block_size, enable_prefix_cache)
