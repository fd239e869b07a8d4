"""Python faces of the native host runtime (libmxrt.so): block manager, GBNF matcher, vector store."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _native


def _rt():
    return _native.runtime()


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class NativeBlockManager:
    """Drop-in for engine.kv_cache.PyBlockManager backed by csrc/runtime/block_manager.cpp.
    Block hashes are 16-byte `bytes`."""

    def __init__(self, num_blocks: int, block_size: int, enable_prefix_cache: bool = True):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.enable_prefix_cache = enable_prefix_cache
        self._h = _rt().mxrt_bm_new(num_blocks, block_size, int(enable_prefix_cache))
        if os.environ.get("MX_KV_LIFO", "0") == "1":  # A/B: reuse released blocks first (KV locality)
            _rt().mxrt_bm_set_lifo(self._h, 1)

    def __del__(self):
        try:
            _rt().mxrt_bm_free(self._h)
        except Exception:
            pass

    @property
    def num_free(self) -> int:
        return _rt().mxrt_bm_num_free(self._h)

    def allocate(self, n: int) -> list[int]:
        out = np.empty(max(n, 1), np.int32)
        if _rt().mxrt_bm_allocate(self._h, n, _ptr(out)) != 0:
            raise MemoryError("KV cache exhausted")
        return out[:n].tolist()

    def release(self, blocks) -> None:
        a = np.asarray(blocks, np.int32)
        if a.size:
            _rt().mxrt_bm_release(self._h, _ptr(a), a.size)

    def match_prefix(self, tokens):
        t = np.asarray(tokens, np.int32)
        n = t.size
        if n == 0:
            return [], []
        cap = max(1, (n - 1) // self.block_size)
        blocks = np.empty(cap, np.int32)
        hashes = np.empty(2 * cap, np.uint64)
        k = _rt().mxrt_bm_match_prefix(self._h, _ptr(t), n, _ptr(blocks), _ptr(hashes))
        return blocks[:k].tolist(), [hashes[2 * i:2 * i + 2].tobytes() for i in range(k)]

    def commit_full_block(self, block: int, parent: bytes, tokens) -> bytes:
        t = np.asarray(tokens, np.int32)
        out = np.empty(2, np.uint64)
        if parent:
            p = np.frombuffer(parent, np.uint64).copy()
            _rt().mxrt_bm_commit(self._h, block, _ptr(p), _ptr(t), _ptr(out))
        else:
            _rt().mxrt_bm_commit(self._h, block, None, _ptr(t), _ptr(out))
        return out.tobytes()

    def stats(self) -> dict:
        o = np.zeros(4, np.int64)
        _rt().mxrt_bm_stats(self._h, _ptr(o))
        return {"hits": int(o[0]), "queries": int(o[1]), "cached_blocks": int(o[2]), "free": int(o[3])}

    @property
    def hits(self):
        return self.stats()["hits"]

    @property
    def queries(self):
        return self.stats()["queries"]

    def usage(self) -> float:
        return 1.0 - self.num_free / max(1, self.num_blocks - 1)


class GrammarError(ValueError):
    pass


class NativeGrammar:
    def __init__(self, gbnf: str):
        err = C.create_string_buffer(512)
        self._h = _rt().mxrt_grammar_parse(gbnf.encode("utf-8"), err, 512)
        if not self._h:
            raise GrammarError(err.value.decode(errors="replace"))

    def __del__(self):
        try:
            _rt().mxrt_grammar_free(self._h)
        except Exception:
            pass


class NativeVocab:
    """Byte strings of every token id, as a trie for grammar masking."""

    def __init__(self, token_bytes: list[bytes]):
        self.n = len(token_bytes)
        offs = np.zeros(self.n + 1, np.int64)
        offs[1:] = np.cumsum([len(b) for b in token_bytes])
        buf = np.frombuffer(b"".join(token_bytes) or b"\0", np.uint8).copy()
        self._keep = (buf, offs)
        self._h = _rt().mxrt_vocab_new(_ptr(buf), _ptr(offs), self.n)

    def __del__(self):
        try:
            _rt().mxrt_vocab_free(self._h)
        except Exception:
            pass


class GrammarMatcher:
    """Per-sequence constrained-decoding state used by the engine (engine.py: allowed_mask /
    accept / is_done)."""

    def __init__(self, grammar: NativeGrammar, vocab: NativeVocab, token_bytes, eos_id: int = -1):
        self.g, self.v, self.tb, self.eos = grammar, vocab, token_bytes, eos_id
        self._h = _rt().mxrt_matcher_new(grammar._h)

    def __del__(self):
        try:
            _rt().mxrt_matcher_free(self._h)
        except Exception:
            pass

    def accept(self, token_id: int) -> bool:
        if token_id == self.eos:
            return True
        b = self.tb[token_id]
        if not b:
            return False
        buf = C.create_string_buffer(b, len(b))
        return bool(_rt().mxrt_matcher_accept(self._h, buf, len(b)))

    def accept_bytes(self, b: bytes) -> bool:
        buf = C.create_string_buffer(b, len(b))
        return bool(_rt().mxrt_matcher_accept(self._h, buf, len(b)))

    def is_done(self) -> bool:
        return bool(_rt().mxrt_matcher_is_done(self._h))

    def allowed_mask(self, V: int) -> np.ndarray:
        words = (V + 31) // 32
        m = np.zeros(words, np.uint32)
        _rt().mxrt_matcher_mask(self._h, self.v._h, _ptr(m), self.eos)
        return m

    # rows of a batched mask computed in parallel (a GPU box's CPU share is 16; os.cpu_count() there reports
    # the whole machine)
    MASK_THREADS = int(os.environ.get("MX_GRAMMAR_THREADS", str(min(16, max(2, (os.cpu_count() or 4) // 2)))))

    @staticmethod
    def masks_into(matchers: list, out: np.ndarray, rows: list[int]):
        """Masks of several matchers sharing one vocabulary and EOS id into out[rows[i]] ([R, words] uint32),
        computed on up to MASK_THREADS threads in one native call (libmxrt mxrt_matcher_mask_batch)."""
        if not matchers:
            return
        m0 = matchers[0]
        hs = (C.c_void_p * len(matchers))(*[m._h for m in matchers])
        tmp = np.zeros((len(matchers), out.shape[1]), np.uint32)
        _rt().mxrt_matcher_mask_batch(hs, len(matchers), m0.v._h, _ptr(tmp), out.shape[1], m0.eos,
                                      GrammarMatcher.MASK_THREADS)
        out[rows] = tmp


class NativeStore:
    def __init__(self):
        self._h = _rt().mxrt_store_new()

    def __del__(self):
        try:
            _rt().mxrt_store_free(self._h)
        except Exception:
            pass

    def __len__(self):
        return int(_rt().mxrt_store_size(self._h))

    @property
    def dim(self):
        return _rt().mxrt_store_dim(self._h)

    def set(self, keys, values: list[bytes]):
        k = np.ascontiguousarray(keys, np.float32)
        if k.ndim == 1:
            k = k[None]
        offs = np.zeros(len(values) + 1, np.int64)
        offs[1:] = np.cumsum([len(v) for v in values])
        buf = np.frombuffer(b"".join(values) or b"\0", np.uint8).copy()
        if _rt().mxrt_store_set(self._h, _ptr(k), k.shape[0], k.shape[1], _ptr(buf), _ptr(offs)) != 0:
            raise ValueError(f"key dimension {k.shape[1]} does not match store dimension {self.dim}")

    def delete(self, keys) -> int:
        k = np.ascontiguousarray(keys, np.float32)
        if k.ndim == 1:
            k = k[None]
        return int(_rt().mxrt_store_delete(self._h, _ptr(k), k.shape[0], k.shape[1]))

    def _row(self, r: int):
        dim = self.dim
        key = np.empty(dim, np.float32)
        n = _rt().mxrt_store_row(self._h, r, _ptr(key), None, 0)
        buf = np.empty(max(n, 1), np.uint8)
        _rt().mxrt_store_row(self._h, r, None, _ptr(buf), n)
        return key, buf[:n].tobytes()

    def get(self, keys):
        k = np.ascontiguousarray(keys, np.float32)
        if k.ndim == 1:
            k = k[None]
        rows = np.empty(k.shape[0], np.int64)
        _rt().mxrt_store_lookup(self._h, _ptr(k), k.shape[0], k.shape[1], _ptr(rows))
        out_k, out_v = [], []
        for r in rows:
            if r >= 0:
                kk, vv = self._row(int(r))
                out_k.append(kk)
                out_v.append(vv)
        return out_k, out_v

    def find(self, key, topk: int):
        q = np.ascontiguousarray(key, np.float32)
        rows = np.empty(max(topk, 1), np.int64)
        sims = np.empty(max(topk, 1), np.float32)
        n = int(_rt().mxrt_store_find(self._h, _ptr(q), q.size, topk, _ptr(rows), _ptr(sims)))
        ks, vs = [], []
        for r in rows[:n]:
            kk, vv = self._row(int(r))
            ks.append(kk)
            vs.append(vv)
        return ks, vs, sims[:n].tolist()
