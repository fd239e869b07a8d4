"""Tensor parallelism for the LLM worker: one process per GPU, RCCL (torch.distributed "nccl")
over xGMI.

Sharding (Megatron-style, as vLLM does inside the reference's python backend,
backend/python/vllm/backend.py:106-107 `tensor_parallel_size`):
  * column-parallel: Q/K/V by heads (KV heads replicated when Hkv < world), gate/up by FFN columns;
  * row-parallel: o_proj and down_proj by input columns, in whole 256-element super-blocks so the
    quantised bytes split without re-quantisation;
  * the residual stream is replicated; each row-parallel projection writes this rank's partial sum
    in 16 bits (the GEMM epilogue's activation format) and ONE all-reduce of it per projection (2 per
    layer; message = tokens x hidden x 2 B, half of an fp32 residual all-reduce) is added to h;
  * MoE layers are expert-parallel (whole experts per rank, models/llama.py load_moe) and the LM head
    vocab-parallel (rows of the vocabulary per rank, logits all-gathered): no rank holds the full head.
"""
from __future__ import annotations

import numpy as np
import torch

from ..formats.gguf import BLOCK, QType


def shard_rows(raw: np.ndarray, lo: int, hi: int) -> np.ndarray:
    return np.ascontiguousarray(raw[lo:hi])


def shard_raw(raw: np.ndarray, qtype: int, N: int, K: int, split, rank: int, size: int, cfg):
    """Returns (raw_shard [N', bytes_per_row'], N', K')."""
    kind = split[0]
    if kind == "col_heads":
        n_heads, hd = split[1], split[2]
        if n_heads >= size:
            assert n_heads % size == 0, f"{n_heads} heads not divisible by tp={size}"
            per = n_heads // size
            lo, hi = rank * per * hd, (rank + 1) * per * hd
        else:  # replicate kv heads: rank r uses head r * n_heads // size
            h = rank * n_heads // size
            lo, hi = h * hd, (h + 1) * hd
        return shard_rows(raw, lo, hi), hi - lo, K
    if kind == "col":
        assert N % size == 0
        per = N // size
        return shard_rows(raw, rank * per, (rank + 1) * per), per, K
    if kind == "row":
        be, bb = BLOCK[QType(qtype)]
        assert K % size == 0
        kper = K // size
        if be > 1:
            assert kper % be == 0, f"row split {kper} not a multiple of block {be}"
        bytes_per_row = raw.shape[1]
        bper = bytes_per_row // size
        return np.ascontiguousarray(raw[:, rank * bper:(rank + 1) * bper]), N, kper
    raise ValueError(kind)


def shard_vec(v: torch.Tensor, n: int, rank: int, size: int) -> torch.Tensor:
    per = n // size
    return v[rank * per:(rank + 1) * per].contiguous()


def all_reduce_(t: torch.Tensor, group=None):
    """In-place sum over the TP group. Without an initialised process group (a single-process rehearsal of
    one rank's shard, bench.py --tp-rehearsal) the collective is a no-op: the shard's compute runs at full
    size, the communication is left out and reported separately."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return t
    dist.all_reduce(t, group=group)
    return t
