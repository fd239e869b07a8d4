"""Llama-family decoder (llama / llama3 / mistral / qwen2 / tinyllama ...) on the MI355X kernels.

This is the compute graph llama.cpp builds inside `llama_decode` for the reference worker
(grpc-server.cpp:2002), re-expressed as a fixed sequence of fused HIP kernels per layer:

    rmsnorm(h) -> {bf16 | q8}            (norm.hip)
    QKV  = x W_qkv^T  -> fp32            (qgemm.hip, fused Q|K|V weight, split-K atomics)
    rope + KV append (paged)             (rope_kv.hip)
    attention: decode rows | prefill rows (attention.hip, paged GQA)
    h += attn W_o^T                       (qgemm.hip EPI_ADD_F32 straight into the residual)
    rmsnorm(h)
    act = silu(x W_g^T) * (x W_u^T)       (qgemm.hip EPI_SWIGLU on 16-row interleaved gate|up)
    h += act W_d^T
    logits = rmsnorm(h[last]) W_out^T     (only rows that need sampling)

Gemma 2/3 (llama.cpp build_gemma2 / build_gemma3) reuse the same graph with: GeGLU (EPI_GEGLU),
post-attention / post-FFN RMSNorm fused into the residual add (norm.hip mxk_rmsnorm_add),
per-layer sliding-window attention (the kernels skip keys outside the window), attention and
final-logit soft-capping, Gemma 3's per-head QK-norm and local RoPE base on the windowed layers.

Decode batches of <= 4 tokens take the int8-dot GEMV path (norm kernels emit q8 directly);
larger batches the dequant-MFMA path. Tensor parallelism (parallel/tp.py) shards heads / FFN
columns, all-reduces the row-parallel projections' 16-bit partial sums into the replicated residual,
runs MoE layers expert-parallel and the LM head vocab-parallel.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import _native as N
from ..formats.gguf import QType
from ..ops import core as K
from ..ops import quant as Q
from ..ops.linear import (ACT_DTYPE, EPI_ADD_F32, EPI_BF16, EPI_F32, EPI_GEGLU, EPI_SWIGLU, QWeight, concat_rows,
                          _fp32_out_ok, dense_min_m, interleave_gate_up, glu_interleaved, qmatmul, qmv_fusable, qmv_rope_ok,
                          qmv_fused, qmv_rope_fused, NormFuse, norm_fusable)
from ..ops import linear as _LIN
from ..ops import autotune as _AT
from ..ops.moe import MoEWeights, moe_ffn
from . import lora_runtime as LR
from .config import LlamaConfig

GEMV_MAX_M = 4
# decode-attention partition length at >= 64 sequences (B x Hkv workgroups already fill the chip; longer
# partitions mean fewer split-K partials to merge; c128 14278 vs 14151 tok/s at 256, within run-to-run noise:
# profiles/r2_decode_part_c128_p{256,512}.json)
DECODE_PART_LARGE_B = int(__import__("os").environ.get("MX_DECODE_PART_LARGE_B", "512"))
DECODE_PART_SMALL_B = int(__import__("os").environ.get("MX_DECODE_PART_SMALL_B", "512"))  # < 8 sequences: 16-wave single-pass
# (batch 1: 64 -> 450, 256 -> 448, 512 -> 431 tok/s, profiles/r2_decode_part_c1_p*.json)
# decode batches up to this size run the RMSNorm / q8 quantisation inside the GEMV prologue (qmv.hip
# SRC_NORM / SRC_ACT). Every workgroup of the GEMV redoes the row statistics, so the fusion pays only at
# batch 1 (profiles/r2_qmv_fuse_fuse{0,1}_c{1,4}.json: c1 387 -> 442 tok/s, c4 961 -> 861)
QMV_FUSE_MAX_M = int(__import__("os").environ.get("MX_QMV_FUSE_MAX_M", "1"))


def vocab_shard(V: int, tp: int) -> int:
    """Rows of the vocab-parallel LM head per rank (whole 32-row t32 groups; the tail is zero-padded)."""
    return -(-V // (tp * 32)) * 32


@dataclass
class LlamaLayer:
    attn_norm: torch.Tensor
    ffn_norm: torch.Tensor
    qkv_parts: list  # [QWeight] Q|K|V fused where the quant types agree (Q4_K_M: v may be Q6_K)
    bqkv: torch.Tensor | None
    wo: QWeight
    wgu: QWeight | None  # interleaved gate|up
    wg: QWeight | None
    wu: QWeight | None
    wd: QWeight | None
    moe: "MoEWeights | None" = None
    q_norm: torch.Tensor | None = None  # [head_dim] fp32 (Qwen3 per-head q/k RMSNorm)
    k_norm: torch.Tensor | None = None
    post_attn_norm: torch.Tensor | None = None  # [hidden] fp32 (Gemma 2/3)
    post_ffn_norm: torch.Tensor | None = None
    window: int = 0  # sliding-window attention (0 = full)
    rope: tuple | None = None  # (inv_freq, attn_factor) of windowed layers with their own RoPE base
    qkv_dense: torch.Tensor | None = None  # dense 16-bit Q|K|V (large-M path) when the parts' quant types differ
    lora: "object | None" = None  # runtime LoRA of this layer (models/lora_runtime.LayerLora)


@dataclass
class ForwardBatch:
    """Flattened scheduler step. Decode tokens (one per sequence) come first, then prefill chunks."""
    tokens: torch.Tensor  # int32 [T]
    positions: torch.Tensor  # int32 [T]
    slots: torch.Tensor  # int32 [T] flat cache slot (-1 = don't store)
    logits_idx: torch.Tensor  # int32 [S_out] rows of T whose logits are needed
    n_decode: int = 0
    dec_block_tables: torch.Tensor | None = None  # [n_decode, maxb]
    dec_seq_lens: torch.Tensor | None = None  # [n_decode] context length incl. the new token
    dec_max_len: int = 0
    pf_block_tables: torch.Tensor | None = None  # [S_p, maxb]
    pf_cu_q: torch.Tensor | None = None  # [S_p + 1] offsets relative to the first prefill token
    pf_ctx_lens: torch.Tensor | None = None  # [S_p]
    pf_q_lens_host: list = field(default_factory=list)
    pf_ctx_lens_host: list = field(default_factory=list)
    pf_tiles: tuple | None = None  # (seq int32 [n], q0 int32 [n]) prefill attention tiles (seq -1 = skip)
    want_hidden: bool = False  # embeddings: return normalised hidden rows instead of logits
    keep_hidden: bool = False  # also stash the final-normed hidden rows in model.last_hidden
    tp_local_logits: bool = False  # tensor parallel: return this rank's vocabulary shard (no all-gather)
    stop_layer: int | None = None  # return the fp32 residual rows after this many layers (HF hidden_states[k])
    embed_rows: list | None = None  # [(row, fp32 [n, hidden])] input embeddings replacing token rows

    @property
    def T(self) -> int:
        return int(self.tokens.shape[0])


class Workspace:
    """Per-engine scratch buffers sized for the largest step; forward() only takes views, so the
    same storage is reused step to step and hipGraph capture sees static addresses."""

    def __init__(self, cfg: LlamaConfig, max_tokens: int, max_seqs: int, device, tp_size: int = 1,
                 max_parts: int = 64):
        dev = torch.device(device)
        H, F = cfg.hidden, cfg.ffn // tp_size
        qd, kvd = cfg.q_dim // tp_size, cfg.kv_dim // tp_size
        T = max_tokens
        self.max_tokens, self.max_seqs = T, max_seqs
        self.h = torch.empty((T, H), dtype=torch.float32, device=dev)
        act = ACT_DTYPE  # 16-bit GEMM operands (f16 by default, ops/linear.py)
        self.xb = torch.empty((T, max(H, F, qd)), dtype=act, device=dev)
        kmax = max(H, F, qd)
        self.xq = torch.empty((T * kmax,), dtype=torch.int8, device=dev)
        self.xds = torch.empty((T * kmax // 32 * 2,), dtype=torch.float32, device=dev)
        # zero-initialised and kept zero between uses: rope_kv re-zeroes the rows it consumes, so the
        # split-K QKV GEMM (atomic accumulate) never needs a separate fill launch
        self.qkv = torch.zeros((T, qd + 2 * kvd), dtype=torch.float32, device=dev)
        # split-K workspace of the batch-1 qkv GEMV with the RoPE epilogue (ops/linear.py qmv_rope_fused): zeroed,
        # and re-zeroed by the kernel after every use
        self.sk_ws = torch.zeros(qd + 2 * kvd, dtype=torch.float32, device=dev)
        self.sk_cnt = torch.zeros(-(-(qd + 2 * kvd) // 32), dtype=torch.int32, device=dev)
        self.q = torch.empty((T, qd), dtype=torch.bfloat16, device=dev)
        self.attn = torch.empty((T, qd), dtype=act, device=dev)
        self.act = torch.empty((T, F), dtype=act, device=dev)
        self.act2 = torch.empty((T, F), dtype=act, device=dev) if dev.type == "cpu" else None
        self.hs = torch.empty((max_seqs, H), dtype=torch.float32, device=dev)
        # projection output before the post-norm (Gemma 2/3)
        self.y = torch.empty((T, H), dtype=torch.float32, device=dev) if cfg.post_norms else None
        self.logits = torch.empty((max_seqs, cfg.vocab), dtype=torch.float32, device=dev)
        if tp_size > 1:
            # row-parallel partial projections, all-reduced in 16 bits (fp32 on the CPU oracle path)
            self.y16 = torch.empty((T, H), dtype=act if dev.type == "cuda" else torch.float32, device=dev)
            # vocab-parallel LM head: this rank's logits, then the all-gathered [tp, S, V/tp] block
            vl = vocab_shard(cfg.vocab, tp_size)
            self.logits_local = torch.empty((max_seqs, vl), dtype=torch.float32, device=dev)
            self.logits_gather = torch.empty((tp_size, max_seqs, vl), dtype=torch.float32, device=dev)
            # vocab-parallel greedy head: one 64-bit (value, index) key per row and rank
            self.am_keys = torch.empty(max_seqs, dtype=torch.int64, device=dev)
            self.am_keys_all = torch.empty(tp_size * max_seqs, dtype=torch.int64, device=dev)
            self.moe_y = torch.empty((T, H), dtype=torch.float32, device=dev) if cfg.n_expert else None
        nh = cfg.n_heads // tp_size
        self.part_ml = torch.empty((max_seqs * nh * max_parts, 2), dtype=torch.float32, device=dev)
        self.part_o = torch.empty((max_seqs * nh * max_parts, cfg.head_dim), dtype=torch.float32, device=dev)
        # per-(sequence, kv head) arrival counters of the decode kernel's fused partition merge (self-resetting)
        self.part_cnt = torch.zeros(max_seqs * max(1, cfg.n_kv_heads // tp_size), dtype=torch.int32, device=dev)
        # RMSNorm split across the GEMMs at M > 4 (ops/linear.py NormFuse): per-row sums of squares (one 128-byte line
        # per row) in two buffers that alternate between producers, and the producers' per-block split tickets; both
        # are zero between uses (each producer re-zeroes the buffer the previous consumer read, tickets self-reset)
        self.norm_ss = torch.zeros((2, T, 32), dtype=torch.float32, device=dev)
        self.norm_tick = torch.zeros(-(-T // 32) * -(-max(H, qd + 2 * kvd) // 32), dtype=torch.int32, device=dev)

    def decode_part_size(self, B: int, Hq: int, max_len: int) -> int:
        """Split-K partition length of the paged decode attention: small batches split the context
        finer so the grid still covers the CUs (B x Hkv x parts workgroups), within the partial-
        result workspace (rows = B * Hq * parts)."""
        cap = self.part_ml.shape[0]
        big = (DECODE_PART_LARGE_B, 256) if B >= 64 else (256,)
        small = (DECODE_PART_SMALL_B, 128, 256) if DECODE_PART_SMALL_B != 64 else (64, 128, 256)
        for part in (small if B < 8 else (128, 256) if B < 32 else big):
            if B * Hq * max(1, -(-max_len // part)) <= cap:
                return part
        return 256

    def q8(self, M: int, K_: int):
        return self.xq[: M * K_].view(M, K_), self.xds[: M * K_ // 16].view(M, K_ // 32, 2)



# decode batches of at least this many rows whose contexts are all <= SINGLE_PART_MAX keys run the decode
# attention as ONE partition per sequence (no partition-merge launch; engine short-context graphs capture it)
SINGLE_PART_MIN_B = int(__import__("os").environ.get("MX_SINGLE_PART_MIN_B", "64"))
SINGLE_PART_MAX = 1024


class LlamaModel:
    def _decode_part(self, ws, nd: int, Hq: int, max_len: int) -> int:
        if max_len and nd >= SINGLE_PART_MIN_B and max_len <= SINGLE_PART_MAX:
            return max(512, -(-max_len // 16) * 16)
        return ws.decode_part_size(nd, Hq, max_len or self.cfg.ctx_train)

    def __init__(self, cfg: LlamaConfig, device="cpu", tp_rank: int = 0, tp_size: int = 1, tp_group=None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.tp_rank, self.tp_size, self.tp_group = tp_rank, tp_size, tp_group
        self.layers: list[LlamaLayer] = []
        self.tok_embd: QWeight | torch.Tensor | None = None
        self.out_norm: torch.Tensor | None = None
        self.lm_head: QWeight | None = None
        rot = cfg.rope_dim
        inv, af = K.rope_inv_freq(rot, cfg.rope_base, cfg.rope_scale, cfg.rope_scaling, cfg.rope_orig_ctx,
                                  llama3=cfg.rope_llama3, freq_factors=cfg.extra.get("rope_freqs"))
        self.inv_freq = inv.to(self.device)
        self.attn_factor = af
        self.scale = cfg.attn_scale or 1.0 / math.sqrt(cfg.head_dim)
        self.local_rope = None
        if cfg.rope_base_local and cfg.sliding_window:
            li, la = K.rope_inv_freq(rot, cfg.rope_base_local)
            self.local_rope = (li.to(self.device), la)
        self.glu_epi = EPI_GEGLU if cfg.ffn_act == "gelu" else EPI_SWIGLU
        self.n_heads = cfg.n_heads // tp_size
        self.n_kv = max(1, cfg.n_kv_heads // tp_size)
        self.stage = False  # middle pipeline stage (hidden in, hidden out)
        self.remote = None  # parallel.pp_rpc.RemoteStages running the layers after ours

    @property
    def kv_layers(self) -> int:
        """Blocks whose KV cache lives in this process (all of them unless the model is split)."""
        return len(self.layers)

    # ------------------------------------------------------------------ loading
    @classmethod
    def load(cls, cfg: LlamaConfig, get_tensor, device="cpu", tp_rank=0, tp_size=1, tp_group=None,
             fuse: bool = True, progress=None, layer_range: tuple | None = None,
             stage: bool = False) -> "LlamaModel":
        """get_tensor(name) -> (raw ndarray, qtype, ggml_shape) or None.

        layer_range=(l0, l1): load only those blocks (pipeline split, parallel/pp_rpc.py); stage=True:
        a middle pipeline stage — no embedding / head, forward() maps hidden rows to hidden rows."""
        from ..parallel import tp as TP
        m = cls(cfg, device, tp_rank, tp_size, tp_group)
        dev = m.device
        plan = getattr(get_tensor, "plan", None)

        def has(name):  # existence without materialising the tensor (synthetic sources carry a plan)
            return (name in plan) if plan is not None else get_tensor(name) is not None

        def f32(name):
            t = get_tensor(name)
            if t is None:
                return None
            raw, qt, shape = t
            from ..ops.quant import dequantize
            return torch.from_numpy(np.ascontiguousarray(dequantize(raw, qt, shape)).reshape(-1).copy()).to(dev)

        def qw(name, split=None):
            shard = getattr(get_tensor, "shard", None)
            if tp_size > 1 and split is not None and shard is not None and has(name):
                # source that generates only this rank's slice (synthetic multi-GPU benches)
                raw, qt, N_, K_ = shard(name, split, tp_rank, tp_size)
                return QWeight.from_ggml(raw, qt, N_, K_, dev, name, t32=True)
            t = get_tensor(name)
            if t is None:
                return None
            raw, qt, shape = t
            K_, N_ = int(shape[0]), int(np.prod(shape[1:]))
            raw = np.asarray(raw).view(np.uint8).reshape(N_, -1)  # ggml bytes, one row per output
            if tp_size > 1 and split is not None:
                raw, N_, K_ = TP.shard_raw(raw, qt, N_, K_, split, tp_rank, tp_size, cfg)
            return QWeight.from_ggml(raw, qt, N_, K_, dev, name, t32=True)

        def qw_rows(name, row_counts, splits):
            """Split a fused [sum(rows), K] ggml tensor into per-part QWeights (phi3 attn_qkv / ffn_up)."""
            t = get_tensor(name)
            raw, qt, shape = t
            K_ = int(shape[0])
            raw = np.asarray(raw).view(np.uint8).reshape(int(np.prod(shape[1:])), -1)
            out, r0 = [], 0
            for n_, sp in zip(row_counts, splits):
                part = raw[r0:r0 + n_]
                r0 += n_
                N_ = n_
                if tp_size > 1:
                    part, N_, K2 = TP.shard_raw(part, qt, N_, K_, sp, tp_rank, tp_size, cfg)
                out.append(QWeight.from_ggml(np.ascontiguousarray(part), qt, N_, K_, dev, name, t32=True))
            return out

        hd = cfg.head_dim
        l0, l1 = layer_range or (0, cfg.n_layers)
        m.stage = stage
        for i in range(l0, l1):
            p = f"blk.{i}."
            if has(p + "attn_qkv.weight"):  # phi3: fused Q|K|V rows
                wq, wk, wv = qw_rows(p + "attn_qkv.weight", [cfg.q_dim, cfg.kv_dim, cfg.kv_dim],
                                     [("col_heads", cfg.n_heads, hd), ("col_heads", cfg.n_kv_heads, hd),
                                      ("col_heads", cfg.n_kv_heads, hd)])
            else:
                wq = qw(p + "attn_q.weight", ("col_heads", cfg.n_heads, hd))
                wk = qw(p + "attn_k.weight", ("col_heads", cfg.n_kv_heads, hd))
                wv = qw(p + "attn_v.weight", ("col_heads", cfg.n_kv_heads, hd))
            bias = None
            if cfg.qkv_bias:
                bq, bk, bv = f32(p + "attn_q.bias"), f32(p + "attn_k.bias"), f32(p + "attn_v.bias")
                if bq is not None:
                    if tp_size > 1:
                        bq, bk, bv = (TP.shard_vec(b, hd * n, tp_rank, tp_size) for b, n in
                                      ((bq, cfg.n_heads), (bk, cfg.n_kv_heads), (bv, cfg.n_kv_heads)))
                    bias = torch.cat([bq, bk, bv]).float().contiguous()
            parts = [[wq]]
            for w in (wk, wv):
                if fuse and w.qtype == parts[-1][-1].qtype and w.K == parts[-1][-1].K:
                    parts[-1].append(w)
                else:
                    parts.append([w])
            qkv_parts = [g[0] if len(g) == 1 else concat_rows(g, p + "attn_qkv") for g in parts]
            moe = None
            wg = wu = wgu = wd = None
            if cfg.n_expert:
                moe = load_moe(m, get_tensor, p, f32, qw, fuse)  # expert-parallel under TP
            else:
                if not has(p + "ffn_gate.weight") and has(p + "ffn_up.weight"):
                    wg, wu = qw_rows(p + "ffn_up.weight", [cfg.ffn, cfg.ffn], [("col", cfg.ffn), ("col", cfg.ffn)])
                else:
                    wg = qw(p + "ffn_gate.weight", ("col", cfg.ffn))
                    wu = qw(p + "ffn_up.weight", ("col", cfg.ffn))
                wgu = interleave_gate_up(wg, wu, p + "ffn_gate_up") if fuse else None
                wd = qw(p + "ffn_down.weight", ("row", cfg.ffn))
            qn = f32(p + "attn_q_norm.weight") if cfg.qk_norm else None
            kn = f32(p + "attn_k_norm.weight") if cfg.qk_norm else None
            pan = f32(p + "post_attention_norm.weight") if cfg.post_norms else None
            pfn = f32(p + "post_ffw_norm.weight") if cfg.post_norms else None
            win = cfg.layer_window(i)
            layer = LlamaLayer(
                attn_norm=f32(p + "attn_norm.weight").float(),
                ffn_norm=f32(p + "ffn_norm.weight").float(),
                qkv_parts=qkv_parts, bqkv=bias,
                wo=qw(p + "attn_output.weight", ("row", cfg.q_dim)),
                wgu=wgu, wg=None if wgu is not None else wg, wu=None if wgu is not None else wu,
                wd=wd, moe=moe,
                q_norm=qn.float().contiguous() if qn is not None else None,
                k_norm=kn.float().contiguous() if kn is not None else None,
                post_attn_norm=pan.float().contiguous() if pan is not None else None,
                post_ffn_norm=pfn.float().contiguous() if pfn is not None else None,
                window=win, rope=m.local_rope if win else None,
            )
            m.layers.append(layer)
            if progress:
                progress(i + 1, cfg.n_layers)
        if stage:
            m.finalize_layout()
            return m
        emb = get_tensor("token_embd.weight")
        raw, qt, shape = emb
        m.tok_embd = QWeight.from_ggml(np.asarray(raw).view(np.uint8).reshape(int(shape[1]), -1), qt,
                                       int(shape[1]), int(shape[0]), dev, "token_embd", t32=True)
        m.out_norm = f32("output_norm.weight").float()
        if tp_size > 1:
            # vocab-parallel LM head: rank r holds vocab rows [r*V/tp, (r+1)*V/tp) (tied embeddings: a
            # slice of token_embd; the lookup keeps the full table)
            hname = "output.weight" if has("output.weight") else "token_embd.weight"
            if not has("output.weight"):
                cfg.tie_embeddings = True
            raw, qt, shape = get_tensor(hname)
            V, K_ = int(shape[1]), int(shape[0])
            rows = np.asarray(raw).view(np.uint8).reshape(V, -1)
            vl = vocab_shard(V, tp_size)
            lo, hi = min(V, tp_rank * vl), min(V, (tp_rank + 1) * vl)
            part = np.zeros((vl, rows.shape[1]), np.uint8)
            part[:hi - lo] = rows[lo:hi]  # zero rows past V: logits 0, trimmed after the gather
            m.lm_head = QWeight.from_ggml(part, qt, vl, K_, dev, "output.shard", t32=True)
        elif not has("output.weight"):
            m.lm_head = m.tok_embd
            cfg.tie_embeddings = True
        else:
            m.lm_head = qw("output.weight")
        m.finalize_layout()
        if tp_size > 1 and m.device.type == "cuda":
            m.enable_custom_allreduce()  # collective: every TP rank loads the model at the same point
        return m

    def finalize_layout(self):
        """Re-lay the dense-layer projections (and the LM head) out in the t32 tiled layout the qmm /
        qmv kernels stream (ops/quant.py tile32). After gate|up interleaving and Q|K|V fusion, which
        work on the row layout. MoE expert stacks (gate|up interleaved per expert, down) and shared experts go t32 too
        when every expert's rows are whole 32-row groups and K is whole super-blocks: the grouped qmm2 GEMM and the
        grouped decode GEMV (ops/moe.py) stream them; stacks that do not qualify keep the row layout and the
        qgemm16 grouped kernel. No-op on CPU / bf16 mode."""
        # the q8-activation decode GEMVs need block-quantised weights: a dense (F16 / BF16) checkpoint runs
        # its small batches through the 16-bit GEMM path instead
        self._gemv_ok = all(not isinstance(w, QWeight) or w.is_quant for L in self.layers
                            for w in (*L.qkv_parts, L.wo, L.wgu, L.wg, L.wu, L.wd))
        if self.device.type != "cuda":
            return
        for L in self.layers:
            for w in (*L.qkv_parts, L.wo, L.wgu, L.wg, L.wu, L.wd):
                if isinstance(w, QWeight):
                    w.to_t32()
            if L.moe is not None:
                L.moe.to_t32()
        if isinstance(self.lm_head, QWeight):
            self.lm_head.to_t32()  # tied embeddings follow (embed() reads either layout)
        if isinstance(self.tok_embd, QWeight) and self.tok_embd is not self.lm_head and \
                int(self.tok_embd.qtype if self.tok_embd.is_quant else -1) in (int(q) for q in Q.T32_ONLY):
            self.tok_embd.to_t32()  # Q5_K / MX4F / MX5F rows are gathered by the t32 dequant kernel
        # anything a t32-only format left in the row layout (expert stacks, odd shapes) -> Q8_0 kernels
        ws = [self.tok_embd, self.lm_head]
        for L in self.layers:
            ws += [*L.qkv_parts, L.wo, L.wgu, L.wg, L.wu, L.wd]
            if L.moe is not None:
                ws += [getattr(L.moe, a, None) for a in ("gate_up", "down", "sh_gate_up", "sh_down", "sh_gate", "sh_up")]
        for w in ws:
            if isinstance(w, QWeight):
                w.ensure_kernel_layout()

    def gemm_specs(self):
        """(QWeight, epilogue, split-able output) of every M > 4 GEMM the forward issues — the shapes the load-time
        autotuner (ops/autotune.py) times, with the epilogues forward() passes for them."""
        tp = self.tp_size > 1
        for L in self.layers:
            for w in L.qkv_parts:
                yield w, EPI_F32, True
            for w in (L.wo, L.wd):
                if w is not None:
                    yield (w, EPI_BF16, False) if tp else (w, EPI_ADD_F32, True)
            if L.wgu is not None:
                yield L.wgu, self.glu_epi, False
            for w in (L.wg, L.wu):
                if w is not None:
                    yield w, EPI_BF16, False
        if isinstance(self.lm_head, QWeight):
            yield self.lm_head, EPI_F32, False

    def weight_bytes(self) -> int:
        n = 0
        for L in self.layers:
            for w in (*L.qkv_parts, L.wo, L.wgu, L.wg, L.wu, L.wd):
                if w is not None:
                    n += w.nbytes()
            if L.moe is not None:
                n += L.moe.nbytes()
        n += self.lm_head.nbytes()
        if self.tok_embd is not self.lm_head:
            n += self.tok_embd.nbytes()
        return n

    def enable_prefill_bf16_cache(self):
        """Dense 16-bit copies of the projections (+ LM head) for the hipBLASLt large-M path."""
        for L in self.layers:
            parts = L.qkv_parts
            if len(parts) > 1 and all(w.is_quant for w in parts) and parts[0].data.is_cuda:
                # one dense Q|K|V matrix: a single GEMM straight into the contiguous fp32 qkv rows instead
                # of one GEMM per quant-type group plus a widening copy into the strided slices
                L.qkv_dense = torch.cat([w.dequant_gpu(ACT_DTYPE) for w in parts])
                parts = ()
            for w in (*parts, L.wo, L.wgu, L.wg, L.wu, L.wd):
                if w is not None:
                    w.build_bf16_cache()
            if L.moe is not None:
                L.moe.build_bf16_cache()
        if isinstance(self.lm_head, QWeight) and self.lm_head.is_quant and self.lm_head.layout != "t32":
            self.lm_head.build_bf16_cache()  # t32 LM heads run qmm at every M (measured faster)

    def dense_cache_bytes(self) -> int:
        """Bytes held by the dense 16-bit weight copies (0 unless enable_prefill_bf16_cache ran)."""
        ws = [self.lm_head] if isinstance(self.lm_head, QWeight) else []
        for L in self.layers:
            ws += [w for w in (*L.qkv_parts, L.wo, L.wgu, L.wg, L.wu, L.wd) if w is not None]
            if L.moe is not None:
                ws += [w for w in (L.moe.sh_gate_up, L.moe.sh_down) if w is not None]
        n = sum(L.qkv_dense.numel() * L.qkv_dense.element_size() for L in self.layers if L.qkv_dense is not None)
        return n + sum(w.bf16_cache.numel() * w.bf16_cache.element_size() for w in ws
                       if getattr(w, "bf16_cache", None) is not None)

    # ------------------------------------------------------------------ forward
    def embed(self, tokens: torch.Tensor, out: torch.Tensor):
        E = self.tok_embd
        if E.device.type == "cpu" or not E.is_quant:
            if E.device.type == "cpu":
                out.copy_(E.dense_f32()[tokens.long()] * self.cfg.embed_scale)
            else:
                K.gather_rows(E.data, tokens, out, self.cfg.embed_scale)
            return out
        from .. import _native as N
        if E.layout == "t32":
            N.kcall("mxk_dequant_t32", int(E.qtype), E.data.data_ptr(), tokens.data_ptr(), tokens.numel(), E.K,
                    None, out.data_ptr(), out.stride(0), N.stream_ptr())
        else:
            N.kcall("mxk_dequant_rows", int(E.qtype), E.data.data_ptr(), N.ptr(E.dplane), tokens.data_ptr(),
                    tokens.numel(), E.K, None, out.data_ptr(), out.stride(0), N.stream_ptr())
        if self.cfg.embed_scale != 1.0:
            out.mul_(self.cfg.embed_scale)
        return out

    def _allreduce(self, t: torch.Tensor):
        if self.tp_size > 1:
            ar = getattr(self, "custom_ar", None)
            if ar is not None:
                ar(t)  # one-shot IPC kernel for small messages, RCCL above its max_bytes
                return
            from ..parallel import tp as TP
            TP.all_reduce_(t, self.tp_group)

    TP_CHUNK_MIN_ROWS = int(__import__("os").environ.get("MX_TP_CHUNK_MIN_ROWS", "64"))
    TP_CHUNKS = int(__import__("os").environ.get("MX_TP_CHUNKS", "2"))

    def _tp_chunks(self, T: int, y16: torch.Tensor) -> int:
        """Row chunks of a row-parallel projection whose all-reduce is overlapped with the next chunk's GEMM:
        MX_TP_CHUNKS (default 2) from MX_TP_CHUNK_MIN_ROWS rows, more when a chunk would not fit the one-shot
        all-reduce's buffer (so large decode batches stay off RCCL); 1 = no overlap."""
        if self.TP_CHUNKS <= 1 or T < self.TP_CHUNK_MIN_ROWS:
            return 1
        n = self.TP_CHUNKS
        ar = getattr(self, "custom_ar", None)
        if ar is not None:
            row_bytes = y16.shape[1] * y16.element_size()
            n = max(n, -(-T * row_bytes // ar.max_bytes))
        return max(1, min(n, 8, T // max(1, self.TP_CHUNK_MIN_ROWS // 4)))  # chunks of >= MIN_ROWS / 4 rows

    def _chunked_proj_allreduce(self, mm, W: QWeight, x, y16, h, T: int, nch: int):
        """h += all-reduce(x W^T) in `nch` row chunks: chunk c's GEMM runs on the compute stream while chunk
        c-1's all-reduce + residual add runs on a second stream (event fork / join, hipGraph-capturable); the
        compute stream waits for the last all-reduce before the next norm reads h. Without a GPU the chunks
        run in order (same arithmetic: the all-reduce of a row chunk is that chunk of the all-reduce)."""
        bounds = [T * c // nch for c in range(nch + 1)]
        ar = getattr(self, "custom_ar", None)
        self.tp_chunked_calls = getattr(self, "tp_chunked_calls", 0) + 1

        def reduce_add(r0, r1):
            if ar is not None and ar.fits(y16[r0:r1]):
                ar.add_into(y16[r0:r1], h[r0:r1])
            else:
                self._allreduce(y16[r0:r1])
                if h.is_cuda:
                    N.ensure_act(y16.dtype)
                    N.kcall("mxk_add_act_into_f32", y16[r0:r1].data_ptr(), y16.stride(0), h[r0:r1].data_ptr(),
                            h.stride(0), r1 - r0, h.shape[1], N.stream_ptr())
                else:
                    h[r0:r1].add_(y16[r0:r1])

        if not y16.is_cuda:
            for r0, r1 in zip(bounds, bounds[1:]):
                mm(W, x[r0:r1], EPI_BF16, y16[r0:r1])
                reduce_add(r0, r1)
            return
        cur = torch.cuda.current_stream(y16.device)
        s2 = getattr(self, "_ar_stream", None)
        if s2 is None:
            s2 = self._ar_stream = torch.cuda.Stream(y16.device)
        for r0, r1 in zip(bounds, bounds[1:]):
            mm(W, x[r0:r1], EPI_BF16, y16[r0:r1])
            ev = torch.cuda.Event()
            ev.record(cur)
            s2.wait_event(ev)
            with torch.cuda.stream(s2):
                reduce_add(r0, r1)
        done = torch.cuda.Event()
        done.record(s2)
        cur.wait_event(done)

    def enable_custom_allreduce(self, max_bytes: int = 1 << 20):
        """Collective over the TP group (call on every rank, outside graph capture): small row-parallel
        all-reduces go through the one-shot hipIpc kernel (parallel/custom_ar.py). MX_CUSTOM_AR=0 disables."""
        import os
        import torch.distributed as dist
        if self.tp_size <= 1 or self.device.type != "cuda" or os.environ.get("MX_CUSTOM_AR", "1") == "0":
            return None
        from ..parallel.custom_ar import OneShotAllReduce
        if not dist.is_initialized():
            # single-process shard rehearsal (bench.py --tp-rehearsal): the same one-launch all-reduce + residual
            # add over this rank's own slot, so the rehearsal's step has the real path's kernels (minus xGMI)
            self.custom_ar = OneShotAllReduce(None, self.device, max_bytes, world=1)
            return self.custom_ar
        self.custom_ar = OneShotAllReduce(self.tp_group, self.device, max_bytes)
        return self.custom_ar

    def prefill_rows(self) -> int:
        """Query rows per prefill-attention tile (attention.hip) for this model's head layout."""
        from .. import _native as N
        return int(N.kernels().mxk_attn_prefill_rows(self.n_heads, self.n_kv))

    def _norm_fuse_on(self, T: int, gemv: bool, fb, ws: Workspace) -> bool:
        """Whether this M = T forward splits each layer's RMSNorms across the GEMMs around them (ops/linear.py
        NormFuse): dense SwiGLU layers, no LoRA / post-norms / dense qkv copy, one rank, every o_proj / down / qkv /
        gate|up GEMM on a qmm2 plan with a fused instance. Cached per (T, tuned-plan count)."""
        if gemv or self.tp_size != 1 or self.device.type != "cuda" or fb.stop_layer is not None or not self.layers:
            return False
        key = (T, len(_AT.TUNED))
        c = self.__dict__.setdefault("_nf_cache", {})
        ok = c.get(key)
        if ok is None:
            H = self.cfg.hidden
            ok = (self.glu_epi == EPI_SWIGLU and T <= ws.norm_ss.shape[1]
                  and -(-T // 32) * -(-H // 32) <= ws.norm_tick.numel() and ws.xb.dtype == torch.float16)
            for L in self.layers if ok else ():
                if (L.moe is not None or L.lora is not None or L.post_attn_norm is not None
                        or L.post_ffn_norm is not None or L.qkv_dense is not None or L.wgu is None
                        or L.attn_norm.dtype != torch.float32 or L.ffn_norm.dtype != torch.float32
                        or not norm_fusable(L.wo, T, EPI_ADD_F32) or not norm_fusable(L.wd, T, EPI_ADD_F32)
                        or not norm_fusable(L.wgu, T, EPI_SWIGLU)
                        or not all(norm_fusable(w, T, EPI_F32, True) for w in L.qkv_parts)):
                    ok = False
                    break
            c[key] = ok
        return ok

    def _rope_fuse_on(self, T: int) -> bool:
        """Every layer's q|k|v GEMM at M = T runs a qmm2 plan with a fused instance (RoPE epilogue, mode bit 4)."""
        key = ("rope", T, len(_AT.TUNED))
        c = self.__dict__.setdefault("_nf_cache", {})
        ok = c.get(key)
        if ok is None:
            ok = all(L.qkv_dense is None and all(norm_fusable(w, T, EPI_F32, True, rope=True) for w in L.qkv_parts)
                     for L in self.layers)
            c[key] = ok
        return ok

    def forward(self, fb: ForwardBatch, kv, ws: Workspace) -> torch.Tensor:
        cfg = self.cfg
        T = fb.T
        H = cfg.hidden
        D = cfg.head_dim
        Hq, Hkv = self.n_heads, self.n_kv
        qd, kvd = Hq * D, Hkv * D
        F = self.layers[0].wd.K if self.layers and self.layers[0].wd is not None else 0
        eps = cfg.rms_eps
        gemv = T <= GEMV_MAX_M and self.device.type == "cuda" and getattr(self, "_gemv_ok", True)
        nd = fb.n_decode
        h = ws.h[:T]
        if not self.stage:  # a pipeline stage finds its input hidden rows in ws.h
            self.embed(fb.tokens, h)
            if fb.embed_rows:
                for r0, e in fb.embed_rows:
                    h[r0:r0 + e.shape[0]].copy_(e)
        xb = ws.xb[:T, :H]
        # M > 4: each layer's RMSNorms split across the GEMMs (o_proj -> gate|up, down -> next qkv), no norm launches
        nf = self._norm_fuse_on(T, gemv, fb, ws)
        nl = len(self.layers)
        nf_rope = (_LIN.ROPE_FUSE and not gemv and self.tp_size == 1 and self.device.type == "cuda" and not cfg.neox
                   and cfg.rope_dim == D and D in (64, 128) and fb.stop_layer is None and ws.q.dtype == torch.bfloat16
                   and -(-T // 32) * -(-(qd + 2 * kvd) // 32) <= ws.norm_tick.numel()
                   and self._rope_fuse_on(T))
        # the step's RoPE table for the epilogue: (cos, sin) x attn_factor per row position, shared by every layer
        rot_tab = None
        if nf_rope:
            ang = fb.positions[:T].float()[:, None] * self.inv_freq[None, :].float()
            rot_tab = torch.stack((torch.cos(ang), torch.sin(ang)), -1).mul_(self.attn_factor).contiguous()
        for li, L in enumerate(self.layers):
            if fb.stop_layer is not None and li >= fb.stop_layer:
                break
            # consumer side of the fused norms (this layer's qkv reads xb = f16(h * attn_norm) from the previous down)
            nf_qkv = NormFuse(2, ss_in=ws.norm_ss[1], eps=eps) if nf and li > 0 else None
            kc, vc = kv.layer(li)
            # ---- attention block ----
            qkv = ws.qkv[:T]
            # batch <= 4: RMSNorm + q8 quantisation fused into each projection's GEMV prologue
            fuse_in = gemv and T <= QMV_FUSE_MAX_M
            fuse_qkv = fuse_in and all(qmv_fusable(w, T, EPI_F32, True) for w in L.qkv_parts)
            if fuse_qkv:
                xq = xds = None
            elif gemv:
                xq, xds = ws.q8(T, H)
                K.rmsnorm(h, L.attn_norm, eps, out_q8=(xq, xds))
            else:
                if nf_qkv is None:
                    K.rmsnorm(h, L.attn_norm, eps, out_bf16=xb)
                xq = xds = None
            if not gemv and not qkv.is_cuda:
                qkv.zero_()
            off = 0
            if (not gemv and L.qkv_dense is not None and qkv.is_cuda and xb.dtype == L.qkv_dense.dtype
                    and T >= dense_min_m(xb.dtype, EPI_F32, True) and _fp32_out_ok(xb.dtype)):
                torch.mm(xb, L.qkv_dense.t(), out_dtype=torch.float32, out=qkv)
                off = qkv.shape[1]
            q = ws.q[:T]
            inv_freq, attn_factor = L.rope or (self.inv_freq, self.attn_factor)
            # batch 1: RoPE + KV append in each qkv part's GEMV epilogue (no rope_kv launch); every part or none
            lo = L.lora
            lo_qkv = lo.qkv if lo is not None else None
            rope_fused = (fuse_qkv and T == 1 and off == 0 and not cfg.neox and cfg.rope_dim == D
                          and L.q_norm is None and lo_qkv is None)
            # M > 4: RoPE + KV append in the q|k|v GEMM epilogue (qmm2 mode bit 4) instead of a rope_kv launch
            rope_ep = (nf_rope and off == 0 and L.q_norm is None and lo_qkv is None and kc.dtype == torch.bfloat16
                       and vc.dtype == torch.bfloat16 and L.rope is None)
            if rope_fused:
                # every part is checked before any launches: parts may mix block formats
                o2 = 0
                for w in L.qkv_parts:
                    rope_fused = rope_fused and qmv_rope_ok(w, h, q, kc, vc, D, o2)
                    o2 += w.N
            if rope_fused:
                o2 = 0
                for w in L.qkv_parts:
                    b = L.bqkv[o2:o2 + w.N] if L.bqkv is not None else None
                    if not qmv_rope_fused(w, h, L.attn_norm, eps, o2, fb.positions, fb.slots, inv_freq, b, attn_factor,
                                          Hq, Hkv, D, q.view(T, Hq, D), kc, vc, kv.block_size,
                                          sk=(ws.sk_ws, ws.sk_cnt)):
                        raise RuntimeError("qkv RoPE fusion applied to some parts only")
                    o2 += w.N
            for w in (L.qkv_parts if off == 0 and not rope_fused else ()):
                sl = qkv[:, off:off + w.N] if len(L.qkv_parts) > 1 else qkv
                if fuse_qkv:
                    qmv_fused(w, h, EPI_F32, sl, norm=L.attn_norm, eps=eps, out_zeroed=True)
                elif gemv:
                    qmatmul(w, None, EPI_F32, sl, xq=xq, xds=xds, out_zeroed=qkv.is_cuda)
                elif rope_ep:
                    qmatmul(w, xb, EPI_F32, sl, out_zeroed=True, fuse=NormFuse(
                        4 | (2 if nf_qkv is not None else 0), ss_in=ws.norm_ss[1], eps=eps, tick=ws.norm_tick,
                        rope=(fb.slots, rot_tab, L.bqkv, q, kc, vc, off, D, Hq, Hkv, kv.block_size)))
                else:
                    qmatmul(w, xb, EPI_F32, sl, out_zeroed=True, fuse=nf_qkv)
                off += w.N
            if lo_qkv is not None:  # runtime LoRA: q|k|v += B (A x) on the normed rows
                if gemv:
                    K.rmsnorm(h, L.attn_norm, eps, out_bf16=xb)
                LR.add_qkv(lo_qkv, xb, qkv)
            if not rope_fused and not rope_ep:
                K.rope_kv(qkv, L.bqkv, fb.positions, fb.slots, inv_freq, attn_factor, Hq, Hkv, D,
                          cfg.rope_dim, cfg.neox, q.view(T, Hq, D), kc, vc, kv.block_size,
                          qk_norm=(L.q_norm, L.k_norm, eps) if L.q_norm is not None else None, zero_after=True)
            attn = ws.attn[:T]
            if nd:
                K.attn_decode(q[:nd].view(nd, Hq, D), kc, vc, fb.dec_block_tables, fb.dec_seq_lens, self.scale,
                              attn[:nd].view(nd, Hq, D), max_seq_len=fb.dec_max_len or None,
                              workspace=(ws.part_ml, ws.part_o, ws.part_cnt), window=L.window, softcap=cfg.attn_softcap,
                              part_size=self._decode_part(ws, nd, Hq, fb.dec_max_len))
            if T > nd:
                K.attn_prefill(q[nd:].view(T - nd, Hq, D), kc, vc, fb.pf_block_tables, fb.pf_cu_q, fb.pf_ctx_lens,
                               self.scale, attn[nd:].view(T - nd, Hq, D), fb.pf_q_lens_host, fb.pf_ctx_lens_host,
                               window=L.window, softcap=cfg.attn_softcap, tiles=fb.pf_tiles)
            if fuse_in and L.post_attn_norm is None and self.tp_size == 1 and qmv_fusable(L.wo, T, EPI_ADD_F32):
                qmv_fused(L.wo, attn, EPI_ADD_F32, h)  # h += attn W_o^T, q8 quantisation in the prologue
            elif fuse_in and self.tp_size > 1 and self._tp_fused_proj(L.wo, attn, h, L.post_attn_norm, ws, T, eps):
                pass  # row-parallel shard: q8 prologue GEMV -> 16-bit partial -> all-reduce + residual
            else:
                if gemv:
                    aq, ads = ws.q8(T, qd)
                    K.quant_q8(attn, aq, ads)
                else:
                    aq = ads = None
                # producer: h += attn W_o^T, then xb = f16(h * ffn_norm) and the rows' sums of squares -> norm_ss[0]
                self._residual_proj(L.wo, attn, aq, ads, h, L.post_attn_norm, ws, T, eps,
                                    fuse=NormFuse(1, ss_out=ws.norm_ss[0], ss_zero=ws.norm_ss[1], gamma=L.ffn_norm,
                                                  xn=xb, tick=ws.norm_tick) if nf else None)
            if lo is not None and lo.o is not None:
                LR.add_residual(lo.o, attn, h)
            # ---- FFN block ----
            if L.moe is not None:
                # the FFN norm runs inside the MoE router kernel (GPU fast path) or just before it
                if self.tp_size > 1:  # expert parallel: this rank's experts' share, summed over ranks
                    y = ws.moe_y[:T]
                    y.zero_()
                    moe_ffn(L.moe, xb, y, norm=(h, L.ffn_norm, eps))
                    self._allreduce(y)
                    h.add_(y)
                else:
                    moe_ffn(L.moe, xb, h, norm=(h, L.ffn_norm, eps))
                continue
            act = ws.act[:T]
            if lo is not None and lo.gate_up is not None:
                # runtime LoRA on gate / up: the update lands on the pre-activation rows, so the gated activation
                # runs after it instead of in the GEMM epilogue
                K.rmsnorm(h, L.ffn_norm, eps, out_bf16=xb)
                self._lora_ffn_in(L, lo.gate_up, xb, act, T)
                self._residual_proj(L.wd, act, None, None, h, L.post_ffn_norm, ws, T, eps)
                if lo.down is not None:
                    LR.add_residual(lo.down, act, h)
                continue
            fuse_gu = fuse_in and L.wgu is not None and qmv_fusable(L.wgu, T, self.glu_epi)
            if fuse_gu:
                pass
            elif gemv:
                xq, xds = ws.q8(T, H)
                K.rmsnorm(h, L.ffn_norm, eps, out_q8=(xq, xds))
            elif not nf:
                K.rmsnorm(h, L.ffn_norm, eps, out_bf16=xb)
            if L.wgu is not None:
                if fuse_gu:
                    qmv_fused(L.wgu, h, self.glu_epi, act, norm=L.ffn_norm, eps=eps)
                elif gemv:
                    qmatmul(L.wgu, None, self.glu_epi, act, xq=xq, xds=xds)
                else:
                    qmatmul(L.wgu, xb, self.glu_epi, act,
                            fuse=NormFuse(2, ss_in=ws.norm_ss[0], eps=eps) if nf else None)
            else:
                g_out = torch.empty((T, F), dtype=ACT_DTYPE, device=h.device)
                u_out = torch.empty((T, F), dtype=ACT_DTYPE, device=h.device)
                xin = xb if not gemv else None
                qmatmul(L.wg, xin, EPI_BF16, g_out, xq=xq, xds=xds)
                qmatmul(L.wu, xin, EPI_BF16, u_out, xq=xq, xds=xds)
                K.glu(g_out, u_out, act, cfg.ffn_act)
            if fuse_in and L.post_ffn_norm is None and self.tp_size == 1 and qmv_fusable(L.wd, T, EPI_ADD_F32):
                qmv_fused(L.wd, act, EPI_ADD_F32, h)
                if lo is not None and lo.down is not None:
                    LR.add_residual(lo.down, act, h)
                continue
            if fuse_in and self.tp_size > 1 and self._tp_fused_proj(L.wd, act, h, L.post_ffn_norm, ws, T, eps):
                continue
            if gemv:
                aq, ads = ws.q8(T, F)
                K.quant_q8(act, aq, ads)
            else:
                aq = ads = None
            nf_down = None
            if nf:  # producer for the next layer's qkv (the last layer's down only re-zeroes norm_ss[0])
                last = li + 1 >= nl
                nf_down = NormFuse(1, ss_out=None if last else ws.norm_ss[1], ss_zero=ws.norm_ss[0],
                                   gamma=None if last else self.layers[li + 1].attn_norm, xn=None if last else xb,
                                   tick=ws.norm_tick)
            self._residual_proj(L.wd, act, aq, ads, h, L.post_ffn_norm, ws, T, eps, fuse=nf_down)
            if lo is not None and lo.down is not None:
                LR.add_residual(lo.down, act, h)
        if self.stage or fb.stop_layer is not None:
            return h
        if self.remote is not None:  # remote layer ranges (parallel/pp_rpc.py), in place on h
            self.remote.run(fb, h)
        # ---- head ----
        S = fb.logits_idx.numel()
        hs = ws.hs[:S]
        K.select_rows(h, fb.logits_idx, hs)
        if fb.want_hidden or fb.keep_hidden:
            hn = hs.float() * torch.rsqrt(hs.float().pow(2).mean(-1, keepdim=True) + eps) * self.out_norm
            if fb.want_hidden:
                return hn
            self.last_hidden = hn
        logits = ws.logits[:S] if self.tp_size == 1 else ws.logits_local[:S]
        if S <= GEMV_MAX_M and self.device.type == "cuda" and isinstance(self.lm_head, QWeight) and \
                qmv_fused(self.lm_head, hs, EPI_F32, logits, norm=self.out_norm, eps=eps):
            pass  # final RMSNorm + q8 quantisation in the LM-head GEMV prologue (one launch)
        elif S <= GEMV_MAX_M and self.device.type == "cuda" and self.lm_head.is_quant:
            xq, xds = ws.q8(S, H)
            K.rmsnorm(hs, self.out_norm, eps, out_q8=(xq, xds))
            qmatmul(self.lm_head, None, EPI_F32, logits, xq=xq, xds=xds)
        else:
            xbs = ws.xb[:S, :H]
            K.rmsnorm(hs, self.out_norm, eps, out_bf16=xbs)
            qmatmul(self.lm_head, xbs, EPI_F32, logits)
        if self.tp_size > 1:
            if fb.tp_local_logits:
                return logits  # the caller reduces the shards (vocab_argmax) or gathers them (finish_logits)
            logits = self._gather_vocab(logits, ws, S)
        if cfg.final_softcap:
            c = cfg.final_softcap
            torch.tanh(logits.div_(c), out=logits).mul_(c)
        return logits

    @torch.no_grad()
    def prompt_hidden(self, ids: list[int], stop_layer: int | None = None) -> torch.Tensor:
        """Hidden states of one prompt, prefilled on a private paged KV cache: the residual stream after
        `stop_layer` layers (transformers' hidden_states[stop_layer]; text encoders of diffusion pipelines
        take hidden_states[-2] = stop_layer n_layers - 1), or the final-normed rows when None.
        -> fp32 [len(ids), hidden]."""
        from ..engine.kv_cache import KVCache
        dev, cfg, P, bs = self.device, self.cfg, len(ids), 16
        blocks = list(range(1, 2 + P // bs))
        kv = KVCache(cfg.n_layers, len(blocks) + 1, self.n_kv, bs, cfg.head_dim, dev)
        ws = Workspace(cfg, max(P, 16), 1, dev)
        i32 = dict(dtype=torch.int32, device=dev)
        fb = ForwardBatch(torch.tensor(ids, **i32), torch.arange(P, **i32),
                          torch.tensor([blocks[p // bs] * bs + p % bs for p in range(P)], **i32),
                          torch.arange(P, **i32), n_decode=0, pf_block_tables=torch.tensor([blocks], **i32),
                          pf_cu_q=torch.tensor([0, P], **i32), pf_ctx_lens=torch.tensor([P], **i32),
                          pf_q_lens_host=[P], pf_ctx_lens_host=[P])
        fb.stop_layer = cfg.n_layers if stop_layer is None else int(stop_layer)
        h = self.forward(fb, kv, ws)[:P].float().clone()
        if stop_layer is None:  # the final norm, as the embeddings path applies it
            h = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + cfg.rms_eps) * self.out_norm.float()
        return h

    def finish_logits(self, logits_local: torch.Tensor, ws: Workspace) -> torch.Tensor:
        """Full logits from a tp_local_logits forward's shard (a collective: every rank calls it)."""
        S = logits_local.shape[0]
        logits = self._gather_vocab(logits_local, ws, S)
        if self.cfg.final_softcap:
            c = self.cfg.final_softcap
            torch.tanh(logits.div_(c), out=logits).mul_(c)
        return logits

    def vocab_argmax(self, logits_local: torch.Tensor, ws: Workspace, out: torch.Tensor) -> torch.Tensor:
        """Tensor-parallel greedy head without the logits all-gather: each rank reduces its vocabulary
        shard to (max, global index) per row, the ranks all-gather those (8 bytes per row and rank instead
        of V/tp fp32 logits — 65 MB at 128 rows, 128k vocabulary, tp 8) and merge them on the device.
        Same token as an argmax over the gathered logits (final softcap is monotonic; ties -> lowest index).
        Collective: every rank calls it."""
        import torch.distributed as dist
        S, vl = logits_local.shape
        tp, r, V = self.tp_size, self.tp_rank, self.cfg.vocab
        nv = max(0, min(V, (r + 1) * vl) - r * vl)  # the last shard's padding columns are not candidates
        if logits_local.is_cuda:
            keys, allk = ws.am_keys[:S], ws.am_keys_all[: tp * S]
            N.kcall("mxk_argmax_keys", logits_local.data_ptr(), logits_local.stride(0), S, nv, r * vl,
                    keys.data_ptr(), N.stream_ptr())
            if dist.is_initialized():
                dist.all_gather_into_tensor(allk, keys, group=self.tp_group)
            else:
                allk.copy_(keys.repeat(tp))
            N.kcall("mxk_argmax_merge", allk.data_ptr(), tp, S, out.data_ptr(), N.stream_ptr())
            return out
        # CPU (gloo) path: (value, index) pairs as float64, the same merge rule
        loc = logits_local[:, :nv].float()
        if nv:
            v, i = loc.max(dim=1)  # first maximum on ties
            pair = torch.stack([v.double(), (i + r * vl).double()], 1)
        else:
            pair = torch.stack([torch.full((S,), float("-inf"), dtype=torch.float64),
                                torch.zeros(S, dtype=torch.float64)], 1)
        allp = torch.empty((tp * S, 2), dtype=torch.float64)
        if dist.is_initialized():
            dist.all_gather_into_tensor(allp, pair.contiguous(), group=self.tp_group)
        else:
            allp.copy_(pair.repeat(tp, 1))
        allp = allp.view(tp, S, 2)
        best = allp[..., 0].max(0).values
        idx = torch.where(allp[..., 0] == best, allp[..., 1], torch.full_like(best, float("inf"))).min(0).values
        out[:S] = idx.to(out.dtype)
        return out

    def _gather_vocab(self, logits_local: torch.Tensor, ws: Workspace, S: int) -> torch.Tensor:
        """Vocab-parallel head: all-gather the [S, V/tp] slices into the full [S, V] logits."""
        import torch.distributed as dist
        vl, tp = logits_local.shape[1], self.tp_size
        g = ws.logits_gather.view(-1)[: tp * S * vl].view(tp * S, vl)  # rank r's rows at [r*S, (r+1)*S)
        if dist.is_initialized():
            dist.all_gather_into_tensor(g, logits_local.contiguous(), group=self.tp_group)
        else:
            g.copy_(logits_local.repeat(tp, 1))
        out = ws.logits[:S]
        V = out.shape[1]
        for r in range(tp):
            lo = r * vl
            if lo >= V:
                break
            out[:, lo:min(V, lo + vl)] = g[r * S:(r + 1) * S, :min(V, lo + vl) - lo]
        return out

    def _lora_ffn_in(self, L, lp, xb: torch.Tensor, act: torch.Tensor, T: int):
        """Gated FFN input with a runtime LoRA on gate / up: 16-bit pre-activations, + the low-rank update, then the
        gated activation (fused gate|up weights: one GEMM on the interleaved rows; separate gate / up otherwise)."""
        F = act.shape[1]
        if L.wgu is not None:
            y = torch.empty((T, 2 * F), dtype=xb.dtype if xb.is_cuda else torch.float32, device=xb.device)
            qmatmul(L.wgu, xb, EPI_BF16, y)
            LR.add_gate_up(lp, xb, y, F)
            glu_interleaved(y, self.glu_epi, act)
            return
        g = torch.empty((T, F), dtype=act.dtype, device=act.device)
        u = torch.empty((T, F), dtype=act.dtype, device=act.device)
        qmatmul(L.wg, xb, EPI_BF16, g)
        qmatmul(L.wu, xb, EPI_BF16, u)
        LR.add_parts(lp, xb, {"ffn_gate": g, "ffn_up": u})
        K.glu(g, u, act, self.cfg.ffn_act)

    def _tp_fused_proj(self, W: QWeight, x, h: torch.Tensor, post_norm, ws: Workspace, T: int, eps: float) -> bool:
        """Tensor-parallel decode (T <= 4) row-parallel projection with the q8 quantisation of `x` in the GEMV
        prologue (no quant_q8 launch, as on one GPU): the shard's 16-bit partial, then the all-reduce + residual.
        False (nothing launched) where the fused GEMV does not apply."""
        y16 = ws.y16[:T]
        if post_norm is not None or not h.is_contiguous() or not qmv_fused(W, x, EPI_BF16, y16):
            return False
        self._reduce_add(y16, h, T)
        return True

    def _reduce_add(self, y16: torch.Tensor, h: torch.Tensor, T: int):
        """h += all-reduce(y16): the one-shot IPC kernel's fused add when present, else the collective then the
        16-bit-into-fp32 add."""
        ar = getattr(self, "custom_ar", None)
        if ar is not None:
            ar.add_into(y16, h)
            return
        self._allreduce(y16)
        if h.is_cuda and y16.is_contiguous():
            N.ensure_act(y16.dtype)
            N.kcall("mxk_add_act_into_f32", y16.data_ptr(), y16.stride(0), h.data_ptr(), h.stride(0), T,
                    h.shape[1], N.stream_ptr())
        else:
            h.add_(y16)

    def _residual_proj(self, W: QWeight, x, xq, xds, h: torch.Tensor, post_norm, ws: Workspace, T: int, eps: float,
                       fuse: NormFuse | None = None):
        """h += x W^T — or, with a Gemma post-norm, h += rmsnorm(x W^T) * post_norm. Under tensor
        parallelism each rank's partial projection is all-reduced in 16 bits (half the fp32 residual's
        bytes; one message per row-parallel projection) and added to the replicated residual."""
        mm = qmatmul
        gemv = xq is not None
        if self.tp_size > 1:
            y16 = ws.y16[:T]
            nch = self._tp_chunks(T, y16) if (post_norm is None and not gemv and h.is_contiguous()) else 1
            if nch > 1:
                self._chunked_proj_allreduce(mm, W, x, y16, h, T, nch)
                return
            if gemv:
                mm(W, None, EPI_BF16, y16, xq=xq, xds=xds)
            else:
                mm(W, x, EPI_BF16, y16)
            ar = getattr(self, "custom_ar", None)
            if post_norm is None and ar is not None and h.is_contiguous():
                ar.add_into(y16, h)  # all-reduce + residual add in one kernel
                return
            self._allreduce(y16)
            if post_norm is None:
                if h.is_cuda and h.is_contiguous() and y16.is_contiguous():
                    N.ensure_act(y16.dtype)
                    N.kcall("mxk_add_act_into_f32", y16.data_ptr(), y16.stride(0), h.data_ptr(), h.stride(0), T,
                            h.shape[1], N.stream_ptr())
                else:
                    h.add_(y16)
            else:
                y = ws.y[:T]
                y.copy_(y16)
                K.rmsnorm_add(y, post_norm, eps, h)
            return
        if post_norm is None:
            if gemv:
                mm(W, None, EPI_ADD_F32, h, xq=xq, xds=xds)
            else:
                mm(W, x, EPI_ADD_F32, h, fuse=fuse)
            self._allreduce(h)
            return
        if fuse is not None:
            raise ValueError("norm fusion with a post-norm")
        y = ws.y[:T]
        if gemv:
            mm(W, None, EPI_F32, y, xq=xq, xds=xds)
        else:
            mm(W, x, EPI_F32, y)
        self._allreduce(y)
        K.rmsnorm_add(y, post_norm, eps, h)


def load_moe(m: LlamaModel, get_tensor, p: str, f32, qw, fuse: bool) -> MoEWeights:
    """Stacked expert tensors (ggml [K, N, E]) -> MoEWeights; gate|up interleaved per expert on GPU.
    Under tensor parallelism the experts are distributed (expert parallelism): rank r keeps experts
    [r*E/tp, (r+1)*E/tp) whole — no block-size constraint on the expert FFN width — and the shared
    expert lives on rank 0; the per-rank partial outputs are all-reduced by the caller."""
    cfg = m.cfg
    E, Fe, H = cfg.n_expert, cfg.expert_ffn, cfg.hidden
    tp, r = m.tp_size, m.tp_rank
    if E % tp:
        raise ValueError(f"{E} experts do not divide over tensor-parallel size {tp}")
    El = E // tp
    e0 = r * El
    router = f32(p + "ffn_gate_inp.weight").float().view(E, H).contiguous()

    def experts(name, rows_per):
        if tp == 1:
            return qw(name)
        raw, qt, shape = get_tensor(name)
        K_ = int(shape[0])
        rows = np.asarray(raw).view(np.uint8).reshape(E * rows_per, -1)[e0 * rows_per:(e0 + El) * rows_per]
        return QWeight.from_ggml(np.ascontiguousarray(rows), qt, El * rows_per, K_, m.device, name)

    wg = experts(p + "ffn_gate_exps.weight", Fe)
    wu = experts(p + "ffn_up_exps.weight", Fe)
    wd = experts(p + "ffn_down_exps.weight", H)
    on_gpu = m.device.type == "cuda"
    gu = interleave_gate_up(wg, wu, p + "ffn_gate_up_exps") if (fuse or on_gpu) else None
    if on_gpu and (gu is None or not gu.is_quant or not wd.is_quant):
        raise NotImplementedError(f"{p}: MoE experts need Q4_K/Q6_K/Q8_0 weights with F % 16 == 0 on the GPU")
    moe = MoEWeights(router=router, gate=None if on_gpu else wg, up=None if on_gpu else wu, gate_up=gu, down=wd,
                     n_expert=E, n_used=cfg.n_expert_used, ffn=Fe, renorm=cfg.moe_renorm, e0=e0, n_local=El)
    if cfg.expert_shared_ffn and r == 0:
        sg, su = qw(p + "ffn_gate_shexp.weight"), qw(p + "ffn_up_shexp.weight")
        moe.sh_down = qw(p + "ffn_down_shexp.weight")
        moe.sh_gate_up = interleave_gate_up(sg, su, p + "ffn_gate_up_shexp") if on_gpu else None
        if moe.sh_gate_up is None:
            moe.sh_gate, moe.sh_up = sg, su
        si = f32(p + "ffn_gate_inp_shexp.weight")
        moe.sh_inp = si.float().contiguous() if si is not None else None
    return moe
