"""Load-time GEMM autotuner for the quantised-weight kernels (qmm2.hip / qmm3.hip).

The K-quant GEMMs run one workgroup per CU (up to 150 KB of LDS each), so a launch's time is set by how its
(row tile x column tile x K split) grid quantises onto the 256 CUs — a hand-written M -> tile rule mispicks
badly between its breakpoints (qkv 6144 x 4096: 55 us at M = 384 against 41 us at M = 512 with the rule's picks,
profiles/r5_gemm_curve.md). Instead, every distinct (N, K, block format, epilogue class) of a loaded model is
timed on the GPU it runs on, for each M bucket the engine produces, over every compiled tile / split
candidate; the fastest plan per bucket is kept in TUNED and ops/linear.py dispatches from it. A plan is
("q2", wm, ks, wn, splits) | ("q3", wm, splits) | ("rows", chunk) (row chunks of `chunk`, each dispatched by
its own bucket). Only kernel choice is tuned: every candidate computes the same product (the GPU tests check
every tile / split / epilogue against the fp32 reference).

Tuning costs ~1-3 s per model (a handful of shapes x buckets x ~40 candidates x ~15 launches); results are
cached per device in $MX_TUNE_CACHE (default ~/.cache/localai_tfp_amd/gemm_tune.json) and reused.
"""
from __future__ import annotations

import json
import logging
import os
import time

import torch

log = logging.getLogger("localai_tfp_amd.autotune")

# M buckets the engine's steps fall into: decode-only batches (graph buckets) and mixed decode + prompt-chunk steps
BUCKETS = (16, 32, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512)
SPLITS = (1, 2, 4, 8)
# (N, K, qtype, epi, can_split) -> [(bucket, plan)] sorted by bucket
TUNED: dict[tuple, list] = {}
TIMES: dict[tuple, list] = {}  # key -> [(bucket, plan, us)] of the plans tuned in this process (reports)
ENABLED = os.environ.get("MX_GEMM_TUNE", "1") != "0"


def _key(N: int, K: int, qtype: int, epi: int, can_split: bool) -> tuple:
    return (int(N), int(K), int(qtype), int(epi), bool(can_split))


def lookup(N: int, K: int, qtype: int, epi: int, can_split: bool, M: int):
    """Tuned plan for this GEMM at M rows, or None (untuned shape, or M beyond the largest bucket)."""
    ent = TUNED.get(_key(N, K, qtype, epi, can_split))
    if not ent:
        return None
    for b, plan in ent:
        if M <= b:
            return plan
    return None


def candidates(M: int, N: int, K: int, qtype: int, can_split: bool) -> list[tuple]:
    from . import linear as L
    nsb = K // 256
    sp = [s for s in SPLITS if (s == 1 or can_split) and nsb // s >= 2]
    out = []
    for wm, ks, wn in L.QMM2_CONFIGS:
        bm = 32 * wm * wn
        if bm > 2 * max(M, 32) and bm > 64:  # a row tile more than twice the rows: never faster
            continue
        for s in sp:
            out.append(("q2", wm, ks, wn, s))
    if M >= 32:
        for wm in (1, 2, 3, 4):
            if 64 * wm > 2 * max(M, 64):
                continue
            for s in sp:
                out.append(("q3", wm, s))
    for c in (128, 256):
        if c < M:
            out.append(("rows", c))
    return out


def _time(fn, iters: int) -> float:
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def tune_weight(W, epi: int, can_split: bool, buckets=BUCKETS, iters: int = 8) -> list:
    """Time every candidate plan of `W` (a t32 K-quant QWeight on the GPU) at each bucket; -> [(bucket, plan)]."""
    from . import linear as L
    dev = W.data.device
    Mmax = max(buckets)
    x = (torch.randn(Mmax, W.K, device=dev) * 0.5).to(torch.float16)
    if epi in L.GLU_EPIS:
        out = torch.empty(Mmax, W.N // 2, device=dev, dtype=torch.float16)
    elif epi == L.EPI_BF16:  # 16-bit activation out: the plan runner requires out.dtype == x.dtype
        out = torch.empty(Mmax, W.N, device=dev, dtype=x.dtype)
    else:
        out = torch.zeros(Mmax, W.N, device=dev, dtype=torch.float32)
    res = []
    key = _key(W.N, W.K, int(W.qtype), epi, can_split)
    TUNED[key] = res  # "rows" plans of a bucket dispatch their chunks through the buckets tuned before it
    for b in sorted(buckets):
        xb, ob = x[:b], out[:b]
        best, best_t = None, float("inf")
        for plan in candidates(b, W.N, W.K, int(W.qtype), can_split):
            if plan[0] == "rows" and not any(bb >= plan[1] for bb, _ in res):
                continue

            def run(p=plan):
                L.run_plan(p, W, xb, epi, ob, True)
            try:
                run()
            except Exception as ex:  # a candidate the library refuses (shape limits): skip it
                log.debug("tune %s M=%d %s: %s", key, b, plan, ex)
                continue
            t = min(_time(run, iters), _time(run, iters))
            if t < best_t:
                best, best_t = plan, t
        if best is not None:
            res.append((b, best))
            TIMES.setdefault(key, []).append((b, best, round(best_t, 2)))
            log.debug("tune %s M=%d -> %s %.1f us", key, b, best, best_t)
    return res


def report() -> list[dict]:
    """The plans tuned in this process with their times (bench / profiles)."""
    return [{"N": k[0], "K": k[1], "qtype": k[2], "epi": k[3], "split": k[4],
             "plans": [[b, list(p), us] for b, p, us in v]} for k, v in TIMES.items()]


def _cache_path() -> str:
    return os.environ.get("MX_TUNE_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "localai_tfp_amd",
                                                           "gemm_tune.json")


_LIB_TAG = None


def _lib_tag() -> str:
    """Hash of the kernel library: plans tuned against another build of the kernels are not reused."""
    global _LIB_TAG
    if _LIB_TAG is None:
        import hashlib
        from .. import _native as N
        try:
            with open(N.kernel_lib_path(), "rb") as f:
                _LIB_TAG = hashlib.sha1(f.read()).hexdigest()[:12]
        except (OSError, AttributeError):
            _LIB_TAG = "unknown"
    return _LIB_TAG


def _device_tag() -> str:
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    return f"{p.name}|{getattr(p, 'gcnArchName', '')}|{p.multi_processor_count}|{_lib_tag()}"


def load_cache() -> dict:
    try:
        with open(_cache_path()) as f:
            d = json.load(f)
        return d.get(_device_tag(), {})
    except (OSError, ValueError):
        return {}


def save_cache(entries: dict):
    path = _cache_path()
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            d = {}
        d.setdefault(_device_tag(), {}).update(entries)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(d, f)
        os.replace(tmp, path)
    except OSError as ex:
        log.warning("gemm tune cache not written (%s)", ex)


def tune_gemms(specs, buckets=BUCKETS) -> float:
    """specs: iterable of (QWeight, epi, can_split). Tunes each distinct GEMM once (cache first); -> seconds spent."""
    from . import linear as L
    if not ENABLED or not torch.cuda.is_available():
        return 0.0
    t0 = time.time()
    cache = load_cache()
    new = {}
    seen = set()
    for W, epi, can_split in specs:
        if (not isinstance(W, L.QWeight) or W.layout != "t32" or not W.data.is_cuda
                or int(W.qtype) not in L.QMM2_QTYPES):
            continue
        key = _key(W.N, W.K, int(W.qtype), epi, can_split)
        if key in seen:
            continue
        seen.add(key)
        ck = ",".join(map(str, key)) + "|" + ",".join(map(str, buckets))
        if ck in cache:
            TUNED[key] = [(b, tuple(p)) for b, p in cache[ck]]
            continue
        res = tune_weight(W, epi, can_split, buckets)
        if res:  # an empty result (every candidate refused) is not cached: the next load tunes it again
            new[ck] = [(b, list(p)) for b, p in res]
        else:
            log.warning("gemm autotune: no plan ran for %s; the untuned fallback rule serves it", key)
    if new:
        save_cache(new)
    dt = time.time() - t0
    log.info("gemm autotune: %d shapes (%d tuned now) in %.1f s", len(seen), len(new), dt)
    return dt
