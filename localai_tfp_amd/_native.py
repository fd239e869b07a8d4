"""ctypes bindings for the in-tree native libraries (``_lib/libmxk.so``, ``_lib/libmxrt.so``).

Every GPU op in :mod:`localai_tfp_amd.ops` goes through :func:`kcall`. On a machine with a GPU the
kernel library is REQUIRED: if it is missing or fails to load, :func:`kernels` raises instead of
falling back to eager PyTorch, so a GPU test can never pass on a silent fallback. The plain
PyTorch implementations in ``ops`` are only used for CPU tensors (CI / CPU plumbing path).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

_LIBDIR = Path(__file__).resolve().parent / "_lib"
_lock = threading.Lock()
_kernels = None
_runtime = None

P = C.c_void_p
I = C.c_int
F = C.c_float
SZ = C.c_size_t
U64 = C.c_uint64

# name -> argtypes (restype is always c_int = hipError_t of the launch)
KERNEL_SIGS = {
    "mxk_rmsnorm": [P, I, P, I, P, P, P, I, P, P, I, I, F, P],
    "mxk_quant_q8": [P, I, P, P, I, I, P],
    "mxk_layernorm": [P, I, P, I, P, P, P, P, P, I, I, I, F, P],
    "mxk_groupnorm_nhwc": [P, P, P, P, I, I, I, I, F, I, P],
    "mxk_layernorm_mod": [P, I, P, P, I, I, P, I, I, I, F, P],
    "mxk_gate_add": [P, I, P, I, P, I, I, I, I, P],
    "mxk_dwconv3_glu": [P, P, P, P, I, I, I, I, I, P],
    "mxk_groupnorm16": [P, P, P, P, I, I, I, I, F, I, P, P],
    "mxk_qgemm_mfma": [I, I, I, I, P, I, P, P, I, I, I, I, P, I, P],
    "mxk_qgemm16": [I, I, I, I, P, I, P, P, I, I, I, I, P, I, P],
    "mxk_qgemm32": [I, I, I, I, P, I, P, P, I, I, I, I, P, I, P],
    "mxk_qmm2": [I, I, I, I, I, P, I, P, I, I, I, I, P, I, P],
    "mxk_qmm2_fused": [I, I, I, I, I, P, I, P, I, I, I, I, P, I, I, P, P, P, P, I, P, P, F, F, P],
    "mxk_qmm2_rope": [I, I, I, I, I, P, I, P, I, I, I, I, P, I, I, P, F, F, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "mxk_qmm2_dbg": [I, I, I, I, P, I, P, I, I, I, P, I, P],
    "mxk_qmm2_set_rot": [I],
    "mxk_qmm3": [I, I, I, P, I, P, I, I, I, I, P, I, P],
    "mxk_sample_trace": [I, P],
    "mxk_qmv1_enable": [I],
    "mxk_qmv1_rope": [I, P, P, F, P, I, I, I, P, P, P, P, F, I, I, I, P, P, P, I, I, P, P, P],
    "mxk_qmm3_dbg": [I, I, P, I, P, I, I, I, P, I, P],
    "mxk_qmm_ws_dbg": [I],
    "mxk_qmv": [I, I, P, P, P, I, I, I, I, P, I, P],
    "mxk_qmv_x": [I, I, I, P, I, P, F, P, I, I, I, I, P, I, P],
    "mxk_dequant_t32": [I, P, P, I, I, P, P, I, P],
    "mxk_set_act_f16": [I],
    "mxk_attn_dense": [P, I, P, I, P, I, P, I, I, I, I, I, I, I, P, P, I, F, I, P, I, P],
    "mxk_get_act_f16": [],
    "mxk_qgemv": [I, I, P, P, P, P, I, I, I, P, I, P],
    "mxk_dequant_rows": [I, P, P, P, I, I, P, P, I, P],
    "mxk_rope_kv": [P, P, P, P, P, F, I, I, I, I, I, I, P, P, P, I, P, P, F, I, I, P],
    "mxk_copy_blocks": [P, P, P, I, I, P],
    "mxk_attn_decode": [P, I, P, P, P, I, P, I, I, I, I, I, F, I, F, I, I, P, I, P, P, I, P],
    "mxk_attn_decode_ts": [P, I, P, P, P, I, P, I, I, I, I, F, I, P, I, P, P],
    "mxk_attn_decode_mfma": [P, I, P, P, P, I, P, I, I, I, I, I, F, I, F, I, I, P, I, P, P, I, P, P],
    "mxk_attn_prefill": [P, P, P, P, I, P, P, I, P, P, I, I, I, I, F, I, F, P, I, I, P],
    "mxk_probe_tr16": [P, P],
    "mxk_attn_prefill_rows": [I, I],
    "mxk_sample": [P, I, I, I, P, P, P, P, P, I, P, P, P, P],
    "mxk_sample_topk_split": [P, I, I, I, P, I, P, P, P, P, I, I, P, P, P, P, P, P, P, P],
    "mxk_sample_params_size": [],
    "mxk_argmax": [P, I, I, I, P, P],
    "mxk_argmax_gated": [P, I, I, I, P, P, P],
    "mxk_fix_tokens": [P, P, P, P, I, P],
    "mxk_argmax_keys": [P, I, I, I, I, P, P],
    "mxk_argmax_merge": [P, I, I, P, P],
    "mxk_glu": [I, P, P, I, P, I, I, I, P],
    "mxk_rmsnorm_add": [P, I, P, P, I, I, I, F, P],
    "mxk_swiglu_il16": [P, I, P, I, I, I, I, P],
    "mxk_act_f32": [P, SZ, I, P],
    "mxk_cast_f32_bf16": [P, I, P, I, I, I, P],
    "mxk_gather_rows": [P, I, P, I, I, F, P, P],
    "mxk_add_bias_f32": [P, I, P, I, I, P],
    "mxk_add_act_into_f32": [P, I, P, I, I, I, P],
    "mxk_select_rows_f32": [P, I, P, I, I, P, I, P],
    "mxk_lstm_scan": [P, P, P, P, P, F, P, I, I, I, P],
    "mxk_lstm_bidir": [P, P, P, P, P, P, I, I, P],
    "mxk_lstm_coop": [P, P, P, P, P, P, I, I, I, P],
    "mxk_wavenet_gate": [P, P, I, I, I, P],
    # xz, ldxz, w, bias, state, kc, slots, positions, slot_div, n_dec, pf_cu, n_pf, xc, xc16, ldo16, Di, stream
    "mxk_ssm_conv": [P, I, P, P, P, I, P, P, I, I, P, I, P, P, I, I, P],
    # xc, dbc, lddbc, wdt, dt_bias, A, D, xz, ldxz, state, slots, positions, slot_div, n_dec, pf_cu, n_pf,
    # y16, ldy, Di, R, d_state, stream
    # x, ldx, shift_state, sx_in, sx_out, maa, dm, out, n_mix, slots, positions, slot_div, n_dec, pf_cu, n_pf, T, C, st
    "mxk_rwkv_shift_mix": [P, I, P, P, P, P, P, P, I, P, P, I, I, P, I, I, I, P],
    # r, k, v, w, g, ld, u, state, lnw, lnb, eps, out, ldo, slots, positions, slot_div, n_dec, pf_cu, n_pf, H, hs, st
    "mxk_rwkv_wkv6": [P, P, P, P, P, I, P, P, P, P, F, P, I, P, P, I, I, P, I, I, I, P],
    # qkv, ld, rows, D, H, head_dim, wq, wk, cs, L, eps, stream
    "mxk_qk_norm_rope": [P, I, I, I, I, I, P, P, P, I, F, P],
    "mxk_qk_norm_rope_gqa": [P, I, I, I, I, I, I, P, P, P, I, F, P],
    "mxk_ssm_scan": [P, P, I, P, P, P, P, P, I, P, P, P, I, I, P, I, P, I, I, I, I, P],
    "mxk_moe_route": [P, I, I, I, I, I, P, P, P],
    # kvf, ks, vs, slots, T, Hkv, D, bs, kc, vc, stream
    "mxk_kvq_append": [I, P, P, P, I, I, I, I, P, P, P],
    # kvf, cache, rows, n, D, out, stream
    "mxk_kvq_dequant_rows": [I, P, P, I, I, P, P],
    # x, ldx, wr, T, H, E, k, renorm, ids, wts, logits (workspace [T, E] fp32), stream
    "mxk_moe_router": [P, I, P, I, I, I, I, I, P, P, P, P, P, I, P, F, P],
    # qtype, epi, W, N, K, ids, P, e0, El, x, ldx, xdiv, C, ldc, stream
    "mxk_qmv_moe": [I, I, P, I, I, P, I, I, I, P, I, I, P, I, P],
    "mxk_moe_route_sort": [P, I, I, I, I, I, P, P, I, P, P, P, P, P, P],
    "mxk_qmv_moe_down": [I, P, I, I, P, P, I, I, I, I, P, I, P, I, P],
    # qtype, epi, wm, A, lda, stok, W, P, E, N, K, tiles, off, C, ldc, stream
    "mxk_qmm2_grouped": [I, I, I, P, I, P, P, I, I, I, I, P, P, P, I, P, P, P],
    "mxk_moe_sort": [P, I, I, I, I, P, P, P, P, P, P, P],
    "mxk_moe_combine": [P, I, P, P, I, I, I, P, I, I, P],
    "mxk_moe_qgemm16": [I, I, I, P, I, P, P, P, P, P, I, I, I, I, P, I, P],
    # x, Nb, H, W, Cp, w, Cout, KH, KW, Kp, stride, dil, pad_h, pad_w, up, Ho, Wo, bias, tadd, ldt, res, ldr, y,
    # ldy, act, zero, cfg, stream
    "mxk_conv2d": [P, I, I, I, I, P, I, I, I, I, I, I, I, I, I, I, I, P, P, I, P, I, P, I, I, P, I, P],
    "mxk_conv_tile_auto": [I, I],
}

HIP_ERRORS = {1: "hipErrorInvalidValue", 2: "hipErrorOutOfMemory", 98: "hipErrorInvalidDeviceFunction",
              209: "hipErrorNoBinaryForGpu", 700: "hipErrorIllegalAddress", 719: "hipErrorLaunchFailure"}


class NativeError(RuntimeError):
    pass


def _load(name: str):
    path = kernel_lib_path() if name == "libmxk.so" else _LIBDIR / name
    if not path.exists():
        raise NativeError(
            f"{path} is missing: build it with `python -m localai_tfp_amd._build` "
            "(or __graft_entry__.build())")
    return C.CDLL(str(path), mode=C.RTLD_GLOBAL)


def kernel_lib_path():
    # MX_KERNEL_LIB: an alternative build of the kernel library (same-box A/B runs of kernel variants)
    alt = os.environ.get("MX_KERNEL_LIB")
    return Path(alt) if alt else _LIBDIR / "libmxk.so"


def kernels():
    """Load libmxk.so (HIP kernels). Raises NativeError if it cannot be loaded."""
    global _kernels
    if _kernels is None:
        with _lock:
            if _kernels is None:
                lib = _load("libmxk.so")
                for n, sig in KERNEL_SIGS.items():
                    fn = getattr(lib, n, None)
                    if fn is None:
                        continue
                    fn.argtypes = sig
                    fn.restype = C.c_int
                _kernels = lib
    return _kernels


def runtime():
    """Load libmxrt.so (host runtime: GGUF parser, block allocator, grammar, store)."""
    global _runtime
    if _runtime is None:
        with _lock:
            if _runtime is None:
                _runtime = _load("libmxrt.so")
                from . import _rt_sigs
                _rt_sigs.bind(_runtime)
    return _runtime


def have_kernels() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False


_act_f16_mode = None


def ensure_act(dtype) -> None:
    """Put the kernel library's 16-bit activation format (bf16 | f16) in line with a tensor dtype
    before a launch that reads or writes 16-bit activations (mxk_set_act_f16; kernels are templated
    on it). Cached on the Python side, so steady-state calls cost one comparison."""
    global _act_f16_mode
    import torch
    want = dtype == torch.float16
    if want != _act_f16_mode:
        kernels().mxk_set_act_f16(int(want))
        _act_f16_mode = want


def kcall(name: str, *args):
    fn = getattr(kernels(), name, None)
    if fn is None:
        raise NativeError(f"{name} not exported by libmxk.so (stale build?)")
    rc = fn(*args)
    if rc != 0:
        raise NativeError(f"{name} failed: {HIP_ERRORS.get(rc, rc)} ({rc})")
    return rc


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    """data pointer of a tensor (None passes through as a null pointer)."""
    if t is None:
        return None
    return t.data_ptr()


def loaded_library_paths():
    """Paths of the native libraries loaded into this process (for diagnostics / tests)."""
    out = []
    for lib in (_kernels, _runtime):
        if lib is not None:
            out.append(lib._name)
    return out


def gpu_required() -> bool:
    """True when a GPU is present: then native kernels are mandatory (no eager fallback)."""
    if os.environ.get("MX_ALLOW_CPU_ONLY"):
        return False
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
