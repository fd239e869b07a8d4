"""roctx ranges (ROCm's marker API, libroctx64) around engine steps and model phases, so a
`rocprofv3 --marker-trace --kernel-trace` timeline groups the kernels of each continuous-batching step
(decode rows / prefill tokens in the range name). Off unless MX_ROCTX=1: one ctypes call per range
costs ~1 us of host time."""
from __future__ import annotations

import contextlib
import ctypes
import os

_LIB = None
ENABLED = os.environ.get("MX_ROCTX") == "1"


def _lib():
    global _LIB, ENABLED
    if _LIB is None:
        # rocprofv3 intercepts the rocprofiler-sdk roctx library; the roctracer-era libroctx64 is
        # only seen by the legacy tools
        for p in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                  "/opt/rocm/lib/libroctx64.so"):
            try:
                _LIB = ctypes.CDLL(p)
                _LIB.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _LIB.roctxRangePushA.restype = ctypes.c_int
                _LIB.roctxRangePop.restype = ctypes.c_int
                _LIB.roctxMarkA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        if _LIB is None:
            ENABLED = False
    return _LIB


def push(name: str):
    if ENABLED and _lib() is not None:
        _LIB.roctxRangePushA(name.encode())


def pop():
    if ENABLED and _lib() is not None:
        _LIB.roctxRangePop()


def mark(name: str):
    if ENABLED and _lib() is not None:
        _LIB.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx API name
    if not ENABLED:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()
