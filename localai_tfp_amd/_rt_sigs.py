"""ctypes signatures of libmxrt.so (host runtime)."""
import ctypes as C

P, I, U64, SZ = C.c_void_p, C.c_int, C.c_uint64, C.c_size_t

RT_SIGS = {}


def bind(lib):
    for name, (res, args) in RT_SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
