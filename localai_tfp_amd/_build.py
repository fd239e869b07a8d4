"""In-tree native build for localai_tfp_amd.

Two shared objects are produced under ``localai_tfp_amd/_lib/``:

* ``libmxk.so``  — every hand-written CDNA4 HIP kernel in ``csrc/kernels/*.hip``, compiled with
  ``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU) behind a flat ``extern "C"`` ABI
  that ``_native.py`` binds with ctypes. Launchers take a ``hipStream_t`` and never allocate, so
  they are safe inside hipGraph capture.
* ``libmxrt.so`` — the host runtime in ``csrc/runtime/*.cpp`` (GGUF mmap parser, paged-KV block
  allocator with prefix hashing, GBNF grammar matcher, vector store, stop-string matcher), plain
  C++17 behind a C ABI.

Objects are rebuilt only when a source/header hash changes. ``python -m localai_tfp_amd._build``
builds everything; ``__graft_entry__.build()`` calls :func:`build_all`.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
LIB = PKG / "_lib"
BUILD = ROOT / "build" / "native"

ARCH = os.environ.get("MX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _hash(paths):
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(str(p.name).encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def _jobs():
    try:
        n = int(os.environ.get("MAX_JOBS", "0"))
    except ValueError:
        n = 0
    if n <= 0:
        n = min(8, os.cpu_count() or 4)
    return max(1, min(n, 16))


# per-source extra compiler flags (none at present)
FILE_FLAGS: dict = {}


_INC = __import__("re").compile(r'^\s*#\s*include\s*"([^"]+)"', __import__("re").M)


def _deps(src: Path, headers) -> list:
    """The in-tree headers `src` includes, transitively (an object is rebuilt only when one of ITS headers changes)."""
    by_name = {h.name: h for h in headers}
    seen, todo = {}, [src]
    while todo:
        for inc in _INC.findall(todo.pop().read_text(errors="replace")):
            h = by_name.get(Path(inc).name)
            if h is not None and h.name not in seen:
                seen[h.name] = h
                todo.append(h)
    return list(seen.values())


def _build_lib(name: str, srcs, headers, compiler, cflags, ldflags, verbose=False) -> Path:
    LIB.mkdir(parents=True, exist_ok=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    out = LIB / name
    # the stamp lives next to the library (both travel with the tree to a GPU box); its key is independent of the
    # checkout location, so an up-to-date library is not rebuilt wherever the tree lands
    stamp = LIB / (name + ".stamp")
    portable = [f for f in cflags if not f.startswith(str(ROOT))]
    key = _hash(list(srcs) + list(headers)) + "|" + " ".join(portable) + "|" + ARCH + "|" + repr(sorted(FILE_FLAGS.items()))
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    # several ranks of one job (torchrun, 8 per node) may find the library stale at once: one builds under an
    # exclusive file lock, the others wait and then see its stamp
    import fcntl
    with open(LIB / (name + ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if out.exists() and stamp.exists() and stamp.read_text() == key:
            return out
        return _build_locked(name, out, stamp, key, srcs, headers, compiler, cflags, ldflags, verbose)


def _build_locked(name, out, stamp, key, srcs, headers, compiler, cflags, ldflags, verbose) -> Path:
    objs = []

    def compile_one(src: Path):
        obj = BUILD / (name + "." + src.stem + ".o")
        okey = BUILD / (name + "." + src.stem + ".key")
        flags = list(cflags) + FILE_FLAGS.get(src.name, [])
        k = _hash([src] + _deps(src, headers)) + "|" + " ".join(flags)
        if obj.exists() and okey.exists() and okey.read_text() == k:
            return obj
        cmd = [compiler, *flags, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        okey.write_text(k)
        return obj

    with cf.ThreadPoolExecutor(_jobs()) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out.with_suffix(".so.tmp")
    _run([compiler, "-shared", *[str(o) for o in objs], "-o", str(tmp), *ldflags])
    os.replace(tmp, out)
    stamp.write_text(key)
    return out


def build_kernels(verbose=False) -> Path:
    kdir = CSRC / "kernels"
    srcs = sorted(kdir.glob("*.hip"))
    headers = sorted(kdir.glob("*.h"))
    cflags = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-munsafe-fp-atomics",
        "-ffp-contract=fast",
        "-I",
        str(kdir),
        "-Wno-unused-result",
    ]
    return _build_lib("libmxk.so", srcs, headers, HIPCC, cflags, ["-fPIC"], verbose)


def build_runtime(verbose=False) -> Path:
    rdir = CSRC / "runtime"
    srcs = sorted(rdir.glob("*.cpp"))
    headers = sorted(rdir.glob("*.h"))
    cflags = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-I", str(rdir)]
    if os.environ.get("MX_SANITIZE"):
        # host-only sanitizer build (ASan/UBSan) of the runtime; never of GPU code.
        cflags += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
        ld = ["-fsanitize=address,undefined", "-pthread"]
    else:
        ld = ["-pthread"]
    return _build_lib("libmxrt.so", srcs, headers, CXX, cflags, ld, verbose)


def build_all(verbose=False):
    if not shutil.which(HIPCC) and not Path(HIPCC).exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    k = build_kernels(verbose)
    r = build_runtime(verbose)
    return k, r


if __name__ == "__main__":
    print(build_all(verbose="-v" in sys.argv))
