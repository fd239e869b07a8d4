"""The host runtime (csrc/runtime: GBNF grammar engine, paged-KV block manager, vector store) built
with AddressSanitizer + UndefinedBehaviorSanitizer and driven by csrc/tests/runtime_sanitize.cpp:
malformed / left-recursive grammars, grammar masks over a byte vocabulary with random input,
allocate / commit / prefix-match / release churn, store set / find / delete. A standalone executable,
so the sanitizer runtime needs no preloading into Python. (GPU sanitizers are not available on the
MI355X pool; the HIP kernels are checked by the -m gpu numerics tests.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_runtime_asan_ubsan(tmp_path):
    rt = os.path.join(ROOT, "csrc", "runtime")
    srcs = sorted(os.path.join(rt, f) for f in os.listdir(rt) if f.endswith(".cpp"))
    exe = str(tmp_path / "runtime_sanitize")
    cc = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                         "-fno-sanitize-recover=undefined", "-I", rt, *srcs,
                         os.path.join(ROOT, "csrc", "tests", "runtime_sanitize.cpp"), "-o", exe],
                        capture_output=True, text=True, timeout=600)
    assert cc.returncode == 0, cc.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "runtime_sanitize: ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
