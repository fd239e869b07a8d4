"""hipGraphLaunch host cost vs node count / node duration, and eager launch cost (microbenchmark)."""
import json
import os
import sys
import time

import torch

dev = torch.device("cuda:0")
x = torch.zeros(1, device=dev)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 350


def body(spin):
    for _ in range(N):
        if spin:
            torch.cuda._sleep(spin)
        else:
            x.add_(1)


def graph(spin):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(spin)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        body(spin)
    torch.cuda.synchronize()
    return g


out = {"env": {k: v for k, v in os.environ.items() if k.startswith("DEBUG_")}, "nodes": N}
for spin in (0, 40000):
    g = graph(spin)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = []
    t0 = time.perf_counter()
    for _ in range(10):
        a = time.perf_counter()
        g.replay()
        t.append(time.perf_counter() - a)
    h = time.perf_counter() - t0
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    out[f"graph_spin{spin}"] = {"replay_host_ms": [round(v * 1e3, 3) for v in t], "host_total_ms": round(h * 1e3, 2),
                                "gpu_total_ms": round(tot * 1e3, 2)}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        body(spin)
    h = time.perf_counter() - t0
    torch.cuda.synchronize()
    out[f"eager_spin{spin}"] = {"host_ms_per_iter": round(h / 3 * 1e3, 3),
                                "total_ms_per_iter": round((time.perf_counter() - t0) / 3 * 1e3, 3)}
print(json.dumps(out))
