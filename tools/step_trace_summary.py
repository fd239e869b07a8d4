"""Summarise an engine step trace (`MX_STEP_TRACE=<file> python bench.py ...`): per step the host timeline
(schedule / plan+launch / sampler launch / process of the previous step incl. its wait) and the device time of the
step plus the device idle before the next one. Answers "where does wall time exceed kernel time": idle is
attributed to the host phase the next step's launch was waiting on.

    python tools/step_trace_summary.py trace.json [last_n_steps]
"""
from __future__ import annotations

import json
import sys

import numpy as np


def summarise(path: str, last: int = 0) -> dict:
    d = json.load(open(path))
    host, gpu = d["host"], d["gpu_ms"]
    n = min(len(host) - 1, len(gpu))
    if last:
        host, gpu = host[-(last + 1):], gpu[-last:]
        n = min(len(host) - 1, len(gpu))
    # host rows: (t0, t1, t_exec, t_samp, t2, wait, t3, graph, nd, npf, items); gpu rows: [busy_ms, idle_after_ms]
    H = np.array([[h[0], h[1], h[2], h[3], h[4], h[5], h[6], float(h[7]), h[8], h[9], h[10]] for h in host[-n - 1:]])
    G = np.array(gpu[-n:])
    wall = np.diff(H[:, 0]) * 1e3
    busy, idle = G[:, 0], G[:, 1]
    sched = (H[1:, 1] - H[1:, 0]) * 1e3
    launch = (H[1:, 2] - H[1:, 1]) * 1e3
    samp = (H[1:, 3] - H[1:, 2]) * 1e3
    wait = H[1:, 5] * 1e3
    proc = (H[1:, 6] - H[1:, 4]) * 1e3 - wait
    # gpu row i is host step i (H[:-1]); the idle after it waits on host step i + 1 (H[1:])
    graph = H[:-1, 7] > 0
    mixed = H[:-1, 9] > 0
    out = {"steps": int(n), "wall_ms": round(float(wall.mean()), 3), "gpu_busy_ms": round(float(busy.mean()), 3),
           "gpu_idle_ms": round(float(idle.mean()), 3), "graph_frac": round(float(graph.mean()), 3),
           "mixed_frac": round(float(mixed.mean()), 3),
           "host_ms": {"sched": round(float(sched.mean()), 3), "plan+launch": round(float(launch.mean()), 3),
                       "sampler": round(float(samp.mean()), 3), "wait": round(float(wait.mean()), 3),
                       "process": round(float(proc.mean()), 3)},
           "idle_pct": {str(q): round(float(np.percentile(idle, q)), 3) for q in (50, 90, 99)}}
    for name, m in (("decode_only", ~mixed), ("mixed", mixed)):
        if m.any():
            out[name] = {"n": int(m.sum()), "busy": round(float(busy[m].mean()), 3), "idle": round(float(idle[m].mean()), 3),
                         "plan+launch": round(float(launch[m].mean()), 3), "sampler": round(float(samp[m].mean()), 3),
                         "process": round(float(proc[m].mean()), 3)}
    big = np.argsort(idle)[-8:][::-1]
    out["largest_idle"] = [{"i": int(i), "idle": round(float(idle[i]), 3), "graph": bool(graph[i]),
                            "nd": int(H[i, 8]), "npf": int(H[i, 9]),
                            "next_sched": round(float(sched[min(i + 1, n - 1)]), 3),
                            "next_launch": round(float(launch[min(i + 1, n - 1)]), 3)} for i in big]
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0), indent=1))
