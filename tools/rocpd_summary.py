#!/usr/bin/env python3
"""Per-kernel table from a rocprofv3 rocpd database (`rocprofv3 --kernel-trace -d DIR -o NAME`), restricted to the
last --window-ms of GPU time (the bench's timed steady-state window, after load-time tuning and graph capture).

    python tools/rocpd_summary.py gpurun_out/k4_prof/k4_results.db --window-ms 1800 --steps 200 --top 30
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window-ms", type=float, default=0.0, help="only kernels that start in the last W ms (0: all)")
    ap.add_argument("--steps", type=int, default=0, help="engine steps inside the window (per-step column)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--gaps", action="store_true", help="also: idle time between consecutive kernels, by next kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    t_end = c.execute("select max(end) from kernels").fetchone()[0]
    t0 = t_end - a.window_ms * 1e6 if a.window_ms else 0
    rows = c.execute("select name, count(*), sum(end - start) / 1e6, avg(end - start) / 1e3 from kernels "
                     "where start >= ? group by name order by 3 desc", (t0,)).fetchall()
    tot_ms = sum(r[2] for r in rows)
    n = sum(r[1] for r in rows)
    busy = c.execute("select min(start), max(end) from kernels where start >= ?", (t0,)).fetchone()
    span = (busy[1] - busy[0]) / 1e6
    print(f"kernel time {tot_ms:.2f} ms over {n} dispatches in a {span:.2f} ms span"
          + (f"; per step: {tot_ms / a.steps:.3f} ms kernels, {span / a.steps:.3f} ms wall" if a.steps else ""))
    print()
    hdr = "| kernel | calls | total ms | avg us | % |" + (" us/step |" if a.steps else "")
    print(hdr)
    print("|---|---|---|---|---|" + ("---|" if a.steps else ""))
    for name, cnt, ms, us in rows[: a.top]:
        nm = name.replace("(anonymous namespace)::", "").split("(")[0][:100]
        line = f"| `{nm}` | {cnt} | {ms:.2f} | {us:.1f} | {100 * ms / tot_ms:.1f} |"
        if a.steps:
            line += f" {ms * 1e3 / a.steps:.1f} |"
        print(line)
    if a.gaps:
        ks = c.execute("select name, start, end from kernels where start >= ? order by start", (t0,)).fetchall()
        by: dict = {}
        tot = 0.0
        hist = [0, 0, 0, 0, 0]  # < 1, 1-2, 2-4, 4-8, >= 8 us
        for (_, _, e0), (nm, s1, _) in zip(ks, ks[1:]):
            g = max(0.0, (s1 - e0) / 1e3)
            if g > 1000:  # between steps (host-bound idle), not a launch gap
                continue
            tot += g
            hist[0 if g < 1 else 1 if g < 2 else 2 if g < 4 else 3 if g < 8 else 4] += 1
            nm = nm.replace("(anonymous namespace)::", "").split("(")[0][:90]
            t = by.setdefault(nm, [0, 0.0])
            t[0] += 1
            t[1] += g
        print()
        print(f"inter-kernel gaps (< 1 ms): {tot / 1e3:.2f} ms total" + (f", {tot / 1e3 / a.steps:.3f} ms/step" if a.steps else "")
              + f"; histogram <1/1-2/2-4/4-8/>=8 us: {hist}")
        print()
        print("| next kernel | gaps | total ms | avg us |")
        print("|---|---|---|---|")
        for nm, (n, g) in sorted(by.items(), key=lambda kv: -kv[1][1])[: a.top]:
            print(f"| `{nm}` | {n} | {g / 1e3:.2f} | {g / n:.2f} |")


if __name__ == "__main__":
    main()
