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
    ap.add_argument("--split-steps", default="", help="kernel-name substring that starts each engine step: per-step "
                    "tables for steps with / without --mixed-marker kernels")
    ap.add_argument("--mixed-marker", default="attn_prefill", help="kernel-name substring of mixed (prefill) steps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    t_end = c.execute("select max(end) from kernels").fetchone()[0]
    t0 = t_end - a.window_ms * 1e6 if a.window_ms else 0
    rows = c.execute("select name, count(*), sum(end - start) / 1e6, avg(end - start) / 1e3 from kernels "
                     "where start >= ? group by name order by 3 desc", (t0,)).fetchall()
    tot_ms = sum(r[2] for r in rows)
    n = sum(r[1] for r in rows)
    if not a.steps and a.split_steps:  # steps in the window = marker kernels in it
        a.steps = c.execute("select count(*) from kernels where start >= ? and name like ?",
                            (t0, f"%{a.split_steps}%")).fetchone()[0]
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
    if a.split_steps:
        split_steps(c, t0, a.split_steps, a.mixed_marker, a.top)
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


def split_steps(c, t0, marker, mixed_marker, top):
    """Per engine step (a step starts at each `marker` kernel): wall, kernel sum, and the per-kernel split of
    decode-only vs mixed steps."""
    ks = c.execute("select name, start, end from kernels where start >= ? order by start", (t0,)).fetchall()
    steps, cur = [], None
    for nm, s0, e0 in ks:
        if marker in nm:
            if cur is not None:
                steps.append(cur)
            cur = []
        if cur is not None:
            cur.append((nm, s0, e0))
    # the last (possibly partial) step is dropped: its wall is not bounded by a next marker
    out = {}
    for st, nxt in zip(steps, steps[1:] + [None]):
        if nxt is None:
            break
        kind = "mixed" if any(mixed_marker in k[0] for k in st) else "decode"
        d = out.setdefault(kind, {"n": 0, "wall": 0.0, "kern": 0.0, "by": {}})
        d["n"] += 1
        d["wall"] += (nxt[0][1] - st[0][1]) / 1e3
        for nm, s0, e0 in st:
            d["kern"] += (e0 - s0) / 1e3
            nm = nm.replace("(anonymous namespace)::", "").split("(")[0][:90]
            d["by"][nm] = d["by"].get(nm, 0.0) + (e0 - s0) / 1e3
    for kind, d in out.items():
        n = d["n"]
        print()
        print(f"{kind} steps: {n}, wall {d['wall'] / n / 1e3:.3f} ms/step, kernels {d['kern'] / n / 1e3:.3f} ms/step")
        print()
        print("| kernel | us/step |")
        print("|---|---|")
        for nm, us in sorted(d["by"].items(), key=lambda kv: -kv[1])[:top]:
            print(f"| `{nm}` | {us / n:.1f} |")


if __name__ == "__main__":
    main()
