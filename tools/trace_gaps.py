#!/usr/bin/env python3
"""GPU idle-gap analysis of a rocprofv3 kernel trace: busy fraction, gap histogram, and the largest
gaps (host-side launch / sync bubbles between kernels).

    python tools/trace_gaps.py gpurun_out/prof_dir
"""
import csv
import glob
import os
import sys


def main(path):
    f = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        print("no kernel trace under", path)
        return
    rows = []
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # last 40% of the run (steady state of the bench window)
    rows = rows[int(len(rows) * 0.6):]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    busy = 0
    end = t0
    gaps = []
    for s, e, n in rows:
        if s > end:
            gaps.append((s - end, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = t1 - t0
    print(f"kernels {len(rows)}  span {span/1e6:.2f} ms  busy {busy/span*100:.1f} %  idle {(span-busy)/1e6:.2f} ms")
    hist = {}
    for g, _ in gaps:
        b = "<5us" if g < 5e3 else "<20us" if g < 2e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
        hist.setdefault(b, [0, 0])
        hist[b][0] += 1
        hist[b][1] += g
    for b in ("<5us", "<20us", "<100us", "<1ms", ">=1ms"):
        if b in hist:
            print(f"  gaps {b:7s} n={hist[b][0]:6d} total {hist[b][1]/1e6:.2f} ms")
    for g, n in sorted(gaps, reverse=True)[:10]:
        print(f"  gap {g/1e3:8.1f} us before {n[:60]}")
    # steady-tail kernel breakdown per engine step (one argmax launch per step)
    steps = sum(1 for _, _, n in rows if n.startswith("argmax_kernel")) or 1
    agg = {}
    for s, e, n in rows:
        k = _short(n)
        a = agg.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += e - s
    tot = sum(v[1] for v in agg.values())
    print(f"\nsteady tail: {steps} steps, GPU busy {tot / steps / 1e3:.1f} us/step")
    print("| kernel | calls/step | us/step | % |\n|---|---:|---:|---:|")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"| {k} | {c / steps:.1f} | {t / steps / 1e3:.1f} | {100 * t / tot:.1f} |")


def _short(name):
    import re
    name = re.sub(r"\(.*$", "", name)
    if name.startswith("Cijk_"):
        mt = re.search(r"MT\d+x\d+x\d+", name)
        return "hipBLASLt " + (mt.group(0) if mt else "")
    return name.replace("void ", "")[:70]


if __name__ == "__main__":
    main(sys.argv[1])
