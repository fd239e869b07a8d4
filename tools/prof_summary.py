"""Summarise a rocprofv3 run (rocpd SQLite `*.db` or `*_kernel_stats.csv`) into a markdown table.

    python tools/prof_summary.py gpurun_out/prof_engine2 --top 30 --steps 200 > profiles/x.md
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sqlite3


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*\)$", "", name)
    if name.startswith("Cijk_") or name.startswith("Custom_Cijk"):
        mt = re.search(r"MT\d+x\d+x\d+", name)
        return f"hipBLASLt {name.split('_')[1 if name.startswith('Cijk') else 2]} {mt.group(0) if mt else ''}"
    return name.replace("void ", "")[:110]


def load(path: str):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    if dbs:
        db = sqlite3.connect(dbs[0])
        return [(n, int(c), float(t)) for n, c, t in
                db.execute("select name,total_calls,total_duration from top_kernels")]  # durations in us
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3) for r in csv.DictReader(fh)]
    raise SystemExit(f"no rocprof output under {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many engine steps")
    a = ap.parse_args()
    rows = sorted(load(a.path), key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot / 1e3:.1f} ms over {sum(r[1] for r in rows)} dispatches\n")
    hdr = "| kernel | calls | total ms | avg us | % |" + (" us/step |" if a.steps else "")
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for n, c, t in rows[: a.top]:
        line = f"| `{_short(n)}` | {c} | {t / 1e3:.2f} | {t / max(c, 1):.1f} | {100 * t / tot:.1f} |"
        if a.steps:
            line += f" {t / a.steps:.1f} |"
        print(line)


if __name__ == "__main__":
    main()
