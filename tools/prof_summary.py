#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv, sys
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'total_ms':>9} {'pct':>6} {'calls':>6} {'avg_us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    name = r["Name"]
    if "(" in name:
        name = name[: name.index("(")]
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f} {r['Calls']:>6} {float(r['AverageNs'])/1e3:9.1f}  {name[:100]}")
print(f"total GPU kernel time: {tot/1e6:.1f} ms")
