#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per (kernel, counter) over dispatches -> markdown.

    python tools/pmc_summary.py gpurun_out/pmc_a [gpurun_out/pmc_b ...]
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    acc = collections.defaultdict(list)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = re.sub(r"\(.*\)$", "", r.get("Kernel_Name", "?"))[:90]
                    acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = sorted({k for k, _ in acc})
    for k in kernels:
        print(f"\n### `{k}`\n\n| counter | mean per dispatch | dispatches |\n|---|---|---|")
        for (kk, c), v in sorted(acc.items()):
            if kk == k:
                print(f"| {c} | {sum(v) / len(v):.4g} | {len(v)} |")


if __name__ == "__main__":
    main()
