#!/usr/bin/env python3
"""Correlate GPU idle gaps with host HIP API calls (rocprofv3 --kernel-trace --hip-runtime-trace
--marker-trace output). Prints, for the steady tail of the run, the API calls active during each large
gap and an aggregate of API time spent inside gaps -> which host call (sync, copy, launch) the GPU
waited on.

    python tools/dbg/hip_gaps.py gpurun_out/prof_hip [min_gap_us]
"""
import collections
import csv
import glob
import os
import sys


def _rows(path, pat):
    f = glob.glob(os.path.join(path, "**", pat), recursive=True)
    if not f:
        return []
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main(path, min_gap_us=300.0):
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60])
                for r in _rows(path, "*kernel_trace.csv"))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", ""))
                 for r in _rows(path, "*hip_api_trace.csv"))
    marks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"][:50])
                   for r in _rows(path, "*marker_api_trace.csv"))
    ks = ks[int(len(ks) * 0.6):]
    t0 = ks[0][0]
    api = [a for a in api if a[1] >= t0]
    print(f"kernels {len(ks)} api calls {len(api)} markers {len(marks)}")
    tot = collections.Counter()
    cnt = collections.Counter()
    for a in api:
        tot[a[2]] += a[1] - a[0]
        cnt[a[2]] += 1
    print("host API time in steady tail (ms, calls):")
    for f, t in tot.most_common(15):
        print(f"  {f:40s} {t / 1e6:9.2f} {cnt[f]:7d}")
    end = ks[0][1]
    gaps = []
    for s, e, n in ks[1:]:
        if s - end > min_gap_us * 1e3:
            gaps.append((end, s, n))
        end = max(end, e)
    ingap = collections.Counter()
    j = 0
    for g0, g1, _ in gaps:
        for a in api:
            if a[1] < g0 or a[0] > g1:
                continue
            ingap[a[2]] += min(a[1], g1) - max(a[0], g0)
    gt = sum(g1 - g0 for g0, g1, _ in gaps)
    print(f"gaps > {min_gap_us} us: {len(gaps)} total {gt / 1e6:.2f} ms; API time inside them:")
    for f, t in ingap.most_common(12):
        print(f"  {f:40s} {t / 1e6:9.2f} ms")
    # which host marker ranges overlap the gaps (innermost ranges: launch / wait / engine.step)
    inm = collections.Counter()
    for g0, g1, _ in gaps:
        for m in marks:
            if m[1] < g0 or m[0] > g1:
                continue
            inm[m[2].split(" ")[0] + " " + (m[2].split(" ")[1] if m[2].startswith("launch") else "")] += min(m[1], g1) - max(m[0], g0)
    print("marker time inside gaps:")
    for f, t in inm.most_common(10):
        print(f"  {f:40s} {t / 1e6:9.2f} ms")
    for g0, g1, n in gaps[3:9]:
        print(f"--- gap {(g1 - g0) / 1e3:.1f} us before {n}")
        mk = [m for m in marks if m[0] <= g1 and m[1] >= g0 - 20e6]
        for m in mk[-6:]:
            print(f"    marker {(m[0] - g0) / 1e3:9.1f} .. {(m[1] - g0) / 1e3:9.1f}  {m[2]}")
        acts = [a for a in api if a[1] >= g0 and a[0] <= g1]
        acts.sort(key=lambda a: a[0])
        for a in acts[:40]:
            if a[1] - a[0] > 5e3 or a[2] not in ("hipLaunchKernel", "hipExtModuleLaunchKernel", "hipModuleLaunchKernel"):
                print(f"    {(a[0] - g0) / 1e3:9.1f} {(a[1] - a[0]) / 1e3:8.1f} {a[2]} tid={a[3]}")
        print(f"    ({len(acts)} API calls in gap)")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 300.0)
