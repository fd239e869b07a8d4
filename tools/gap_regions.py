"""Attribute GPU idle gaps of a rocprofv3 kernel+marker trace (rocpd .db) to the host roctx ranges active
during them (MX_ROCTX=1 engine ranges): which engine phase leaves the GPU idle.

    python tools/gap_regions.py gpurun_out/prof_dir [--min-us 300]
"""
import bisect
import collections
import glob
import os
import sqlite3
import sys


def main(path, min_us=300.0):
    db = sqlite3.connect(glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0])
    ks = list(db.execute("select start,end from kernels order by start"))
    ks = ks[int(len(ks) * 0.5):]
    cols = [r[1] for r in db.execute("pragma table_info(regions)")]
    # the roctx message (range label) is in the region's args / extdata JSON, the name is the API call
    lab = next((c for c in ("extdata", "args", "message") if c in cols), "name")
    sample = list(db.execute(f"select name, {lab} from regions where category like '%MARKER%' limit 3"))
    print("regions columns:", cols, "label column:", lab, "sample:", sample)
    raw = list(db.execute(f"select start,end,{lab} from regions where category like '%MARKER%' order by start"))
    import re
    regs = []
    for s, e, t in raw:
        m = re.search(r'(engine\.step|schedule|plan|launch graph|launch eager|process_prev|wait|decode=)', str(t))
        regs.append((s, e, m.group(1) if m else str(t)[:30]))
    gaps, end = [], ks[0][0]
    for s, e in ks:
        if s - end > min_us * 1e3:
            gaps.append((end, s))
        end = max(end, e)
    span = end - ks[0][0]
    tot = sum(b - a for a, b in gaps)
    print(f"gaps >= {min_us:.0f} us: {len(gaps)}, {tot / 1e6:.1f} ms of {span / 1e6:.1f} ms ({100 * tot / span:.1f} %)")
    starts = [r[0] for r in regs]
    acc = collections.Counter()
    for a, b in gaps:
        i = bisect.bisect_right(starts, b)
        for s, e, n in regs[max(0, i - 400):i]:
            ov = min(b, e) - max(a, s)
            if ov > 0:
                acc[n.split(" ")[0]] += ov
    for n, v in acc.most_common(12):
        print(f"  {n:24s} {v / 1e6:8.2f} ms overlapping gaps")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], float(a[a.index("--min-us") + 1]) if "--min-us" in a else 300.0)
