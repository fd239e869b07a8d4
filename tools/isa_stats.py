"""Static ISA census of a hipcc --save-temps .s file: per kernel, the basic block(s) holding the most MFMAs
(the main loop) and their VALU / SALU / LDS / VMEM / wait instruction counts per MFMA.

    python tools/isa_stats.py build/isa/qmm2-hip-amdgcn-amd-amdhsa-gfx950.s [kernel-substring]
"""
import re
import sys
from collections import Counter


def kernels(path):
    cur, lines = None, []
    for ln in open(path):
        m = re.match(r"^([_A-Za-z0-9.$]+):\s*(;.*)?$", ln)
        if m and not ln.startswith(".") and m.group(1).startswith("_Z") and not m.group(1).startswith(".L"):
            if cur:
                yield cur, lines
            cur, lines = m.group(1), []
            continue
        if cur is not None:
            if ln.strip().startswith(".Lfunc_end"):
                yield cur, lines
                cur, lines = None, []
            else:
                lines.append(ln)


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_write", "ds_bpermute", "ds_swizzle", "ds_permute")):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "global_store", "buffer_store", "global_atomic")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith(("s_nop",)):
        return "nop"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def blocks(lines):
    name, body = "entry", []
    for ln in lines:
        s = ln.strip()
        if re.match(r"^\.LBB[0-9_]+:", s):
            yield name, body
            name, body = s.split(":")[0], []
            continue
        if not s or s.startswith((";", ".")):
            continue
        body.append(s.split()[0])
    yield name, body


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for k, lines in kernels(path):
        if pat not in k:
            continue
        bl = [(n, Counter(classify(o) for o in b), Counter(b)) for n, b in blocks(lines)]
        tot = Counter()
        for _, c, _ in bl:
            tot += c
        main_b = max(bl, key=lambda t: t[1]["mfma"])
        n, c, ops = main_b
        mf = max(1, c["mfma"])
        print(f"== {k[:140]}")
        print(f"   kernel total: " + " ".join(f"{t}={tot[t]}" for t in sorted(tot)))
        print(f"   hottest block {n}: " + " ".join(f"{t}={c[t]}" for t in sorted(c)) +
              f" | per MFMA: valu={c['valu'] / mf:.2f} salu={c['salu'] / mf:.2f} lds={c['lds'] / mf:.2f}")
        if "-v" in sys.argv:
            for o, cnt in ops.most_common(40):
                print(f"      {cnt:5d} {o}")


if __name__ == "__main__":
    main()
