"""Compressed instruction sequence of a kernel's hottest basic block (MFMA / LDS / waits / VALU runs):
    python tools/isa_seq.py file.s kernel-substring [max-items]"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_stats import kernels  # noqa: E402


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    for name, lines in kernels(path):
        if sub not in name:
            continue
        blocks, cur, label = {}, [], "entry"
        for ln in lines:
            t = ln.strip()
            if t.startswith(".LBB") and t.endswith(":") or (t.startswith(".LBB") and ":" in t):
                blocks[label] = cur
                label, cur = t.split(":")[0], []
                continue
            if t and not t.startswith(";") and not t.startswith("."):
                cur.append(t)
        blocks[label] = cur
        label = max(blocks, key=lambda k: sum(1 for x in blocks[k] if x.startswith("v_mfma")))
        out = []
        for t in blocks[label]:
            op = t.split()[0]
            if op.startswith("v_mfma"):
                out.append("MFMA")
            elif op.startswith("ds_"):
                out.append(op)
            elif op.startswith("s_waitcnt") or op == "s_barrier" or op.startswith("global_load") or op.startswith("buffer_"):
                out.append(t[:40])
            elif op.startswith("v_"):
                out.append("v")
            elif op.startswith("s_"):
                out.append("s")
        res, prev, n = [], None, 0
        for o in out + [None]:
            if o == prev:
                n += 1
                continue
            if prev:
                res.append(f"{prev}x{n}" if n > 1 else prev)
            prev, n = o, 1
        print(name, label)
        print(" | ".join(res[:lim]))
        break


if __name__ == "__main__":
    main()
